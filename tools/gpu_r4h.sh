# round-4: deform numerics diagnosis, BN kernel tests after the streaming-unroll change, bench, steady-state profile
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
step() {
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "step $log rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
step r4h_deform_diag.log 200 python -u tools/deform_diag.py
step r4h_bn_tests.log 400 $PYT tests/test_hip_kernels.py -k "bn or batchnorm"
step r4h_resnet_tests.log 400 $PYT tests/test_resnet_gpu.py
step r4h_bench.log 400 python -u bench.py --steps 30 --warmup 10
step r4h_prof.log 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4h_prof -o run -- python3 bench.py --steps 6 --warmup 10
python tools/trace_window.py gpurun_out/r4h_prof --steps 5 > gpurun_out/r4h_prof_window.txt 2>&1
echo done
