# round-4 GPU run: stem kernel tests, BN-fusion test, bench (+ loss trace), rocprof kernel trace
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <log> <timeout> cmd...: stop the whole run after a fault / abort / time limit
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "step $log rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
PYT="python -u -m pytest -v --timeout 600 --timeout-method thread -p no:cacheprovider"
step r4d_stem_tests.log 300 $PYT tests/test_conv_stem.py
step r4d_fuse_test.log 300 $PYT tests/test_resnet_gpu.py::test_resnet_bn_backward_fusion_matches_unfused
step r4d_dist_tests.log 300 $PYT tests/test_distributed_gpu.py
MXAMD_BENCH_VERBOSE=1 step r4d_bench.log 400 python -u bench.py --steps 30 --warmup 10
step r4d_prof.log 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4d_prof -o run -- python3 bench.py --steps 6 --warmup 10
python tools/trace_window.py gpurun_out/r4d_prof --steps 5 > gpurun_out/r4d_prof_window.txt 2>&1
python tools/prof_summary.py gpurun_out/r4d_prof 16 > gpurun_out/r4d_prof_summary.txt 2>&1
