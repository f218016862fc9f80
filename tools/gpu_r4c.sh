# round-4 combined GPU run: stem kernel tests, determinism / graph-vs-eager tests, bench, rocprof
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
PYT="python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider"
step r4c_stem_tests.log 300 $PYT tests/test_conv_stem.py
step r4c_det_tests.log 900 $PYT tests/test_resnet_gpu.py tests/test_engine_device.py tests/test_hip_kernels.py::test_lamb_arena_kernel_matches_per_segment_reference
step r4c_bench.log 400 python -u bench.py --steps 30 --warmup 10
step r4c_prof.log 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r4c_prof -o run -- python3 bench.py --steps 6 --warmup 10
python tools/prof_summary.py gpurun_out/r4c_prof 16 > gpurun_out/r4c_prof_summary.txt 2>&1
