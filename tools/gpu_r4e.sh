# round-4: graph-captured RCCL bucket all-reduce test, fused fwd/bwd kernels, full GPU suite, bench
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "step $log rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
step r4e_dist_tests.log 300 $PYT tests/test_distributed_gpu.py
step r4e_fused.log 300 $PYT -m gpu tests/test_graph_passes.py
step r4e_gpu_all.log 900 $PYT -m gpu tests
step r4e_bench.log 400 python -u bench.py --steps 30 --warmup 10
