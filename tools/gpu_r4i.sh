# round-4: full GPU suite on the current tree, smoke, bench
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
step r4i_gpu_all.log 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step r4i_smoke.log 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step r4i_bench.log 400 python -u bench.py --steps 30 --warmup 10
echo done
