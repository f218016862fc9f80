# round-4 GPU run: bench, copy/compute overlap trace, full GPU test suite (dist/fused/deform/dw incl.)
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
step() {
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$GRAFT_REPO_ROOT/gpurun_out/$log" 2>&1
  local rc=$?
  echo "step $log rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
step r4e_bench.log 300 python -u bench.py --steps 30 --warmup 10
cd /tmp
step r4e_overlap.log 150 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4e_overlap -o run -- python3 $GRAFT_REPO_ROOT/tools/overlap_probe.py
cd $GRAFT_REPO_ROOT
python tools/overlap_report.py gpurun_out/r4e_overlap > gpurun_out/r4e_overlap_report.txt 2>&1
step r4e_gpu_all.log 680 $PYT -m gpu tests
