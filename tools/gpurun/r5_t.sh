# round 5: kernel-time A/B of the residual-tail shortcut-statistics grid (MXAMD_BN_TAIL_BLOCKS)
set -o pipefail
TAG=${1:-r5t}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_bn_shortcut_stats.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for b in 1024 2048 4096; do
  export MXAMD_BN_TAIL_BLOCKS=$b
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof$b -- \
    python bench.py --steps 8 --warmup 6 > gpurun_out/${TAG}_prof$b.log 2>&1 || exit $?
  python tools/trace_window.py gpurun_out/${TAG}_prof$b --steps 5 --top 80 > gpurun_out/${TAG}_window$b.txt || exit $?
  echo "== tail blocks $b"; sed -n 1,4p gpurun_out/${TAG}_window$b.txt | cut -c1-100
  grep -E "bn_reduce|bn_tail" gpurun_out/${TAG}_window$b.txt | cut -c1-90
done
