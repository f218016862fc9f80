# round 5: A/B of the tail dz non-temporal store (MXAMD_BN_NT 1 vs 3), tests, window
set -o pipefail
TAG=${1:-r5w}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_bn_shortcut_stats.py tests/test_resnet_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
for run in a1 b3 c1 d3; do
  nt=${run:1:1}
  MXAMD_BN_NT=$nt timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_$run.log 2>&1 || exit $?
  echo "nt=$nt $(tail -1 gpurun_out/${TAG}_bench_$run.log | grep -o '"value": [0-9.]*')"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -- \
  python bench.py --steps 8 --warmup 6 > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
python tools/trace_window.py gpurun_out/${TAG}_prof --steps 5 --top 60 > gpurun_out/${TAG}_window.txt
head -12 gpurun_out/${TAG}_window.txt | cut -c1-160
grep -E "bn_" gpurun_out/${TAG}_window.txt | cut -c1-100
