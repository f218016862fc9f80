# round 5: A/B of the shortcut-BN statistics in the residual-tail backward (MXAMD_BN_TAIL_DS 0 vs 1)
set -o pipefail
TAG=${1:-r5w}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for run in a0 b1 c0 d1; do
  nt=${run:1:1}
  MXAMD_BN_TAIL_DS=$nt timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_$run.log 2>&1 || exit $?
  echo "tail_ds=$nt $(tail -1 gpurun_out/${TAG}_bench_$run.log | grep -o '"value": [0-9.]*')"
done
