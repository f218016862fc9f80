# round 5: A/B of the BN reduction grid size (MXAMD_BN_BLOCKS) and the tail shortcut-stats fusion
set -o pipefail
TAG=${1:-r5r}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for cfg in "512 1" "512 0" "1024 1" "2048 1" "2048 0"; do
  set -- $cfg
  MXAMD_BN_BLOCKS=$1 MXAMD_BN_TAIL_DS=$2 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 \
    > gpurun_out/${TAG}_bench_b$1_ds$2.log 2>&1 || exit $?
  echo "blocks=$1 tail_ds=$2 $(tail -1 gpurun_out/${TAG}_bench_b$1_ds$2.log | grep -o "\"value\": [0-9.]*")"
done
