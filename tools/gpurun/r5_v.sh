# round 5: non-temporal policy of the BN apply kernels (MXAMD_BN_NT): probe + bench A/B
set -o pipefail
TAG=${1:-r5v}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PYTHONPATH=$PWD
for nt in 0 1 2; do
  echo "== nt $nt"
  for shp in "256 56 56 256" "256 28 28 512" "256 14 14 1024"; do
    MXAMD_BN_NT=$nt timeout -k 10 120 python tools/bn_apply_probe.py --shape $shp || exit $?
  done
done
for nt in 0 1 2; do
  MXAMD_BN_NT=$nt timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_nt$nt.log 2>&1 || exit $?
  echo "nt=$nt $(tail -1 gpurun_out/${TAG}_bench_nt$nt.log | grep -o '"value": [0-9.]*')"
done
