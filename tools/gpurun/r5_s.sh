# round 5: kernel-time A/B of the BN reduction grid size (MXAMD_BN_BLOCKS) under rocprofv3
set -o pipefail
TAG=${1:-r5s}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for b in 512 1024; do
  export MXAMD_BN_BLOCKS=$b
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof$b -- \
    python bench.py --steps 8 --warmup 6 > gpurun_out/${TAG}_prof$b.log 2>&1 || exit $?
  python tools/trace_window.py gpurun_out/${TAG}_prof$b --steps 5 --top 80 > gpurun_out/${TAG}_window$b.txt || exit $?
  echo "== blocks $b"; sed -n 1,4p gpurun_out/${TAG}_window$b.txt | cut -c1-100
  grep -E "bn_reduce|bn_tail" gpurun_out/${TAG}_window$b.txt | cut -c1-90
done
