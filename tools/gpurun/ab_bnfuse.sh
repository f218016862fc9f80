# A/B: BN-backward statistics fused into dgrad epilogues vs separate reduce, 1-GPU ResNet-50 bench;
# then GraphStep-vs-eager debug on resnet50_v1b.  usage: bash tools/gpurun/ab_bnfuse.sh TAG
set -o pipefail
TAG=${1:-ab}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_fuse1.log 2>&1 && tail -1 gpurun_out/${TAG}_fuse1.log && \
MXAMD_BN_BWD_FUSE=0 timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_fuse0.log 2>&1 && tail -1 gpurun_out/${TAG}_fuse0.log && \
timeout -k 10 300 python -u tools/debug_graph_vs_eager.py resnet50_v1b 5 > gpurun_out/${TAG}_graphdbg.log 2>&1; rc=$?; grep -E "loss|worst|<<" gpurun_out/${TAG}_graphdbg.log | head -30
exit $rc
