set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/debug_graph_vs_eager.py resnet18_v1 5 > gpurun_out/graphdbg_r18.log 2>&1; rc=$?; grep -E "loss|worst|<<" gpurun_out/graphdbg_r18.log | head -40
exit $rc
