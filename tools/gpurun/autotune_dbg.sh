set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u tools/debug_autotune_grads.py resnet18_v1 > gpurun_out/atdbg_r18.log 2>&1; rc=$?; head -80 gpurun_out/atdbg_r18.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/debug_autotune_grads.py resnet18_v1 --nofuse > gpurun_out/atdbg_r18_nofuse.log 2>&1; head -5 gpurun_out/atdbg_r18_nofuse.log
