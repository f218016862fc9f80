set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/bench_fc_splitk_fwd.py > gpurun_out/fc_splitk_fwd.log 2>&1; tail -12 gpurun_out/fc_splitk_fwd.log
