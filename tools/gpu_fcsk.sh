set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/bench_fc_splitk.py > gpurun_out/fc_splitk.log 2>&1; cat gpurun_out/fc_splitk.log | tail -8
