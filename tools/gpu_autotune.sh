set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/autotune_report.py > gpurun_out/autotune_report.log 2>&1; tail -5 gpurun_out/autotune_report.log
