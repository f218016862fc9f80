# GPU tests (optionally a subset) + 1-GPU bench + rocprofv3 stats.  usage: bash tools/gpurun/tests_bench.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-run}
K=${2:-}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -n "$K" ]; then KARG="-k $K"; else KARG=""; fi
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/ $KARG > gpurun_out/${TAG}_gpu_tests.log 2>&1; tail -5 gpurun_out/${TAG}_gpu_tests.log; grep -E "^FAILED" gpurun_out/${TAG}_gpu_tests.log | head -20
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 && tail -1 gpurun_out/${TAG}_bench.log && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -- python bench.py --steps 8 --warmup 6 > gpurun_out/${TAG}_prof.log 2>&1 && \
python tools/trace_window.py gpurun_out/${TAG}_prof --steps 6 --top 45 > gpurun_out/${TAG}_prof_window.txt && head -12 gpurun_out/${TAG}_prof_window.txt
