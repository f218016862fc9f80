# Round-end style check on one MI355X: GPU tests, smoke, 1-GPU bench, rocprofv3 kernel stats.
# usage: gpurun --timeout 1200 -- bash tools/gpurun/full_check.sh TAG
set -o pipefail
TAG=${1:-run}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/${TAG}_gpu_tests.log 2>&1; tail -3 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 && tail -1 gpurun_out/${TAG}_smoke.log && \
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 && tail -1 gpurun_out/${TAG}_bench.log && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -- python bench.py --steps 8 --warmup 6 > gpurun_out/${TAG}_prof.log 2>&1 && \
python tools/prof_summary.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_prof_summary.txt && head -12 gpurun_out/${TAG}_prof_summary.txt
