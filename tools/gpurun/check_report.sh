# GPU tests, 1-GPU bench, steady-state rocprofv3 window and the per-shape autotune/roofline report.
# usage: bash tools/gpurun/check_report.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-run}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/${TAG}_gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${TAG}_gpu_tests.log; grep -E "^FAILED" gpurun_out/${TAG}_gpu_tests.log | head -20
  [ $rc -le 1 ] || exit $rc
fi
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 && tail -1 gpurun_out/${TAG}_bench.log && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -- python bench.py --steps 8 --warmup 6 > gpurun_out/${TAG}_prof.log 2>&1 && \
python tools/trace_window.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_window.txt && head -12 gpurun_out/${TAG}_window.txt && \
timeout -k 10 300 python -u tools/autotune_report.py > gpurun_out/${TAG}_autotune.log 2>&1 && tail -3 gpurun_out/${TAG}_autotune.log
