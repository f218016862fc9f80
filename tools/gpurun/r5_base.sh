# round 5: GPU tests + the driver's bench command + a steady-state rocprof window.
# usage: bash tools/gpurun/r5_base.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-r5a}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench2.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench2.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -- \
  python bench.py --steps 8 --warmup 6 > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
python tools/trace_window.py gpurun_out/${TAG}_prof --steps 5 --top 60 > gpurun_out/${TAG}_window.txt
head -12 gpurun_out/${TAG}_window.txt
