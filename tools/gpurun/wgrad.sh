set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_kernels.py -k "wgrad" > gpurun_out/wgrad_tests.log 2>&1; rc=$?; tail -5 gpurun_out/wgrad_tests.log; [ $rc -eq 0 ] && \
timeout -k 10 400 python -u tools/bench_wgrad.py > gpurun_out/wgrad_bench.log 2>&1; tail -30 gpurun_out/wgrad_bench.log
