set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench_1gpu.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_bert.py > gpurun_out/bench_bert.log 2>&1
