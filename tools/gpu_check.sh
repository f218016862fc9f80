set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 env MXAMD_BENCH_VERBOSE=1 python -u bench.py --steps 20 --warmup 10 > gpurun_out/bench.log 2>&1
