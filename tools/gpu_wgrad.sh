set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -v --timeout 120 --timeout-method thread -k "wgrad or bn" > gpurun_out/wgrad_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_wgrad.py > gpurun_out/bench_wgrad.log 2>&1 && \
timeout -k 10 300 env MXAMD_BENCH_VERBOSE=1 python -u bench.py --steps 20 --warmup 10 > gpurun_out/bench.log 2>&1
