set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q --timeout 120 --timeout-method thread -k "conv or bottleneck or resnet or autotune" > gpurun_out/conv_tests.log 2>&1 && \
timeout -k 10 400 env MXAMD_BENCH_VERBOSE=1 python -u bench.py --steps 20 --warmup 10 > gpurun_out/bench.log 2>&1
