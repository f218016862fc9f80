#!/bin/bash
# clean-built extensions: smoke, a kernel-test subset, headline bench
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6ba_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/r6ba_smoke.log; exit 1; }
tail -1 gpurun_out/r6ba_smoke.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_pw.py tests/test_bn_relu_maxpool.py tests/test_gemm.py tests/test_hip_kernels.py tests/test_resnet_gpu.py > gpurun_out/r6ba_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r6ba_tests.log; exit 1; }
tail -1 gpurun_out/r6ba_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/r6ba_bench.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/r6ba_bench.log; exit 1; }
tail -1 gpurun_out/r6ba_bench.log | cut -c1-200
