#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_up2.py tests/test_hip_kernels.py -k "up2 or conv_big" > gpurun_out/r6k_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r6k_tests.log; exit 1; }
tail -1 gpurun_out/r6k_tests.log
MXAMD_BENCH_VERBOSE=1 bash tools/gpu_bench.sh r6k && grep conv-algo gpurun_out/r6k_bench.log > gpurun_out/r6k_conv_choices.txt; grep -E "up[0-9]|miopen" gpurun_out/r6k_conv_choices.txt | cut -c1-220
