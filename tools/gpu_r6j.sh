#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_halo.py > gpurun_out/r6j_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r6j_tests.log; exit 1; }
tail -1 gpurun_out/r6j_tests.log
MXAMD_BENCH_VERBOSE=1 bash tools/gpu_bench.sh r6j && grep conv-algo gpurun_out/r6j_bench.log > gpurun_out/r6j_conv_choices.txt; grep -c conv-algo gpurun_out/r6j_conv_choices.txt
