#!/bin/bash
# dilated convs on the big-tile / wgrad kernels: tests + conv_gen / dilated bench vs MIOpen
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_dilated.py tests/test_hip_kernels.py -k "dilat or conv_big" > gpurun_out/r6p_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r6p_tests.log; exit 1; }
tail -1 gpurun_out/r6p_tests.log
timeout -k 10 400 python -u tools/bench_conv_gen.py > gpurun_out/r6p_conv_gen.txt 2>&1 || { echo CONVGEN FAILED; tail -20 gpurun_out/r6p_conv_gen.txt; exit 1; }
cat gpurun_out/r6p_conv_gen.txt
