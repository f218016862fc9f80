#!/bin/bash
# round 6a: 32x32x16 conv_big variants -- correctness + per-shape timing vs the 16x16x32 tiles
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py -k "conv_big_bn_stats" > gpurun_out/r6a_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r6a_tests.log; exit 1; }
tail -3 gpurun_out/r6a_tests.log
timeout -k 10 500 python -u tools/bench_conv_variants.py --rounds 2 > gpurun_out/r6a_conv_variants.txt 2>&1
rc=$?
tail -50 gpurun_out/r6a_conv_variants.txt
exit $rc
