#!/bin/bash
# round 6h: halo-tile 3x3 conv -- tests, then per-shape timing
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_halo.py > gpurun_out/r6h_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r6h_tests.log; exit 1; }
tail -2 gpurun_out/r6h_tests.log
timeout -k 10 500 python -u tools/bench_conv_variants.py --rounds 2 --stats > gpurun_out/r6h_conv_variants.txt 2>&1
rc=$?
head -5 gpurun_out/r6h_conv_variants.txt; tail -1 gpurun_out/r6h_conv_variants.txt
exit $rc
