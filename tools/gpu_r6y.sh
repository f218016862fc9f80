#!/bin/bash
# stem forward with three workgroups per CU: tests + timing
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_stem.py > gpurun_out/r6y_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r6y_tests.log; exit 1; }
tail -1 gpurun_out/r6y_tests.log
timeout -k 10 120 python3 -u tools/stem_probe.py > gpurun_out/r6y_stem.log 2>&1 || { echo STEM FAILED; tail -20 gpurun_out/r6y_stem.log; exit 1; }
cat gpurun_out/r6y_stem.log
