#!/bin/bash
# gemm.hip with all fragments of a K-step read ahead of the MFMAs: tests + BERT-shape microbench
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm.py > gpurun_out/r6w_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r6w_tests.log; exit 1; }
tail -1 gpurun_out/r6w_tests.log
timeout -k 10 600 python -u tools/bench_gemm.py --iters 30 > gpurun_out/r6w_gemm.log 2>&1 || { echo GEMM FAILED; tail -20 gpurun_out/r6w_gemm.log; exit 1; }
grep -E "^(fwd|dgrad|wgrad|total)|gemm\((1|2|6|12|13), " gpurun_out/r6w_gemm.log | head -70
