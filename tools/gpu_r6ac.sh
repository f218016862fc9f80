#!/bin/bash
# GEMM microbench with the whole-wave 192 / 384-column tiles (gemm.hip cfgs 14-17) vs hipBLASLt
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 120 python -u -m pytest -x -q --timeout 60 --timeout-method thread tests/test_gemm.py > gpurun_out/r6ac_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r6ac_tests.log; exit 1; }
tail -3 gpurun_out/r6ac_tests.log
timeout -k 10 400 python -u tools/bench_gemm.py --iters 30 > gpurun_out/r6ac_gemm.log 2>&1 || { echo BENCH FAILED; tail -30 gpurun_out/r6ac_gemm.log; exit 1; }
cat gpurun_out/r6ac_gemm.log
