#!/bin/bash
# bias gradients written in the bias dtype: affected tests + SSD / BERT benches
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm.py tests/test_gelu_bias_partials.py tests/test_add_dropout_ln.py tests/test_ssd.py tests/test_conv_kpad.py tests/test_deform_conv.py tests/test_models.py > gpurun_out/r6as_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r6as_tests.log; exit 1; }
tail -1 gpurun_out/r6as_tests.log
timeout -k 10 400 python -u tools/bench_ssd.py --steps 20 --warmup 5 > gpurun_out/r6as_ssd.log 2>&1 || { echo SSD FAILED; tail -20 gpurun_out/r6as_ssd.log; exit 1; }
tail -1 gpurun_out/r6as_ssd.log | cut -c1-200
timeout -k 10 300 python -u tools/bench_bert.py --graph --gemm-table none --steps 20 --warmup 5 > gpurun_out/r6as_bert.log 2>&1 || { echo BERT FAILED; tail -20 gpurun_out/r6as_bert.log; exit 1; }
tail -1 gpurun_out/r6as_bert.log | cut -c1-200
