#!/bin/bash
# one tiled-transpose helper for every weight transpose (tee / up2 dgrads, FC / RNN / deformable GEMMs):
# affected tests + ResNet-50, BERT-base and SSD-512 benches
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_rnn_kernels.py tests/test_deform_conv.py tests/test_gemm.py tests/test_gelu_bias_partials.py tests/test_conv_pw.py tests/test_resnet_gpu.py tests/test_conv_strided_dgrad.py > gpurun_out/r6ag_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r6ag_tests.log; exit 1; }
tail -1 gpurun_out/r6ag_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6ag_bench.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/r6ag_bench.log; exit 1; }
tail -1 gpurun_out/r6ag_bench.log | cut -c1-200
timeout -k 10 300 python -u tools/bench_bert.py --graph --gemm-table none --steps 20 --warmup 5 > gpurun_out/r6ag_bert.log 2>&1 || { echo BERT FAILED; tail -20 gpurun_out/r6ag_bert.log; exit 1; }
tail -1 gpurun_out/r6ag_bert.log | cut -c1-200
timeout -k 10 400 python -u tools/bench_ssd.py --steps 20 --warmup 5 > gpurun_out/r6ag_ssd.log 2>&1 || { echo SSD FAILED; tail -20 gpurun_out/r6ag_ssd.log; exit 1; }
tail -1 gpurun_out/r6ag_ssd.log | cut -c1-200
