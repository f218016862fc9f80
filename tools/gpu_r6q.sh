#!/bin/bash
# dilated convs (tests + bench vs MIOpen); fused residual-dropout-LayerNorm (tests + BERT-base bench + window)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_dilated.py tests/test_add_dropout_ln.py tests/test_models.py > gpurun_out/r6q_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r6q_tests.log; exit 1; }
tail -1 gpurun_out/r6q_tests.log
timeout -k 10 400 python -u tools/bench_conv_gen.py > gpurun_out/r6q_conv_gen.txt 2>&1 || { echo CONVGEN FAILED; tail -20 gpurun_out/r6q_conv_gen.txt; exit 1; }
grep deeplab gpurun_out/r6q_conv_gen.txt; tail -1 gpurun_out/r6q_conv_gen.txt
timeout -k 10 400 python -u tools/bench_bert.py --graph --gemm-table none --steps 20 --warmup 5 > gpurun_out/r6q_bert.log 2>&1 || { echo BERT FAILED; tail -20 gpurun_out/r6q_bert.log; exit 1; }
tail -1 gpurun_out/r6q_bert.log | cut -c1-250
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6q_prof -o trace -- python3 -u tools/bench_bert.py --graph --gemm-table none --steps 8 --warmup 4 > gpurun_out/r6q_prof.log 2>&1 || { echo PROF FAILED; tail -5 gpurun_out/r6q_prof.log; exit 1; }
python tools/trace_window.py gpurun_out/r6q_prof --steps 5 --top 45 > gpurun_out/r6q_window.txt 2>&1; head -40 gpurun_out/r6q_window.txt | cut -c1-170
rm -rf gpurun_out/r6q_prof
