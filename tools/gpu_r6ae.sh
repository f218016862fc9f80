#!/bin/bash
# BERT-base: GEMM bias read in the operand dtype; GELU backward emits the FFN-1 bias partials; choices + window
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/gelu_colpart_probe.py > gpurun_out/r6ae_gelu_probe.log 2>&1 && cat gpurun_out/r6ae_gelu_probe.log && timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm.py tests/test_gelu_bias_partials.py tests/test_add_dropout_ln.py tests/test_models.py > gpurun_out/r6ae_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r6ae_tests.log; exit 1; }
tail -1 gpurun_out/r6ae_tests.log
MXAMD_BENCH_VERBOSE=1 timeout -k 10 400 python -u tools/bench_bert.py --graph --gemm-table none --steps 20 --warmup 5 > gpurun_out/r6ae_bert.log 2>&1 || { echo BERT FAILED; tail -20 gpurun_out/r6ae_bert.log; exit 1; }
grep -v "algo" gpurun_out/r6ae_bert.log | tail -1 | cut -c1-200
grep "algo" gpurun_out/r6ae_bert.log | cut -c1-230 > gpurun_out/r6ae_bert_choices.txt || true
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6ae_prof -o trace -- python3 -u tools/bench_bert.py --graph --gemm-table none --steps 8 --warmup 4 > gpurun_out/r6ae_prof.log 2>&1 || { echo PROF FAILED; tail -5 gpurun_out/r6ae_prof.log; exit 1; }
python tools/trace_window.py gpurun_out/r6ae_prof --steps 5 --top 45 > gpurun_out/r6ae_window.txt 2>&1; head -30 gpurun_out/r6ae_window.txt | cut -c1-170
rm -rf gpurun_out/r6ae_prof
