#!/bin/bash
# GraphStep on the GPU: numerics tests, then BERT-base eager vs HIP-graph-captured step.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_graph_step.py \
    > gpurun_out/graph_tests.log 2>&1 || { tail -40 gpurun_out/graph_tests.log; exit 1; }
tail -3 gpurun_out/graph_tests.log
timeout -k 10 300 python tools/bench_bert.py --steps 20 --warmup 5 > gpurun_out/bert_eager.log 2>&1 \
    || { tail -30 gpurun_out/bert_eager.log; exit 1; }
tail -1 gpurun_out/bert_eager.log
timeout -k 10 300 python tools/bench_bert.py --steps 20 --warmup 5 --graph > gpurun_out/bert_graph.log 2>&1 \
    || { tail -30 gpurun_out/bert_graph.log; exit 1; }
tail -1 gpurun_out/bert_graph.log
