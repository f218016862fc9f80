#!/bin/bash
# same-box A/B: BERT-base with / without the residual-gradient handoff + fused bias partials (x2 each)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
for h in 1 0; do
MXAMD_RESIDUAL_HANDOFF=$h timeout -k 10 300 python -u tools/bench_bert.py --graph --gemm-table none --steps 30 --warmup 5 > gpurun_out/r6u_bert_h${h}_$i.log 2>&1 || { echo BERT FAILED; tail -20 gpurun_out/r6u_bert_h${h}_$i.log; exit 1; }
echo "handoff=$h run $i: $(tail -1 gpurun_out/r6u_bert_h${h}_$i.log | cut -c1-110)"
done
done
