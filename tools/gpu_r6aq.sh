#!/bin/bash
# eager (graph off: the N>1 code path) ResNet-50 on one GPU, final tree
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --graph off > gpurun_out/r6aq_bench_eager.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/r6aq_bench_eager.log; exit 1; }
tail -1 gpurun_out/r6aq_bench_eager.log | cut -c1-220
