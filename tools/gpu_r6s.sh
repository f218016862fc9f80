#!/bin/bash
# GEMM microbench on the BERT-base shapes: hipBLASLt vs every in-tree candidate
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/autotune_timing_probe.py > gpurun_out/r6s_probe.log 2>&1 || { echo PROBE FAILED; tail -20 gpurun_out/r6s_probe.log; exit 1; }
cat gpurun_out/r6s_probe.log
