#!/bin/bash
# same-box A/B of the autotuner's vendor margin on ResNet-50 (0, 0.03 default, 0.06), twice each
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for i in 1 2; do
for m in 0.03 0.0 0.06; do
MXAMD_VENDOR_MARGIN=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6bc_m${m}_$i.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/r6bc_m${m}_$i.log; exit 1; }
echo "margin $m run $i: $(tail -1 gpurun_out/r6bc_m${m}_$i.log | cut -c88-130)"
done
done
