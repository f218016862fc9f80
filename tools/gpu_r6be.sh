#!/bin/bash
# same-box A/B: conv_big with / without the static s_setprio(1) for waves 4-7 (two prebuilt libraries)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
SO=$(ls mxnet_maintenance_amd/_lib/_hip_kernels*.so)
for i in 1 2 3; do
for v in noprio prio; do
cp abtmp/$v.so "$SO"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6be_${v}_$i.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/r6be_${v}_$i.log; exit 1; }
echo "$v run $i: $(tail -1 gpurun_out/r6be_${v}_$i.log | cut -c88-135)"
done
done
cp abtmp/prio.so "$SO"
