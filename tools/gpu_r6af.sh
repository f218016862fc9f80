#!/bin/bash
# ResNet-50 copy sources; hipBLASLt kernel per BERT FC GEMM
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/copy_sources_probe.py resnet > gpurun_out/r6af_copies.log 2>&1 || { echo PROBE FAILED; tail -30 gpurun_out/r6af_copies.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6af_copies.log | tail -40
timeout -k 10 200 python -u tools/mm_kernel_names.py > gpurun_out/r6af_mm.log 2>&1 || { echo MM FAILED; tail -30 gpurun_out/r6af_mm.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6af_mm.log
