#!/bin/bash
# SSD-512 copy sources on the current tree
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/copy_sources_probe.py ssd > gpurun_out/r6ar_copies.log 2>&1 || { echo PROBE FAILED; tail -30 gpurun_out/r6ar_copies.log; exit 1; }
grep -v "amdgpu.ids\|Warning\|warn" gpurun_out/r6ar_copies.log | tail -45
