#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/copy_sources_probe.py > gpurun_out/r6ab_copies.log 2>&1 || { echo PROBE FAILED; tail -30 gpurun_out/r6ab_copies.log; exit 1; }
tail -46 gpurun_out/r6ab_copies.log
