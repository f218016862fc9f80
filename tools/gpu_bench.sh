#!/bin/bash
# bench + steady-state rocprof window: bash tools/gpu_bench.sh <tag> [extra bench args]
set -o pipefail
cd "$(dirname "$0")/.."
tag=${1:-r6}
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 "$@" > gpurun_out/${tag}_bench.log 2>&1 || { echo BENCH FAILED; tail -30 gpurun_out/${tag}_bench.log; exit 1; }
tail -2 gpurun_out/${tag}_bench.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o trace -- python3 -u bench.py --steps 10 --warmup 4 "$@" > gpurun_out/${tag}_prof.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/${tag}_prof.log; exit 1; }
python tools/trace_window.py gpurun_out/${tag}_prof --steps 5 --top 60 > gpurun_out/${tag}_window.txt 2>&1
head -75 gpurun_out/${tag}_window.txt
rm -rf gpurun_out/${tag}_prof
