#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ssd.py tests/test_deform_conv.py > gpurun_out/r6l_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r6l_tests.log; exit 1; }
tail -1 gpurun_out/r6l_tests.log
timeout -k 10 400 python -u tools/bench_ssd.py --steps 20 --warmup 5 > gpurun_out/r6l_ssd.log 2>&1; tail -1 gpurun_out/r6l_ssd.log | cut -c1-200
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6l_prof -o trace -- python3 -u tools/bench_ssd.py --steps 8 --warmup 4 > gpurun_out/r6l_prof.log 2>&1 || { echo PROF FAILED; tail -5 gpurun_out/r6l_prof.log; exit 1; }
python tools/trace_window.py gpurun_out/r6l_prof --steps 4 --top 45 > gpurun_out/r6l_window.txt 2>&1; head -55 gpurun_out/r6l_window.txt
rm -rf gpurun_out/r6l_prof
