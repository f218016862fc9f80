#!/bin/bash
# channels-last deformable conv (fused backward): tests, SSD-512 bench + window
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_deform_conv.py tests/test_conv_kpad.py > gpurun_out/r6o_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r6o_tests.log; exit 1; }
tail -1 gpurun_out/r6o_tests.log
MXAMD_BENCH_VERBOSE=1 timeout -k 10 400 python -u tools/bench_ssd.py --steps 20 --warmup 5 > gpurun_out/r6o_ssd.log 2>&1 || { echo SSD FAILED; tail -20 gpurun_out/r6o_ssd.log; exit 1; }
grep -v conv-algo gpurun_out/r6o_ssd.log | tail -1 | cut -c1-160
grep conv-algo gpurun_out/r6o_ssd.log > gpurun_out/r6o_ssd_choices.txt || true
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6o_prof -o trace -- python3 -u tools/bench_ssd.py --steps 8 --warmup 4 > gpurun_out/r6o_prof.log 2>&1 || { echo PROF FAILED; tail -5 gpurun_out/r6o_prof.log; exit 1; }
python tools/trace_window.py gpurun_out/r6o_prof --steps 4 --top 60 > gpurun_out/r6o_window.txt 2>&1; head -12 gpurun_out/r6o_window.txt | cut -c1-160
grep -i deform gpurun_out/r6o_window.txt | cut -c1-140
rm -rf gpurun_out/r6o_prof
timeout -k 10 300 python -u tools/bench_conv_gen.py > gpurun_out/r6o_conv_gen.txt 2>&1 || { echo CONVGEN FAILED; tail -20 gpurun_out/r6o_conv_gen.txt; exit 1; }
cat gpurun_out/r6o_conv_gen.txt
