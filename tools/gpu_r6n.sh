#!/bin/bash
# SSD-512: output-channel-padded head / offset convs on the in-tree kernels (A/B vs MIOpen), choices, window
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_kpad.py tests/test_deform_conv.py > gpurun_out/r6n_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r6n_tests.log; exit 1; }
tail -1 gpurun_out/r6n_tests.log
MXAMD_BENCH_VERBOSE=1 timeout -k 10 400 python -u tools/bench_ssd.py --steps 20 --warmup 5 > gpurun_out/r6n_ssd_kpad.log 2>&1 || { echo SSD FAILED; tail -20 gpurun_out/r6n_ssd_kpad.log; exit 1; }
grep -v conv-algo gpurun_out/r6n_ssd_kpad.log | tail -1 | cut -c1-160
grep conv-algo gpurun_out/r6n_ssd_kpad.log > gpurun_out/r6n_ssd_choices.txt || true
MXAMD_CONV_KPAD=0 timeout -k 10 400 python -u tools/bench_ssd.py --steps 20 --warmup 5 > gpurun_out/r6n_ssd_nokpad.log 2>&1 || { echo SSD0 FAILED; tail -20 gpurun_out/r6n_ssd_nokpad.log; exit 1; }
tail -1 gpurun_out/r6n_ssd_nokpad.log | cut -c1-160
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6n_prof -o trace -- python3 -u tools/bench_ssd.py --steps 8 --warmup 4 > gpurun_out/r6n_prof.log 2>&1 || { echo PROF FAILED; tail -5 gpurun_out/r6n_prof.log; exit 1; }
python tools/trace_window.py gpurun_out/r6n_prof --steps 4 --top 60 > gpurun_out/r6n_window.txt 2>&1; head -12 gpurun_out/r6n_window.txt | cut -c1-160
rm -rf gpurun_out/r6n_prof
