#!/bin/bash
# lazy shortcut gradient incl. the projection-shortcut BatchNorm: tests, A/B bench, window
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_conv_pw.py tests/test_resnet_gpu.py tests/test_bn_relu_maxpool.py > gpurun_out/r6an_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r6an_tests.log; exit 1; }
tail -1 gpurun_out/r6an_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6an_bench.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/r6an_bench.log; exit 1; }
tail -1 gpurun_out/r6an_bench.log | cut -c1-200
MXAMD_LAZY_SHORTCUT_GRAD=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6an_bench_off.log 2>&1 || { echo BENCH OFF FAILED; tail -20 gpurun_out/r6an_bench_off.log; exit 1; }
tail -1 gpurun_out/r6an_bench_off.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6an_prof -o trace -- python3 -u bench.py --steps 8 --warmup 4 > gpurun_out/r6an_prof.log 2>&1 || { echo PROF FAILED; tail -5 gpurun_out/r6an_prof.log; exit 1; }
python tools/trace_window.py gpurun_out/r6an_prof --steps 5 --top 60 > gpurun_out/r6an_window.txt 2>&1; head -11 gpurun_out/r6an_window.txt | cut -c1-160
grep -E "bn_bwd_apply|conv_pw_stream" gpurun_out/r6an_window.txt | cut -c1-150
rm -rf gpurun_out/r6an_prof
