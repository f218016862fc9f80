#!/bin/bash
# BN finalize one wave per channel: BN tests, ResNet-50 bench + window (finalize kernel totals)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_relu_maxpool.py tests/test_resnet_gpu.py tests/test_hip_kernels.py tests/test_conv_pw.py -k "bn or norm or resnet or pool or pw" > gpurun_out/r6ak_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r6ak_tests.log; exit 1; }
tail -1 gpurun_out/r6ak_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6ak_bench.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/r6ak_bench.log; exit 1; }
tail -1 gpurun_out/r6ak_bench.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6ak_prof -o trace -- python3 -u bench.py --steps 8 --warmup 4 > gpurun_out/r6ak_prof.log 2>&1 || { echo PROF FAILED; tail -5 gpurun_out/r6ak_prof.log; exit 1; }
python tools/trace_window.py gpurun_out/r6ak_prof --steps 5 --top 70 > gpurun_out/r6ak_window.txt 2>&1; head -11 gpurun_out/r6ak_window.txt | cut -c1-160
grep -E "finalize|pool" gpurun_out/r6ak_window.txt | cut -c1-150
rm -rf gpurun_out/r6ak_prof
