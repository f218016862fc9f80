#!/bin/bash
# LDS mask bytes read through aligned dwords: tests, probe, bench
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_pw.py > gpurun_out/r6ax_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r6ax_tests.log; exit 1; }
tail -1 gpurun_out/r6ax_tests.log
timeout -k 10 200 python -u tools/pw_amask_probe.py > gpurun_out/r6ax_probe.log 2>&1 || { echo PROBE FAILED; tail -20 gpurun_out/r6ax_probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6ax_probe.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6ax_bench.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/r6ax_bench.log; exit 1; }
tail -1 gpurun_out/r6ax_bench.log | cut -c1-200
