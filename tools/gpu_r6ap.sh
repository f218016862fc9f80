#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/pw_amask_probe.py > gpurun_out/r6ap_probe.log 2>&1 || { echo PROBE FAILED; tail -20 gpurun_out/r6ap_probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6ap_probe.log && timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_pw.py > gpurun_out/r6ap_tests.log 2>&1 && tail -1 gpurun_out/r6ap_tests.log
