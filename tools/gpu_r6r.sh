#!/bin/bash
# full GPU suite + smoke + headline bench + window on the current tree
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/r6r_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r6r_tests.log; exit 1; }
tail -2 gpurun_out/r6r_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6r_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/r6r_smoke.log; exit 1; }
tail -1 gpurun_out/r6r_smoke.log
MXAMD_BENCH_VERBOSE=1 bash tools/gpu_bench.sh r6r && grep conv-algo gpurun_out/r6r_bench.log > gpurun_out/r6r_conv_choices.txt; grep -c conv-algo gpurun_out/r6r_conv_choices.txt
