#!/bin/bash
# full GPU suite + smoke + headline bench + window on the current tree
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/r6az_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r6az_tests.log; exit 1; }
tail -2 gpurun_out/r6az_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6az_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/r6az_smoke.log; exit 1; }
tail -1 gpurun_out/r6az_smoke.log
MXAMD_BENCH_VERBOSE=1 bash tools/gpu_bench.sh r6az && grep conv-algo gpurun_out/r6az_bench.log > gpurun_out/r6az_conv_choices.txt; grep -c conv-algo gpurun_out/r6az_conv_choices.txt
timeout -k 10 300 python -u tools/bench_bert.py --graph --gemm-table none --steps 20 --warmup 5 > gpurun_out/r6az_bert.log 2>&1 || { echo BERT FAILED; tail -20 gpurun_out/r6az_bert.log; exit 1; }
tail -1 gpurun_out/r6az_bert.log | cut -c1-200
timeout -k 10 400 python -u tools/bench_ssd.py --steps 20 --warmup 5 > gpurun_out/r6az_ssd.log 2>&1 || { echo SSD FAILED; tail -20 gpurun_out/r6az_ssd.log; exit 1; }
tail -1 gpurun_out/r6az_ssd.log | cut -c1-200
