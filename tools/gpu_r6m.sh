#!/bin/bash
# deformable conv on the in-tree GEMMs: tests, SSD-512 bench + conv choices + rocprof window; 1-GPU eager ResNet-50
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_deform_conv.py tests/test_ssd.py > gpurun_out/r6m_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r6m_tests.log; exit 1; }
tail -1 gpurun_out/r6m_tests.log
MXAMD_BENCH_VERBOSE=1 timeout -k 10 400 python -u tools/bench_ssd.py --steps 20 --warmup 5 > gpurun_out/r6m_ssd.log 2>&1 || { echo SSD FAILED; tail -20 gpurun_out/r6m_ssd.log; exit 1; }
tail -1 gpurun_out/r6m_ssd.log | cut -c1-200
grep -E "conv-algo|algo " gpurun_out/r6m_ssd.log > gpurun_out/r6m_ssd_choices.txt || true
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6m_prof -o trace -- python3 -u tools/bench_ssd.py --steps 8 --warmup 4 > gpurun_out/r6m_prof.log 2>&1 || { echo PROF FAILED; tail -5 gpurun_out/r6m_prof.log; exit 1; }
python tools/trace_window.py gpurun_out/r6m_prof --steps 4 --top 45 > gpurun_out/r6m_window.txt 2>&1; head -30 gpurun_out/r6m_window.txt | cut -c1-160
rm -rf gpurun_out/r6m_prof
timeout -k 10 400 python -u bench.py --graph off --steps 20 --warmup 5 > gpurun_out/r6m_bench_eager.log 2>&1 || { echo EAGER FAILED; tail -20 gpurun_out/r6m_bench_eager.log; exit 1; }
tail -1 gpurun_out/r6m_bench_eager.log | cut -c1-300
