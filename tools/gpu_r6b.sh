#!/bin/bash
# round 6b: 224/448-pixel conv_big tiles, kvstore failure recovery, worker-stream allocator records
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py -k "conv_big_bn_stats or pool" tests/test_kvstore_engine.py tests/test_worker_streams.py > gpurun_out/r6b_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r6b_tests.log; exit 1; }
tail -3 gpurun_out/r6b_tests.log
timeout -k 10 500 python -u tools/bench_conv_variants.py --rounds 2 > gpurun_out/r6b_conv_variants.txt 2>&1
rc=$?
tail -50 gpurun_out/r6b_conv_variants.txt
exit $rc
