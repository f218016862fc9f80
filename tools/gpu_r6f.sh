#!/bin/bash
# round 6f: native worker-stream dispatcher (engine tests, worker-stream GPU tests, overhead probe)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_worker_streams.py tests/test_worker_streams_cpu.py tests/test_engine_device.py tests/test_kvstore_engine.py tests/test_async_errors.py tests/test_c_api_more.py > gpurun_out/r6f_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r6f_tests.log; exit 1; }
tail -2 gpurun_out/r6f_tests.log
timeout -k 10 300 python -u tools/dispatch_overhead_probe.py > gpurun_out/r6f_dispatch_probe.log 2>&1; tail -3 gpurun_out/r6f_dispatch_probe.log
