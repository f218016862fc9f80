# round 5: vectorized tap transposes, relative-norm dW checks, worker streams (nested ops stay on the
# operator's stream) + spin-op overlap probe, BERT GEMM candidate dump, ResNet + SSD benches
set -o pipefail
TAG=${1:-r5m}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_pointwise_hip.py tests/test_hip_kernels.py tests/test_worker_streams.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/worker_streams_probe.py --workers 1 > gpurun_out/${TAG}_ws.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/worker_streams_probe.py --workers 2 >> gpurun_out/${TAG}_ws.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_wsprof -- \
  python tools/worker_streams_probe.py --workers 2 >> gpurun_out/${TAG}_ws.log 2>&1 || exit $?
python tools/worker_streams_probe.py --report gpurun_out/${TAG}_wsprof >> gpurun_out/${TAG}_ws.log 2>&1
grep -E "workers=|kernels per|overlapped" gpurun_out/${TAG}_ws.log
MXAMD_BENCH_VERBOSE=1 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2> gpurun_out/${TAG}_bench.err || exit $?
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-250
MXAMD_BENCH_VERBOSE=1 timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 --graph > gpurun_out/${TAG}_bert.log 2> gpurun_out/${TAG}_bert.err || exit $?
tail -1 gpurun_out/${TAG}_bert.log | cut -c1-200
grep "^algo" gpurun_out/${TAG}_bert.err | cut -c1-230
timeout -k 10 400 python -u tools/bench_ssd.py --batch 32 --steps 10 --warmup 3 > gpurun_out/${TAG}_ssd.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_ssd.log | cut -c1-250
