# round 5: shared MFMA header (all kernels), pw BN-backward epilogue + transposed weights, tap transposes,
# BERT colsum two-launch fix, FC large-tile candidates, imperative worker streams.
# full GPU suite, ResNet bench + window, BERT bench, worker-stream overlap probe
set -o pipefail
TAG=${1:-r5l}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
MXAMD_BENCH_VERBOSE=1 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2> gpurun_out/${TAG}_bench.err || exit $?
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-250
grep -E "conv-algo (pw|[a-z0-9]+\+bn)" gpurun_out/${TAG}_bench.err | cut -c1-160
MXAMD_BENCH_VERBOSE=1 timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 --graph > gpurun_out/${TAG}_bert.log 2> gpurun_out/${TAG}_bert.err || exit $?
tail -1 gpurun_out/${TAG}_bert.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -- \
  python bench.py --steps 8 --warmup 6 > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
python tools/trace_window.py gpurun_out/${TAG}_prof --steps 5 --top 60 > gpurun_out/${TAG}_window.txt
head -14 gpurun_out/${TAG}_window.txt | cut -c1-160
timeout -k 10 120 python -u tools/worker_streams_probe.py --workers 1 > gpurun_out/${TAG}_ws.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/worker_streams_probe.py --workers 2 >> gpurun_out/${TAG}_ws.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_wsprof -- \
  python tools/worker_streams_probe.py --workers 2 >> gpurun_out/${TAG}_ws.log 2>&1 || exit $?
python tools/worker_streams_probe.py --report gpurun_out/${TAG}_wsprof >> gpurun_out/${TAG}_ws.log 2>&1
cat gpurun_out/${TAG}_ws.log | grep -v amdgpu.ids
