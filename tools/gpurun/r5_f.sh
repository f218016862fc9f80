# round 5: pointwise kernels + pw addend (tee dgrad) + multi-stream graph tests; ResNet/SSD A/B of
# MXNET_GRAPH_STREAMS; profile window
set -o pipefail
TAG=${1:-r5f}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_pointwise_hip.py tests/test_conv_pw.py tests/test_graph_streams.py -m gpu -q -x --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
MXAMD_BENCH_VERBOSE=1 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2> gpurun_out/${TAG}_bench.err || exit $?
tail -1 gpurun_out/${TAG}_bench.log
grep "conv-algo" gpurun_out/${TAG}_bench.err | grep teedgrad | cut -c1-200
MXNET_GRAPH_STREAMS=2 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_s2.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench_s2.log
timeout -k 10 400 python -u tools/bench_ssd.py --batch 32 --steps 20 --warmup 5 --graph 1 > gpurun_out/${TAG}_ssd.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_ssd.log
MXNET_GRAPH_STREAMS=3 timeout -k 10 400 python -u tools/bench_ssd.py --batch 32 --steps 20 --warmup 5 --graph 1 > gpurun_out/${TAG}_ssd_s3.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_ssd_s3.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -- \
  python bench.py --steps 8 --warmup 6 > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
python tools/trace_window.py gpurun_out/${TAG}_prof --steps 5 --top 60 > gpurun_out/${TAG}_window.txt
head -12 gpurun_out/${TAG}_window.txt
