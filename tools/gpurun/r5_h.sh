# round 5: pw addend via LDS-DMA stage + 1-WG/CU pw shapes, colsum single launch; ResNet bench + window
set -o pipefail
TAG=${1:-r5h}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_conv_pw.py tests/test_pointwise_hip.py -m gpu -q -x --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
MXAMD_BENCH_VERBOSE=1 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2> gpurun_out/${TAG}_bench.err || exit $?
tail -1 gpurun_out/${TAG}_bench.log
grep "conv-algo pw" gpurun_out/${TAG}_bench.err | cut -c1-180
timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 --graph > gpurun_out/${TAG}_bert.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bert.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -- \
  python bench.py --steps 8 --warmup 6 > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
python tools/trace_window.py gpurun_out/${TAG}_prof --steps 5 --top 60 > gpurun_out/${TAG}_window.txt
head -12 gpurun_out/${TAG}_window.txt
MXNET_GRAPH_STREAMS=3 timeout -k 10 400 python -u tools/bench_ssd.py --batch 32 --steps 10 --warmup 3 --graph 0 > gpurun_out/${TAG}_ssd_s3_eager.log 2>&1
echo "ssd streams eager rc=$?"; tail -2 gpurun_out/${TAG}_ssd_s3_eager.log | cut -c1-300
