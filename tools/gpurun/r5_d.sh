# round 5: RNN split-K kernels + LSTM A/B, streaming 1x1 conv tests, ResNet bench, SSD graph
set -o pipefail
TAG=${1:-r5d}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_rnn_kernels.py tests/test_conv_pw.py -m gpu -q --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 200 python -u tools/bench_lstm_lm.py > gpurun_out/${TAG}_lstm_intree.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_lstm_intree.log
timeout -k 10 200 python -u tools/bench_lstm_lm.py --dtype bfloat16 > gpurun_out/${TAG}_lstm_intree_bf16.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_lstm_intree_bf16.log
MXAMD_RNN_VENDOR=1 timeout -k 10 200 python -u tools/bench_lstm_lm.py --dtype bfloat16 > gpurun_out/${TAG}_lstm_vendor_bf16.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_lstm_vendor_bf16.log
MXAMD_BENCH_VERBOSE=1 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2> gpurun_out/${TAG}_bench.err || exit $?
tail -1 gpurun_out/${TAG}_bench.log
grep -c "conv-algo pw" gpurun_out/${TAG}_bench.err
timeout -k 10 400 python -u tools/bench_ssd.py --batch 32 --steps 20 --warmup 5 --graph 1 > gpurun_out/${TAG}_ssd_graph.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_ssd_graph.log
