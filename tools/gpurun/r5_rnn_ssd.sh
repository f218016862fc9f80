# round 5: RNN kernel tests, LSTM LM A/B + profile, SSD-512 graph vs eager
set -o pipefail
TAG=${1:-r5c}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_rnn_kernels.py -m gpu -q --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_rnn_tests.log 2>&1
echo "rnn tests rc=$?"; tail -3 gpurun_out/${TAG}_rnn_tests.log
timeout -k 10 200 python -u tools/bench_lstm_lm.py > gpurun_out/${TAG}_lstm_intree.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_lstm_intree.log
MXAMD_RNN_VENDOR=1 timeout -k 10 200 python -u tools/bench_lstm_lm.py > gpurun_out/${TAG}_lstm_vendor.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_lstm_vendor.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_lstm_prof -- \
  python tools/bench_lstm_lm.py --steps 5 --warmup 3 > gpurun_out/${TAG}_lstm_prof.log 2>&1 || exit $?
python tools/prof_summary.py gpurun_out/${TAG}_lstm_prof > gpurun_out/${TAG}_lstm_prof_summary.txt 2>&1
head -30 gpurun_out/${TAG}_lstm_prof_summary.txt
timeout -k 10 400 python -u tools/bench_ssd.py --batch 32 --steps 20 --warmup 5 --graph 1 > gpurun_out/${TAG}_ssd_graph.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_ssd_graph.log
timeout -k 10 400 python -u tools/bench_ssd.py --batch 32 --steps 20 --warmup 5 --graph 0 > gpurun_out/${TAG}_ssd_eager.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_ssd_eager.log
