# round 5: pw transposed-weight loads + tap-transpose dgrad weights (tests, ResNet bench), then the BERT regression A/B
# kvstore engine ops, plus a steady-state window of the graph step
set -o pipefail
TAG=${1:-r5i}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_conv_pw.py tests/test_pointwise_hip.py -m gpu -q -x --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
MXAMD_BENCH_VERBOSE=1 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2> gpurun_out/${TAG}_bench.err || exit $?
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-250
timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 --graph > gpurun_out/${TAG}_bert.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bert.log | cut -c1-200
MXAMD_HIP_ELEMWISE=0 timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 --graph > gpurun_out/${TAG}_bert_noew.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bert_noew.log | cut -c1-200
MXAMD_KVSTORE_ENGINE=0 timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 --graph > gpurun_out/${TAG}_bert_nokv.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bert_nokv.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -- \
  python tools/bench_bert.py --steps 8 --warmup 6 --graph > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
python tools/trace_window.py gpurun_out/${TAG}_prof --steps 5 --top 40 > gpurun_out/${TAG}_window.txt
head -40 gpurun_out/${TAG}_window.txt | cut -c1-160
