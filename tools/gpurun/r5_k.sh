# round 5: pw BN-backward statistics epilogue + pw transposed weights + tap transposes; BERT bias-grad colsum
# back to two launches (the fenced single launch cost 2.9 ms/step); tests, ResNet bench + window, BERT
set -o pipefail
TAG=${1:-r5k}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_conv_pw.py tests/test_pointwise_hip.py -m gpu -q -x --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
MXAMD_BENCH_VERBOSE=1 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2> gpurun_out/${TAG}_bench.err || exit $?
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-250
grep -E "conv-algo (pw|[a-z0-9]+\+bn)" gpurun_out/${TAG}_bench.err | cut -c1-160
timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 --graph > gpurun_out/${TAG}_bert.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bert.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -- \
  python bench.py --steps 8 --warmup 6 > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
python tools/trace_window.py gpurun_out/${TAG}_prof --steps 5 --top 60 > gpurun_out/${TAG}_window.txt
head -14 gpurun_out/${TAG}_window.txt | cut -c1-160
