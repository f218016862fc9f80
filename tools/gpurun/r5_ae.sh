# round 5: LayerNorm reads bf16/fp16 gamma/beta directly -- transformer-path tests + BERT bench
set -o pipefail
TAG=${1:-r5ae}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py tests/test_models.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
for r in a b; do
  timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 --graph > gpurun_out/${TAG}_bert_$r.log 2>&1 || exit $?
  echo "bert $r $(tail -1 gpurun_out/${TAG}_bert_$r.log | grep -o '"value": [0-9.]*')"
done
