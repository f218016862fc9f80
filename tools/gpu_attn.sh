set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/prof_bert_attn
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_attention.py > gpurun_out/attn_tests.log 2>&1 || { tail -40 gpurun_out/attn_tests.log; exit 1; }
tail -2 gpurun_out/attn_tests.log
timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 --graph > gpurun_out/bench_bert_attn.log 2>&1 && tail -1 gpurun_out/bench_bert_attn.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert_attn -- python tools/bench_bert.py --steps 8 --warmup 4 --graph > gpurun_out/prof_bert_attn.log 2>&1
