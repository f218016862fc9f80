set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/prof_bert_ln
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_kernels.py -k "splitk or linear or colsum or layernorm" tests/test_graph_step.py > gpurun_out/ln_tests.log 2>&1 || { tail -40 gpurun_out/ln_tests.log; exit 1; }
tail -1 gpurun_out/ln_tests.log
timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 --graph > gpurun_out/bench_bert_ln.log 2>&1 && tail -1 gpurun_out/bench_bert_ln.log && \
timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 --graph --batch 64 > gpurun_out/bench_bert_ln_b64.log 2>&1 && tail -1 gpurun_out/bench_bert_ln_b64.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert_ln -- python tools/bench_bert.py --steps 8 --warmup 4 --graph > gpurun_out/prof_bert_ln.log 2>&1
