set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/prof_bert_graph2
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_kernels.py tests/test_graph_step.py > gpurun_out/hip_tests4.log 2>&1 || { tail -30 gpurun_out/hip_tests4.log; exit 1; }
tail -1 gpurun_out/hip_tests4.log
timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 --graph > gpurun_out/bench_bert_b32_graph2.log 2>&1 && tail -1 gpurun_out/bench_bert_b32_graph2.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert_graph2 -- python tools/bench_bert.py --steps 8 --warmup 4 --graph > gpurun_out/prof_bert_graph2.log 2>&1
