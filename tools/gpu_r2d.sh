set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all.log 2>&1 || { tail -40 gpurun_out/gpu_all.log; exit 1; }
tail -3 gpurun_out/gpu_all.log
timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 --graph > gpurun_out/bench_bert_b32_graph.log 2>&1 || { tail -30 gpurun_out/bench_bert_b32_graph.log; exit 1; }
tail -1 gpurun_out/bench_bert_b32_graph.log
