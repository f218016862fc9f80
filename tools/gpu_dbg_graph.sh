set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_kernels.py -k "colsum or linear" > gpurun_out/colsum_tests2.log 2>&1 || { tail -40 gpurun_out/colsum_tests2.log; exit 1; }
tail -1 gpurun_out/colsum_tests2.log
timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 --graph > gpurun_out/bench_bert_colsum2.log 2>&1 && tail -1 gpurun_out/bench_bert_colsum2.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert_colsum2 -- python tools/bench_bert.py --steps 8 --warmup 4 --graph > gpurun_out/prof_bert_colsum2.log 2>&1 && \
timeout -k 10 400 python -u tools/debug_graph_resnet.py --lr 0.1 --batch 64 --size 224 --steps 12 > gpurun_out/dbg_graph_resnet.log 2>&1; tail -14 gpurun_out/dbg_graph_resnet.log
