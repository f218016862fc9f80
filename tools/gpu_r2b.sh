set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/prof_bert
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 10 > gpurun_out/bench_statscharge.log 2>&1 && \
tail -1 gpurun_out/bench_statscharge.log && \
timeout -k 10 300 python -u tools/bench_bert.py --steps 10 --warmup 5 --batch 64 --graph > gpurun_out/bench_bert_b64_graph.log 2>&1 && \
tail -1 gpurun_out/bench_bert_b64_graph.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert -- python tools/bench_bert.py --steps 6 --warmup 3 > gpurun_out/prof_bert.log 2>&1
