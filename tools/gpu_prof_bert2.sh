set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/prof_bert
timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 > gpurun_out/bench_bert_b32.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_bert.py --steps 10 --warmup 5 --batch 64 > gpurun_out/bench_bert_b64.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert -- python tools/bench_bert.py --steps 6 --warmup 3 > gpurun_out/prof_bert.log 2>&1
