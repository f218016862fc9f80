set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 > gpurun_out/bench_bert_again.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert -- python tools/bench_bert.py --steps 6 --warmup 3 > gpurun_out/prof_bert.log 2>&1 && \
MXAMD_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29544 tools/bench_bert.py --steps 3 --warmup 2 > gpurun_out/bench_bert_2rank_gloo.log 2>&1
