set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/prof_resnet_final
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all_final.log 2>&1; tail -3 gpurun_out/gpu_all_final.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 && tail -1 gpurun_out/smoke_final.log && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench_final.log 2>&1 && tail -1 gpurun_out/bench_final.log && \
timeout -k 10 300 python -u bench.py --gpus 2 --batch 64 --steps 3 --warmup 2 > gpurun_out/bench_2rank_final.log 2>&1 && tail -1 gpurun_out/bench_2rank_final.log && \
timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 --graph > gpurun_out/bench_bert_final.log 2>&1 && tail -1 gpurun_out/bench_bert_final.log && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_resnet_final -- python bench.py --steps 8 --warmup 6 > gpurun_out/prof_resnet_final.log 2>&1
