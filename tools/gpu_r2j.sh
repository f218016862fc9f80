set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all_r2j.log 2>&1; tail -5 gpurun_out/gpu_all_r2j.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r2j.log 2>&1 && tail -2 gpurun_out/smoke_r2j.log && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r2j.log 2>&1 && tail -1 gpurun_out/bench_r2j.log && \
timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 --graph > gpurun_out/bench_bert_r2j.log 2>&1 && tail -1 gpurun_out/bench_bert_r2j.log
