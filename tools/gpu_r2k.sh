set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/prof_resnet_r2k
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_all_r2k.log 2>&1 || { tail -40 gpurun_out/gpu_all_r2k.log; exit 1; }
tail -2 gpurun_out/gpu_all_r2k.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r2k.log 2>&1 && tail -1 gpurun_out/bench_r2k.log && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_resnet_r2k -- python bench.py --steps 8 --warmup 6 > gpurun_out/prof_resnet_r2k.log 2>&1
