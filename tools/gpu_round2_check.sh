set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench_1gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py --gpus 2 --batch 64 --steps 3 --warmup 2 > gpurun_out/bench_2rank_selflaunch.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_resnet -- python bench.py --steps 6 --warmup 4 > gpurun_out/prof_resnet.log 2>&1
