set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/prof_resnet_margin
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_margin5.log 2>&1 && tail -1 gpurun_out/bench_margin5.log && \
MXAMD_VENDOR_MARGIN=0 timeout -k 10 300 python -u bench.py > gpurun_out/bench_margin0.log 2>&1 && tail -1 gpurun_out/bench_margin0.log && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench_margin5b.log 2>&1 && tail -1 gpurun_out/bench_margin5b.log && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_resnet_margin -- python bench.py --steps 8 --warmup 6 > gpurun_out/prof_resnet_margin.log 2>&1
