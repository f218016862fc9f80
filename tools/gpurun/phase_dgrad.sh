# Strided-dgrad phase kernel: numerics tests, conv kernel regression tests, 1-GPU bench + steady-state profile.
# usage: bash tools/gpurun/phase_dgrad.sh TAG
set -o pipefail
TAG=${1:-phase}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_strided_dgrad.py tests/test_hip_kernels.py > gpurun_out/${TAG}_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] && \
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 && tail -1 gpurun_out/${TAG}_bench.log && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -- python bench.py --steps 8 --warmup 6 > gpurun_out/${TAG}_prof.log 2>&1 && \
python tools/trace_window.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_window.txt && head -40 gpurun_out/${TAG}_window.txt && \
timeout -k 10 300 python -u tools/autotune_report.py > gpurun_out/${TAG}_autotune.log 2>&1 && grep -B1 "dgrad.*(2, 2)" gpurun_out/${TAG}_autotune.log | head -30
