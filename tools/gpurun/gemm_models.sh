# GEMM/conv tests, ResNet-50 bench + steady-state profile + autotune report, BERT-base bench + profile.
set -o pipefail
TAG=${1:-gm}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm.py tests/test_hip_kernels.py tests/test_resnet_gpu.py tests/test_attention.py > gpurun_out/${TAG}_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${TAG}_tests.log; grep -E "^(FAILED|E  )" gpurun_out/${TAG}_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 && tail -1 gpurun_out/${TAG}_bench.log && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -- python bench.py --steps 8 --warmup 6 > gpurun_out/${TAG}_prof.log 2>&1 && \
python tools/trace_window.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_window.txt && head -10 gpurun_out/${TAG}_window.txt && \
timeout -k 10 300 python -u tools/autotune_report.py > gpurun_out/${TAG}_autotune.log 2>&1 && tail -2 gpurun_out/${TAG}_autotune.log && \
timeout -k 10 300 python -u tools/bench_bert.py --graph > gpurun_out/${TAG}_bert.log 2>&1 && tail -1 gpurun_out/${TAG}_bert.log && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_bprof -- python tools/bench_bert.py --graph --steps 8 --warmup 4 > gpurun_out/${TAG}_bprof.log 2>&1 && \
python tools/trace_window.py gpurun_out/${TAG}_bprof > gpurun_out/${TAG}_bwindow.txt && head -12 gpurun_out/${TAG}_bwindow.txt
