# GEMM kernel tests + conv/BN kernel tests + GEMM microbench + 1-GPU ResNet bench.
set -o pipefail
TAG=${1:-gemm}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm.py tests/test_hip_kernels.py tests/test_resnet_gpu.py > gpurun_out/${TAG}_tests.log 2>&1; rc=$?; tail -4 gpurun_out/${TAG}_tests.log; grep -E "^(FAILED|E  )" gpurun_out/${TAG}_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_gemm.py > gpurun_out/${TAG}_bench_gemm.log 2>&1; rc=$?; grep -E "^(fwd|dgrad|wgrad|total)" gpurun_out/${TAG}_bench_gemm.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 && tail -1 gpurun_out/${TAG}_bench.log
