# BN-backward fusion: kernel/model tests (fused, then unfused for bisection) + fused-vs-unfused dgrad timing
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_hip_kernels.py tests/test_resnet_gpu.py -k "bn_backward_stats_fused or resnet" > gpurun_out/bnfuse_tests.log 2>&1; rc=$?; tail -8 gpurun_out/bnfuse_tests.log
[ $rc -le 1 ] || exit $rc
MXAMD_BN_BWD_FUSE=0 timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_resnet_gpu.py -k "graph_step" > gpurun_out/bnfuse_tests_off.log 2>&1; rc=$?; tail -5 gpurun_out/bnfuse_tests_off.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/bench_bn_fuse.py --rounds 3 > gpurun_out/bnfuse_bench.log 2>&1; tail -16 gpurun_out/bnfuse_bench.log
