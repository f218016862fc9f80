set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_hip_kernels.py -k "conv_ring or conv_big" > gpurun_out/ring_tests.log 2>&1; rc=$?; tail -5 gpurun_out/ring_tests.log; [ $rc -eq 0 ] && \
timeout -k 10 400 python -u tools/bench_conv_variants.py --rounds 3 > gpurun_out/ring_bench.log 2>&1; tail -40 gpurun_out/ring_bench.log
