set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py -k "nchw" > gpurun_out/nchw_test.log 2>&1 || { tail -30 gpurun_out/nchw_test.log; exit 1; }
tail -1 gpurun_out/nchw_test.log
timeout -k 10 400 python -u bench.py --layout NCHW --steps 20 --warmup 10 > gpurun_out/rn_nchw.log 2>&1; tail -3 gpurun_out/rn_nchw.log
