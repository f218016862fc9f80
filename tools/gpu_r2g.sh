set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py -k "int8 or quantized" > gpurun_out/int8_tests.log 2>&1; tail -25 gpurun_out/int8_tests.log
