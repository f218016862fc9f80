# Re-run the engine cross-stream and ResNet graph-vs-eager GPU tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_engine_device.py tests/test_resnet_gpu.py > gpurun_out/flaky_tests.log 2>&1; rc=$?; tail -4 gpurun_out/flaky_tests.log; exit $rc
