# round 5: run selected GPU test files. usage: bash tools/gpurun/r5_newtests.sh TAG test_files...
set -o pipefail
TAG=${1:-r5t}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest "$@" -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${TAG}_tests.log | tail -60
exit $rc
