# 1-GPU ResNet-50 bench + rocprofv3 kernel stats only.  usage: bash tools/gpurun/bench_prof.sh TAG [bench args]
set -o pipefail
TAG=${1:-run}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u bench.py "$@" > gpurun_out/${TAG}_bench.log 2>&1 && tail -1 gpurun_out/${TAG}_bench.log && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -- python bench.py --steps 8 --warmup 6 "$@" > gpurun_out/${TAG}_prof.log 2>&1 && \
python tools/prof_summary.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_prof_summary.txt && head -14 gpurun_out/${TAG}_prof_summary.txt
