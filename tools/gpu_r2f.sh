set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/prof_rn_graph
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u bench.py > gpurun_out/rn_default.log 2>&1 && tail -1 gpurun_out/rn_default.log && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rn_graph -- python bench.py --steps 8 --warmup 6 > gpurun_out/prof_rn_graph.log 2>&1
