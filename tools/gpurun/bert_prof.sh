# BERT-base pre-training bench (HIP graph) + steady-state rocprofv3 window.
# usage: bash tools/gpurun/bert_prof.sh TAG
set -o pipefail
TAG=${1:-bert}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/bench_bert.py --graph > gpurun_out/${TAG}_bert.log 2>&1 && tail -1 gpurun_out/${TAG}_bert.log && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_bprof -- python tools/bench_bert.py --graph --steps 8 --warmup 4 > gpurun_out/${TAG}_bprof.log 2>&1 && \
python tools/trace_window.py gpurun_out/${TAG}_bprof > gpurun_out/${TAG}_bwindow.txt && head -30 gpurun_out/${TAG}_bwindow.txt
