# round 5: steady-state kernel windows of the final tree (ResNet-50 b256, BERT-base b32 graph step)
set -o pipefail
TAG=${1:-r5ad}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_bert_prof -- \
  python tools/bench_bert.py --steps 8 --warmup 6 --graph > gpurun_out/${TAG}_bert_prof.log 2>&1 || exit $?
python tools/trace_window.py gpurun_out/${TAG}_bert_prof --steps 5 --top 50 > gpurun_out/${TAG}_bert_window.txt || exit $?
head -14 gpurun_out/${TAG}_bert_window.txt | cut -c1-150
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -- \
  python bench.py --steps 8 --warmup 6 > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
python tools/trace_window.py gpurun_out/${TAG}_prof --steps 5 --top 80 > gpurun_out/${TAG}_window.txt || exit $?
head -10 gpurun_out/${TAG}_window.txt | cut -c1-150
