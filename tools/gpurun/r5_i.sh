# round 5: BERT b32 graph regression hunt (455k r4 -> 350k r5h): A/B of the in-tree elementwise routing,
# kvstore engine ops, plus a steady-state window of the graph step
set -o pipefail
TAG=${1:-r5i}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 --graph > gpurun_out/${TAG}_bert.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bert.log | cut -c1-200
MXAMD_HIP_ELEMWISE=0 timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 --graph > gpurun_out/${TAG}_bert_noew.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bert_noew.log | cut -c1-200
MXAMD_KVSTORE_ENGINE=0 timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 --graph > gpurun_out/${TAG}_bert_nokv.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bert_nokv.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -- \
  python tools/bench_bert.py --steps 8 --warmup 6 --graph > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
python tools/trace_window.py gpurun_out/${TAG}_prof --steps 5 --top 40 > gpurun_out/${TAG}_window.txt
head -40 gpurun_out/${TAG}_window.txt | cut -c1-160
