# round-4: BERT-base b32 graph-step profile (kernel categories, hipBLASLt share)
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
step() {
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$R/gpurun_out/$log" 2>&1
  local rc=$?
  echo "step $log rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
step r4j_bert.log 300 python -u tools/bench_bert.py --batch 32 --steps 20 --warmup 5 --graph
cd /tmp
step r4j_bert_prof.log 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r4j_bert_prof -o run -- python3 $R/tools/bench_bert.py --batch 32 --steps 6 --warmup 5 --graph
cd $R
python tools/prof_summary.py gpurun_out/r4j_bert_prof 25 > gpurun_out/r4j_bert_prof_summary.txt 2>&1
echo done
