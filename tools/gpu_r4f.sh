# round-4: deform conv tests (fp32 column grads), SSD-512 b32 with deformable extras + rocprof, BERT bench
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
step() {
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$GRAFT_REPO_ROOT/gpurun_out/$log" 2>&1
  local rc=$?
  echo "step $log rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
step r4f_deform.log 200 $PYT tests/test_deform_conv.py
step r4f_ssd.log 300 python -u tools/bench_ssd.py --batch 32 --steps 10 --warmup 5
cd /tmp
step r4f_ssd_prof.log 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4f_ssd_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_ssd.py --batch 32 --steps 4 --warmup 3
cd $GRAFT_REPO_ROOT
python tools/prof_summary.py gpurun_out/r4f_ssd_prof 25 > gpurun_out/r4f_ssd_prof_summary.txt 2>&1
step r4f_bert.log 300 python -u tools/bench_bert.py --batch 32 --steps 20 --warmup 5 --graph
step r4f_convbig.log 300 $PYT tests/test_hip_kernels.py -k "conv_big or bn_bwd or teedgrad"
step r4f_bench.log 400 python -u bench.py --steps 30 --warmup 10
