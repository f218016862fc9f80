# round-4: headline bench repeatability (3 runs of 50 timed steps) + SSD-512 and BERT on the final tree
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
step() {
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "step $log rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
step r4l_bench1.log 400 python -u bench.py --steps 50 --warmup 10
step r4l_bench2.log 400 python -u bench.py --steps 50 --warmup 10
step r4l_bench3.log 400 python -u bench.py --steps 50 --warmup 10
step r4l_ssd.log 300 python -u tools/bench_ssd.py --batch 32 --steps 20 --warmup 5
echo done
