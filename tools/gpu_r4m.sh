# round-4: SSD-512 repeatability (two runs of 20 timed steps) on the final tree
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
step r4m_ssd1.log 300 python -u tools/bench_ssd.py --batch 32 --steps 20 --warmup 5
step r4m_ssd2.log 300 python -u tools/bench_ssd.py --batch 32 --steps 20 --warmup 10
echo done
