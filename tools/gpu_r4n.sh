# round-4: SSD-512 A/B — the tree of commit a2473c8 (r4f-era, in _ab_old/) vs HEAD, same box, alternating
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step() {
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$R/gpurun_out/$log" 2>&1
  local rc=$?
  echo "step $log rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
step r4n_old1.log 300 python -u $R/_ab_old/tools/bench_ssd.py --batch 32 --steps 20 --warmup 5
step r4n_new1.log 300 python -u $R/tools/bench_ssd.py --batch 32 --steps 20 --warmup 5
step r4n_old2.log 300 python -u $R/_ab_old/tools/bench_ssd.py --batch 32 --steps 20 --warmup 5
step r4n_new2.log 300 python -u $R/tools/bench_ssd.py --batch 32 --steps 20 --warmup 5
echo done
