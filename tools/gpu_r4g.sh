# round-4: deform test re-check, conv tile probes (timing + PMC counters), verbose bench (autotune table)
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
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
step r4g_deform.log 200 $PYT tests/test_deform_conv.py
P="python -u tools/conv_pmc_probe.py"
{
for v in 10 11 13 14 15 20 21 22; do $P --H 56 --C 64 --K 256 --k 1 --variant $v || exit 1; done
for v in 10 11 13 14 15; do $P --H 56 --C 64 --K 256 --k 1 --variant $v --addend 1 || exit 1; done
for v in 11 12 14; do $P --H 56 --C 64 --K 128 --k 1 --variant $v --addend 1 || exit 1; done
for v in 10 11 12 13 20 21 22 24; do $P --H 14 --C 256 --K 256 --k 3 --variant $v || exit 1; done
for v in 11 12 20 22; do $P --H 28 --C 128 --K 128 --k 3 --variant $v || exit 1; done
for v in 12 23 25; do $P --H 56 --C 64 --K 64 --k 3 --variant $v || exit 1; done
} > $R/gpurun_out/r4g_probe.log 2>&1
echo "probe rc=$?"
cd /tmp
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"
for cfg in "56 64 256 1 10" "56 64 256 1 14" "14 256 256 3 10" "56 64 64 3 23"; do
  set -- $cfg
  tag=H$1C$2K$3k$4v$5
  step r4g_pmcA_$tag.log 60 rocprofv3 --pmc $SQ --output-format csv -d $R/gpurun_out/r4g_pmcA_$tag -o run -- python3 $R/tools/conv_pmc_probe.py --H $1 --C $2 --K $3 --k $4 --variant $5 --iters 5
  step r4g_pmcB_$tag.log 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/r4g_pmcB_$tag -o run -- python3 $R/tools/conv_pmc_probe.py --H $1 --C $2 --K $3 --k $4 --variant $5 --iters 5
  step r4g_pmcC_$tag.log 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r4g_pmcC_$tag -o run -- python3 $R/tools/conv_pmc_probe.py --H $1 --C $2 --K $3 --k $4 --variant $5 --iters 5
done
cd $R
MXAMD_BENCH_VERBOSE=1 timeout -k 10 400 python -u bench.py --steps 10 --warmup 5 > gpurun_out/r4g_bench.log 2> gpurun_out/r4g_bench_algos.log
echo "bench rc=$?"
