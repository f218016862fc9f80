#!/bin/bash
# gemm.hip L2 behaviour on the BERT FFN shape: TCC hit / miss and SQ waits per kernel
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/r6x_pmc -o pmc -- python3 tools/gemm_pmc_probe.py > gpurun_out/r6x_pmc.log 2>&1 || { echo PMC FAILED; tail -20 gpurun_out/r6x_pmc.log; exit 1; }
python3 - <<'PY'
import csv, collections, glob
f = glob.glob('gpurun_out/r6x_pmc/**/*counter_collection.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    agg[r.get('Kernel_Name', '')[:90]][r['Counter_Name']] += float(r['Counter_Value'])
for k, v in agg.items():
    if not ('gemm' in k or 'Cijk' in k):
        continue
    hit = v['TCC_HIT_sum'] / max(v['TCC_HIT_sum'] + v['TCC_MISS_sum'], 1)
    wc = max(v['SQ_WAVE_CYCLES'], 1)
    print('%s\n  L2 hit %.1f%%  waits %.0f%%  issue-stall %.0f%%  active %.0f%%  MFMA-busy %.3g  hits %.3g misses %.3g' % (
        k, 100 * hit, 100 * v['SQ_WAIT_ANY'] / wc, 100 * v['SQ_WAIT_INST_ANY'] / wc, 100 * v['SQ_ACTIVE_INST_ANY'] / wc,
        v['SQ_VALU_MFMA_BUSY_CYCLES'], v['TCC_HIT_sum'], v['TCC_MISS_sum']))
PY
for grp in 0 8 4 16; do
MXAMD_GEMM_GROUP=$grp timeout -k 10 300 python -u tools/bench_gemm.py --iters 30 > gpurun_out/r6x_gemm_g$grp.log 2>&1 || { echo GEMM FAILED; tail -20 gpurun_out/r6x_gemm_g$grp.log; exit 1; }
echo "== group $grp"; grep -E "^(fwd|dgrad) " gpurun_out/r6x_gemm_g$grp.log | cut -c1-120
grep -E "gemm\(" gpurun_out/r6x_gemm_g$grp.log | sort -t'(' -k2 | head -0
done
