#!/bin/bash
# stem kernels: timing + one SQ counter pass
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python3 -u tools/stem_probe.py > gpurun_out/r6v_stem.log 2>&1 || { echo STEM FAILED; tail -20 gpurun_out/r6v_stem.log; exit 1; }
cat gpurun_out/r6v_stem.log
REPS=2 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/r6v_pmc -o pmc -- python3 tools/stem_probe.py > gpurun_out/r6v_pmc.log 2>&1 || { echo PMC FAILED; tail -20 gpurun_out/r6v_pmc.log; exit 1; }
find gpurun_out/r6v_pmc -name "*counter_collection.csv" | head -1 | xargs -I{} python3 -c "
import csv,collections,sys
rows=list(csv.DictReader(open('{}')))
agg=collections.defaultdict(lambda: collections.defaultdict(float)); cnt=collections.Counter()
for r in rows:
    k=r.get('Kernel_Name','')[:60]
    agg[k][r['Counter_Name']]+=float(r['Counter_Value'])
    cnt[(k,r['Counter_Name'])]+=1
for k,v in agg.items():
    if 'stem' not in k: continue
    print(k); print('  '+' '.join('%s=%.3g'%(n,x) for n,x in sorted(v.items())))
"
