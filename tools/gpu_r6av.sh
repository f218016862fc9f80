#!/bin/bash
# counters: tee data gradient with the materialised vs the masked addend
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d gpurun_out/r6av_pmc -o pmc -- python3 -u tools/pw_amask_probe.py > gpurun_out/r6av_pmc.log 2>&1 || { echo PMC FAILED; tail -10 gpurun_out/r6av_pmc.log; exit 1; }
python - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/r6av_pmc/**/*counter_collection*.csv', recursive=True)
print(f)
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for path in f:
    for r in csv.DictReader(open(path)):
        k = r.get('Kernel_Name', '')
        if 'conv_pw_stream' not in k:
            continue
        key = k[k.find('<') + 1:k.find('>')]
        agg[key][r['Counter_Name']] += float(r['Counter_Value'])
        cnt[(key, r['Counter_Name'])] += 1
for key, d in agg.items():
    n = max(cnt[(key, c)] for c in d)
    print(key)
    print('   ' + '  '.join('%s=%.3g' % (c, v / n) for c, v in sorted(d.items())))
PY
rm -rf gpurun_out/r6av_pmc
