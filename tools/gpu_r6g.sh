#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/worker_streams_probe.py --workers 1 > gpurun_out/r6g_ws1.log 2>&1; tail -1 gpurun_out/r6g_ws1.log
timeout -k 10 120 python -u tools/worker_streams_probe.py --workers 2 > gpurun_out/r6g_ws2.log 2>&1; tail -1 gpurun_out/r6g_ws2.log
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6g_trace -o run -- python3 tools/worker_streams_probe.py --workers 2 > gpurun_out/r6g_prof.log 2>&1
python tools/worker_streams_probe.py --report gpurun_out/r6g_trace | tee gpurun_out/r6g_report.txt
python - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r6g_trace/**/*kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
t0 = int(rows[0]['Start_Timestamp'])
for r in rows[-30:]:
    print(r.get('Stream_Id'), r.get('Queue_Id'), (int(r['Start_Timestamp'])-t0)//1000, (int(r['End_Timestamp'])-t0)//1000, r['Kernel_Name'][:50])
PY
rm -rf gpurun_out/r6g_trace
