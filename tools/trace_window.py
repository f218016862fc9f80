#!/usr/bin/env python
"""Per-step kernel breakdown from a rocprofv3 kernel trace, restricted to steady-state steps.

Step boundaries are the fused optimizer launches (flat_sgd); the window spans
the last ``--steps`` complete steps in the trace.  Usage:
    python tools/trace_window.py <trace dir> [--steps N] [--top K]
"""
import argparse
import collections
import csv
import glob
import re
import sys

sys.path.insert(0, __file__.rsplit('/', 1)[0])
from prof_summary import classify  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('d')
    ap.add_argument('--steps', type=int, default=6)
    ap.add_argument('--top', type=int, default=40)
    a = ap.parse_args()
    f = glob.glob(a.d + '/**/*kernel_trace.csv', recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    sgd = [int(r['End_Timestamp']) for r in rows if any(k in r['Kernel_Name'] for k in ('flat_sgd', 'flat_adam', 'lamb_phase2'))]
    # one step ends at its last optimizer launch; group launches closer than 1 ms
    ends = []
    for t in sgd:
        if ends and t - ends[-1] < 1_000_000:
            ends[-1] = t
        else:
            ends.append(t)
    if len(ends) < a.steps + 1:
        raise SystemExit('trace holds only %d step boundaries' % len(ends))
    lo, hi = ends[-a.steps - 1], ends[-1]
    n = a.steps
    win = [r for r in rows if lo < int(r['Start_Timestamp']) <= hi]
    tot = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in win)
    print('steady-state window: %d steps, kernel time %.2f ms/step, wall %.2f ms/step (profiled)'
          % (n, tot / 1e6 / n, (hi - lo) / 1e6 / n))
    by = collections.defaultdict(lambda: [0, 0])
    cls = collections.Counter()
    for r in win:
        d = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
        name = re.sub(r'\s+', ' ', r['Kernel_Name'])
        by[name][0] += d
        by[name][1] += 1
        cls[classify(name)] += d
    for c, v in cls.most_common():
        print('  %-32s %8.3f ms/step  %5.1f%%' % (c, v / 1e6 / n, 100 * v / tot))
    print('top kernels (ms/step, calls/step):')
    for name, (d, c) in sorted(by.items(), key=lambda kv: -kv[1][0])[:a.top]:
        print('  %8.3f  %5.1f  %s' % (d / 1e6 / n, c / n, name[:120]))


if __name__ == '__main__':
    main()
