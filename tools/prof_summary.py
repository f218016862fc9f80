#!/usr/bin/env python
"""Summarise a rocprofv3 --kernel-trace --stats CSV directory: top kernels and per-class totals."""
import csv
import glob
import re
import sys


def classify(name):
    n = name.lower()
    if ('mxamd::' in n and ('conv' in n or 'gemm' in n or 'slab_reduce' in n)) or 'wgrad_reduce' in n:
        return 'conv/gemm (in-tree HIP MFMA)'
    if 'igemm' in n or 'conv' in n or 'gemm' in n or 'ck::' in n or 'xdl' in n or 'cijk' in n:
        return 'conv/gemm (MIOpen/hipBLASLt)'
    if 'attn' in n or 'fmha' in n or 'flash' in n or 'attention' in n:
        return 'attention (in-tree MFMA attn_* / SDPA)'
    if 'multibox' in n:
        return 'detection (MultiBoxTarget)'
    if 'bn_' in n or 'batch_norm' in n:
        return 'batchnorm'
    if 'layernorm' in n or 'column_sum' in n:
        return 'layernorm'
    if 'gelu' in n or 'dropout' in n:
        return 'gelu/dropout'
    if 'pool' in n or 'gap_' in n:
        return 'pooling'
    if 'sgd' in n or 'adam' in n or 'lamb_' in n or 'sumsq' in n or 'finite' in n:
        return 'optimizer'
    if 'softmax' in n or 'cross' in n:
        return 'softmax/ce'
    if 'elementwise' in n or 'functor' in n or 'fill' in n or 'copy' in n:
        return 'elementwise/copy (torch)'
    return 'other'


def main(d, steps):
    f = glob.glob(d + '/**/*kernel_stats.csv', recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    if steps <= 0:
        # one fused optimizer launch per training step (warmup included)
        steps = max(1, sum(int(r['Calls']) for r in rows if any(k in r['Name'] for k in ('flat_sgd', 'flat_adam', 'lamb_phase2'))))
    tot = sum(float(r['TotalDurationNs']) for r in rows)
    print('total kernel time %.2f ms (%d steps profiled -> %.2f ms/step)' % (tot / 1e6, steps, tot / 1e6 / steps))
    cls = {}
    for r in rows:
        c = classify(r['Name'])
        cls[c] = cls.get(c, 0) + float(r['TotalDurationNs'])
    for c, v in sorted(cls.items(), key=lambda kv: -kv[1]):
        print('  %-32s %8.2f ms/step  %5.1f%%' % (c, v / 1e6 / steps, 100 * v / tot))
    print('top kernels:')
    for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:40]:
        print('  %8.3f ms/step %5.1f%% %6s  %s' % (float(r['TotalDurationNs']) / 1e6 / steps, float(r['Percentage']),
                                              r['Calls'], re.sub(r'\s+', ' ', r['Name'])[:110]))


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 0)
