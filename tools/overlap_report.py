"""Summarise copy/compute overlap from a rocprofv3 --kernel-trace --memory-copy-trace CSV run:
for every host-to-device copy, the fraction of its duration covered by kernels running at the
same time (on any stream)."""
import csv
import glob
import os
import sys


def _rows(pattern):
    for path in glob.glob(pattern, recursive=True):
        with open(path) as f:
            yield from csv.DictReader(f)


def main(root):
    kernels = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r.get('Kernel_Name', ''))
                     for r in _rows(os.path.join(root, '**', '*kernel_trace.csv')))
    copies = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r.get('Direction', r.get('Operation', '')))
              for r in _rows(os.path.join(root, '**', '*memory_copy_trace.csv'))]
    h2d = [c for c in copies if 'HOST_TO_DEVICE' in c[2].upper() and c[1] - c[0] > 100000]
    print('kernels %d, copies %d, large H2D copies %d' % (len(kernels), len(copies), len(h2d)))
    for s, e, d in h2d:
        covered = 0
        for ks, ke, _ in kernels:
            lo, hi = max(s, ks), min(e, ke)
            if hi > lo:
                covered += hi - lo
        print('H2D %.3f ms  overlapped by kernels %.0f%%' % ((e - s) / 1e6, 100.0 * min(1.0, covered / (e - s))))


if __name__ == '__main__':
    main(sys.argv[1])
