"""Time every in-tree forward-conv tile variant against the vendor path on the ResNet-50 v1b (b256,
NHWC fp16) layer shapes, forward and dgrad-as-forward (stride-1 only).  Interleaved rounds in one
process; prints per-shape min-over-rounds ms for each family and the per-step totals.

    python tools/bench_conv_variants.py [--batch 256] [--rounds 3] [--only ring,big]
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxnet_maintenance_amd.ops import kernel_fns as KF  # noqa: E402

# (H_in, Cin, Cout, k, stride, count per step)
LAYERS = [
    (56, 64, 64, 1, 1, 1), (56, 64, 64, 3, 1, 3), (56, 64, 256, 1, 1, 4), (56, 256, 64, 1, 1, 2),
    (56, 256, 128, 1, 1, 1), (56, 128, 128, 3, 2, 1), (28, 128, 512, 1, 1, 4), (56, 256, 512, 1, 2, 1),
    (28, 512, 128, 1, 1, 3), (28, 128, 128, 3, 1, 3),
    (28, 512, 256, 1, 1, 1), (28, 256, 256, 3, 2, 1), (14, 256, 1024, 1, 1, 6), (28, 512, 1024, 1, 2, 1),
    (14, 1024, 256, 1, 1, 5), (14, 256, 256, 3, 1, 5),
    (14, 1024, 512, 1, 1, 1), (14, 512, 512, 3, 2, 1), (7, 512, 2048, 1, 1, 3), (14, 1024, 2048, 1, 2, 1),
    (7, 2048, 512, 1, 1, 2), (7, 512, 512, 3, 1, 2),
]


def timeit(fn, iters=8):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def family(v):
    if v == 'halo':
        return 'halo'
    if v in KF._RING_VARIANTS:
        return 'ring'
    if v in KF._BIG_VARIANTS:
        return 'big32' if 16 <= v <= 19 else ('big224' if v in (26, 27) else 'big')
    return 'glds' if v in (5, 6) else 'reg'


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=256)
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--stats', action='store_true', help='BN statistics epilogue on')
    a = ap.parse_args()
    N = a.batch
    dt = torch.float16
    fams = ('ring', 'big', 'big32', 'big224', 'glds', 'halo', 'vendor')
    tot = {f: 0.0 for f in fams}
    best_tot = 0.0
    for (H, Cin, Cout, k, s, cnt) in LAYERS:
        for kind in ('fwd', 'dgrad'):
            if kind == 'dgrad':
                if s != 1:
                    continue
                Cin, Cout = Cout, Cin   # dgrad = forward conv of dy with the flipped weight
            pad = k // 2
            Ho = (H + 2 * pad - k) // s + 1
            x = torch.randn(N, H, H, Cin, device='cuda', dtype=dt)
            w = torch.randn(Cout, k, k, Cin, device='cuda', dtype=dt) * 0.05
            cands = {}
            for v in KF._fwd_variants(Cin, Cout):
                cands[v] = (lambda v=v: KF.conv_fwd(x, w, (s, s), (pad, pad), None, v, bn_stats=a.stats))
            if KF.halo_ok(x, w, (s, s), (pad, pad)):
                cands['halo'] = (lambda: KF.conv_halo(x, w, bn_stats=a.stats))
            xc, wc = x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2)
            cands['vendor'] = lambda: F.conv2d(xc, wc, None, s, pad)
            ref = cands['vendor']().permute(0, 2, 3, 1).float()
            bad = []
            for v, fn in cands.items():
                if v != 'vendor':
                    err = float((fn().float() - ref).abs().max() / (ref.abs().max() + 1e-6))
                    if not err < 2e-2:
                        bad.append((v, err))
            t = {v: 1e9 for v in cands}
            for _ in range(a.rounds):
                for v, fn in cands.items():
                    t[v] = min(t[v], timeit(fn))
            fl = 2.0 * N * Ho * Ho * Cout * Cin * k * k
            line = '%-5s H%-3d %4d->%-4d k%d s%d x%d %6.1fGF |' % (kind, H, Cin, Cout, k, s, cnt, fl / 1e9)
            fbest = {}
            for f in fams:
                vs = [(tt, v) for v, tt in t.items() if (v == 'vendor') == (f == 'vendor') and
                      (f == 'vendor' or family(v) == f) and v not in dict(bad)]
                if vs:
                    fbest[f] = min(vs)
                    tot[f] += fbest[f][0] * cnt
                    line += ' %s %.3f(%s)' % (f, fbest[f][0], fbest[f][1])
            b = min(fbest.values())
            best_tot += b[0] * cnt
            line += ' | best %s %.0f TF/s' % (b[1], fl / b[0] / 1e9)
            if bad:
                line += ' BAD:%s' % bad
            print(line, flush=True)
    print('per-step totals (ms):', ' '.join('%s %.2f' % kv for kv in tot.items()), 'best-of-all %.2f' % best_tot)


if __name__ == '__main__':
    main()
