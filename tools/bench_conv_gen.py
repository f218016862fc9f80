"""Per-shape timing of the generic in-tree convolution (src/kernels/conv_gen.hip and, for dilated
3x3 convs, the dilated conv_big path) against MIOpen on the layers of a ResNeXt-50 32x4d (grouped
3x3, 32 groups) and a DeepLab-v3 dilated ResNet (rate 2/4/6/12 3x3), fp16 NHWC, forward, data
gradient and weight gradient separately.  Prints one row per (shape, pass) with ms and TF/s for
each side and the winner.

    python tools/bench_conv_gen.py [--batch 64] [--reps 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from mxnet_maintenance_amd.ops import conv_gen as CG  # noqa: E402
from mxnet_maintenance_amd.ops import kernel_fns as KF  # noqa: E402


def best_of(fns, reps):
    """(ms, name) of the fastest closure."""
    return min((timeit(f, reps), n) for n, f in fns)

# name, H(=W), C, K, groups, stride, dilation
SHAPES = [
    ('resnext50_s1_3x3g32', 56, 128, 128, 32, 1, 1),
    ('resnext50_s2_3x3g32', 28, 256, 256, 32, 1, 1),
    ('resnext50_s2_3x3g32_s2', 56, 256, 256, 32, 2, 1),
    ('resnext50_s3_3x3g32', 14, 512, 512, 32, 1, 1),
    ('resnext50_s4_3x3g32', 7, 1024, 1024, 32, 1, 1),
    ('deeplab_s3_3x3_r2', 64, 256, 256, 1, 1, 2),
    ('deeplab_s4_3x3_r4', 64, 512, 512, 1, 1, 4),
    ('deeplab_aspp_3x3_r12', 64, 2048, 256, 1, 1, 12),
]


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=64)
    ap.add_argument('--reps', type=int, default=20)
    args = ap.parse_args()
    dt = torch.float16
    N = args.batch
    print('%-26s %-6s %9s %9s %8s %8s %s' % ('layer', 'pass', 'gen ms', 'miopen', 'gen TF/s', 'mio TF/s', 'winner'))
    wins = total = 0
    for name, H, C, K, G, s, d in SHAPES:
        pad = d
        Ho = (H + 2 * pad - d * 2 - 1) // s + 1
        flops = 2.0 * N * Ho * Ho * K * (C // G) * 9
        x = torch.randn(N, H, H, C, device='cuda', dtype=dt)
        w = torch.randn(K, 3, 3, C // G, device='cuda', dtype=dt) * 0.05
        x5, w5 = x.unsqueeze(1), w.unsqueeze(1)
        dy5 = torch.randn(N, 1, Ho, Ho, K, device='cuda', dtype=dt)
        xn = x.permute(0, 3, 1, 2)                        # channels-last memory for MIOpen
        wn = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        dyn = dy5.squeeze(1).permute(0, 3, 1, 2)
        st, pd, dl = (1, s, s), (0, pad, pad), (1, d, d)
        if G == 1:
            # dilated: conv_big with dilated taps (fwd; stride-1 dgrad on the flipped weight), conv_wgrad
            vs = [v for v, (bco, _b) in sorted(KF._BIG_VARIANTS.items()) if K % bco == 0 and v not in KF._BIG_SKINNY]
            wt = KF._dgrad_weight(w)
            dy4 = dy5.squeeze(1)
            pp = (d * 2 - pad, d * 2 - pad)
            lib = KF._K.lib()
            rings = [r for r in range(1, 10) if lib.conv_nhwc_wgrad_ring_ok(C, K, 3, 3, r)]
            fwd_c = [('hip%d' % v, lambda v=v: KF.conv_fwd(x, w, (s, s), (pad, pad), None, v, dil=(d, d))) for v in vs]
            dgr_c = [('hip%d' % v, lambda v=v: KF.conv_fwd(dy4, wt, (1, 1), pp, None, v, dil=(d, d))) for v in vs]
            wgr_c = [('hip', lambda: KF.conv_wgrad(x, dy4, w.shape, (s, s), (pad, pad), dil=(d, d)))] + \
                    [('ring%d' % r, lambda r=r: KF.conv_wgrad(x, dy4, w.shape, (s, s), (pad, pad), ring=r, dil=(d, d)))
                     for r in rings]
            passes = {'fwd': fwd_c, 'dgrad': dgr_c, 'wgrad': wgr_c}
            mio = {
                'fwd': lambda: F.conv2d(xn, wn, None, s, pad, d, G),
                'dgrad': lambda: torch.ops.aten.convolution_backward(dyn, xn, wn, None, (s, s), (pad, pad), (d, d),
                                                                     False, (0, 0), G, (True, False, False)),
                'wgrad': lambda: torch.ops.aten.convolution_backward(dyn, xn, wn, None, (s, s), (pad, pad), (d, d),
                                                                     False, (0, 0), G, (False, True, False)),
            }
            for pname, fns in passes.items():
                tg, nm = best_of(fns, args.reps)
                tm = timeit(mio[pname], args.reps)
                win = 'in-tree' if tg <= tm else 'miopen'
                wins += win == 'in-tree'
                total += 1
                print('%-26s %-6s %9.3f %9.3f %8.0f %8.0f %s (%s)' % (name, pname, tg, tm, flops / tg / 1e9,
                                                                       flops / tm / 1e9, win, nm), flush=True)
            continue
        passes = {
            'fwd': (lambda: CG.conv_gen_fwd(x5, w5, None, G, st, pd, dl),
                    lambda: F.conv2d(xn, wn, None, s, pad, d, G)),
            'dgrad': (lambda: CG.conv_gen_dgrad(dy5, w5, (1, H, H), G, st, pd, dl),
                      lambda: torch.ops.aten.convolution_backward(dyn, xn, wn, None, (s, s), (pad, pad), (d, d),
                                                                  False, (0, 0), G, (True, False, False))),
            'wgrad': (lambda: CG.conv_gen_wgrad(x5, dy5, w5.shape, G, st, pd, dl),
                      lambda: torch.ops.aten.convolution_backward(dyn, xn, wn, None, (s, s), (pad, pad), (d, d),
                                                                  False, (0, 0), G, (False, True, False))),
        }
        for pname, (gen, mio) in passes.items():
            tg, tm = timeit(gen, args.reps), timeit(mio, args.reps)
            win = 'gen' if tg <= tm else 'miopen'
            wins += win == 'gen'
            total += 1
            print('%-26s %-6s %9.3f %9.3f %8.0f %8.0f %s' % (name, pname, tg, tm, flops / tg / 1e9, flops / tm / 1e9,
                                                             win), flush=True)
    print('in-tree faster on %d of %d (shape, pass) pairs' % (wins, total))


if __name__ == '__main__':
    main()
