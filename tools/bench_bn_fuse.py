"""Is folding the BatchNorm-backward statistics into the dgrad epilogue a win?  For every ResNet-50 v1b
(b256 NHWC fp16) stride-1 dgrad that feeds a BN+ReLU, time

  unfused: best dgrad variant (ring / big / glds)  +  bn_reduce over (dy, z)
  fused:   best big-tile dgrad with the BN-backward epilogue (no reduce pass)

and print per-shape ms and the per-step totals.

    python tools/bench_bn_fuse.py [--batch 256] [--rounds 3]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxnet_maintenance_amd.ops import kernel_fns as KF  # noqa: E402

# stride-1 dgrads whose output is the gradient of a BN+ReLU output: (H, Cin(BN channels), Cout, k, count)
SHAPES = [
    (56, 64, 64, 3, 3), (56, 64, 256, 1, 3), (28, 128, 128, 3, 4), (28, 128, 512, 1, 4),
    (14, 256, 256, 3, 6), (14, 256, 1024, 1, 6), (7, 512, 512, 3, 3), (7, 512, 2048, 1, 3),
    (56, 256, 64, 1, 2), (28, 512, 128, 1, 3), (14, 1024, 256, 1, 5), (7, 2048, 512, 1, 2),
]


def timeit(fn, iters=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=256)
    ap.add_argument('--rounds', type=int, default=3)
    a = ap.parse_args()
    N, dt = a.batch, torch.float16
    tu = tf = 0.0
    for (H, C, K, k, cnt) in SHAPES:
        p = k // 2
        dy = torch.randn(N, H, H, K, device='cuda', dtype=dt)
        w = torch.randn(K, k, k, C, device='cuda', dtype=dt) * 0.05
        z = torch.randn(N, H, H, C, device='cuda', dtype=dt)
        mean = torch.zeros(C, device='cuda')
        scale = torch.ones(C, device='cuda')
        shift = torch.zeros(C, device='cuda')
        wd = KF._dgrad_weight(w)
        unf, fus = {}, {}
        for _ in range(a.rounds):
            for v in KF._fwd_variants(K, C):
                if v not in KF._RING_VARIANTS and v not in KF._BIG_VARIANTS and v not in (5, 6):
                    continue
                def run_u(v=v):
                    y = KF.conv_fwd(dy, wd, (1, 1), (k - 1 - p, k - 1 - p), None, v)
                    KF._bn_stats_pass(y)        # the backward reduce reads dy and z: two passes' bytes
                    KF._bn_stats_pass(z)
                    return y
                t = timeit(run_u)
                unf[v] = min(unf.get(v, 1e9), t)
                if v in KF._BIG_VARIANTS:
                    def run_f(v=v):
                        return KF.conv_fwd(dy, wd, (1, 1), (k - 1 - p, k - 1 - p), None, v,
                                           bn_bwd=(z, mean, scale, shift, None, 2, None))
                    fus[v] = min(fus.get(v, 1e9), timeit(run_f))
        bu = min(unf.items(), key=lambda kv: kv[1])
        bf = min(fus.items(), key=lambda kv: kv[1]) if fus else (None, float('inf'))
        tu += cnt * bu[1]
        tf += cnt * min(bu[1], bf[1])
        print('dgrad H%-3d %5d<-%-5d k%d x%d | unfused best %s %.3f | fused best %s %.3f | %s'
              % (H, C, K, k, cnt, bu[0], bu[1], bf[0], bf[1], 'FUSE' if bf[1] < bu[1] else 'keep'), flush=True)
    print('per-step totals (ms): unfused %.2f  with fusion where it wins %.2f' % (tu, tf))


if __name__ == '__main__':
    main()
