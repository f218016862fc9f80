"""Weight-gradient timing per ResNet-50 v1b layer (batch 256, NHWC fp16, one MI355X).

MIOpen (torch convolution_backward) vs the in-tree MFMA kernel
(src/kernels/conv_wgrad.hip).  Prints ms and TFLOP/s per layer and the
per-step totals (layer time x occurrences).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_convs import LAYERS, timeit  # noqa: E402
from mxnet_maintenance_amd.ops import kernel_fns as KF  # noqa: E402


def main():
    B = int(os.environ.get('BATCH', '256'))
    tot = {'miopen': 0.0, 'hip': 0.0}
    for (H, C, K, k, s, cnt) in LAYERS:
        pad = k // 2
        x = torch.randn(B, H, H, C, device='cuda', dtype=torch.float16)
        w = torch.randn(K, k, k, C, device='cuda', dtype=torch.float16)
        Ho = (H + 2 * pad - k) // s + 1
        dy = torch.randn(B, Ho, Ho, K, device='cuda', dtype=torch.float16)
        fl = 2.0 * B * Ho * Ho * K * C * k * k
        t_m = timeit(lambda: KF._conv_bwd_torch(dy, x, w, (s, s), (pad, pad), (False, True)))
        line = 'H=%3d C=%4d K=%4d k=%d s=%d x%d  miopen %.3f ms (%4.0f TF/s)' % (H, C, K, k, s, cnt, t_m,
                                                                             fl / t_m / 1e9)
        tot['miopen'] += t_m * cnt
        if KF.conv_wgrad_ok(x, w):
            t_r = timeit(lambda: KF.conv_wgrad(x, dy, w.shape, (s, s), (pad, pad), dma=False))
            t_h = timeit(lambda: KF.conv_wgrad(x, dy, w.shape, (s, s), (pad, pad)))
            line += '  hip-reg %.3f ms (%4.0f TF/s)  hip-dma %.3f ms (%4.0f TF/s)' % (t_r, fl / t_r / 1e9, t_h,
                                                                                  fl / t_h / 1e9)
            lib = KF._K.lib()
            for v in range(1, 10):
                if lib.conv_nhwc_wgrad_ring_ok(C, K, k, k, v):
                    t_v = timeit(lambda: KF.conv_wgrad(x, dy, w.shape, (s, s), (pad, pad), ring=v))
                    line += '  ring%d %.3f' % (v, t_v)
                    t_h = min(t_h, t_v)
            t_h = min(t_h, t_r)
            tot['hip'] += t_h * cnt
            line += '  | best-hip %.3f (%4.0f TF/s)' % (t_h, fl / t_h / 1e9)
        else:
            tot['hip'] += t_m * cnt
        print(line, flush=True)
        del x, w, dy
    print('per-step wgrad total: miopen %.3f ms, best-with-hip %.3f ms' % (tot['miopen'], tot['hip']))


if __name__ == '__main__':
    main()
