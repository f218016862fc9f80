"""One forward conv shape on one in-tree tile variant, repeated: the target of a rocprofv3 --pmc pass.

    rocprofv3 --pmc SQ_WAVE_CYCLES ... -- python3 tools/conv_pmc_probe.py --H 56 --C 64 --K 256 --k 1 --variant 10

Prints the mean time per launch (torch events) so a counter pass can be related to its wall time;
the shapes are ResNet-50 v1b layers at batch 256 (NHWC fp16).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxnet_maintenance_amd.ops import kernel_fns as KF  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=256)
    ap.add_argument('--H', type=int, default=56)
    ap.add_argument('--C', type=int, default=64)
    ap.add_argument('--K', type=int, default=256)
    ap.add_argument('--k', type=int, default=1)
    ap.add_argument('--stride', type=int, default=1)
    ap.add_argument('--variant', type=int, default=10)
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--addend', type=int, default=0)
    a = ap.parse_args()
    torch.manual_seed(0)
    x = torch.randn(a.batch, a.H, a.H, a.C, device='cuda').half()
    w = (torch.randn(a.K, a.k, a.k, a.C, device='cuda') / (a.k * a.k * a.C) ** 0.5).half()
    pad = a.k // 2
    add = None
    if a.addend:
        Ho = (a.H + 2 * pad - a.k) // a.stride + 1
        add = torch.randn(a.batch, Ho, Ho, a.K, device='cuda').half()
    run = lambda: KF.conv_fwd(x, w, (a.stride, a.stride), (pad, pad), None, a.variant, addend=add)  # noqa: E731
    run()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        run()
    e.record()
    e.synchronize()
    ms = s.elapsed_time(e) / a.iters
    Ho = (a.H + 2 * pad - a.k) // a.stride + 1
    flops = 2.0 * a.batch * Ho * Ho * a.K * a.k * a.k * a.C
    byts = 2.0 * (x.numel() + w.numel() + a.batch * Ho * Ho * a.K * (2 if a.addend else 1))
    print('shape H%d C%d K%d k%d s%d variant %d: %.4f ms  %.1f TF/s  %.2f TB/s (compulsory bytes)'
          % (a.H, a.C, a.K, a.k, a.stride, a.variant, ms, flops / ms / 1e9, byts / ms / 1e9), flush=True)


if __name__ == '__main__':
    main()
