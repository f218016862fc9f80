"""Bandwidth probe of the BatchNorm apply kernels (src/kernels/bn_nhwc.hip bn_apply_kernel) on one
ResNet-sized tensor: plain, +ReLU, +addend, +addend+ReLU+mask.  Prints GB/s per variant.

    python tools/bn_apply_probe.py [--shape 256 56 56 256]
"""
import argparse
import json

import torch

from mxnet_maintenance_amd.ops import kernels as K
from mxnet_maintenance_amd.ops import kernel_fns as KF


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--shape', type=int, nargs=4, default=[256, 56, 56, 256])
    ap.add_argument('--iters', type=int, default=20)
    a = ap.parse_args()
    lib = K.lib()
    N, H, W, C = a.shape
    R = N * H * W
    dev = 'cuda'
    x = torch.randn(a.shape, device=dev, dtype=torch.float16)
    add = torch.randn(a.shape, device=dev, dtype=torch.float16)
    y = torch.empty_like(x)
    mask = torch.empty(x.numel() // 8, dtype=torch.uint8, device=dev)
    f = [torch.rand(C, device=dev) + 0.5 for _ in range(9)]
    s = torch.cuda.current_stream().cuda_stream
    out = {}
    for name, has_add, relu, has_mask in (('plain', 0, 0, 0), ('relu', 0, 1, 0), ('add', 1, 0, 0),
                                          ('add_relu', 1, 1, 0), ('add_relu_mask', 1, 1, 1)):
        def run():
            lib.bn_nhwc_forward(KF._DT[x.dtype], x.data_ptr(), add.data_ptr() if has_add else 0, y.data_ptr(),
                                mask.data_ptr() if has_mask else 0, f[0].data_ptr(), f[1].data_ptr(),
                                f[2].data_ptr(), 0, f[2].data_ptr(), f[3].data_ptr(), f[4].data_ptr(),
                                f[5].data_ptr(), f[6].data_ptr(), R, C, 1e-5, 0, relu, 0, 0.0, 0, 0, 0, s)
        for _ in range(3):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        nbytes = x.numel() * 2 * (2 + has_add) + (mask.numel() if has_mask else 0)
        out[name] = {'ms': round(ms, 4), 'GB/s': round(nbytes / ms / 1e6, 1)}
    print(json.dumps({'shape': a.shape, 'results': out}))


if __name__ == '__main__':
    main()
