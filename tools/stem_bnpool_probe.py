"""Stem BatchNorm + ReLU + 3x3/2 max pooling on ResNet-50's 256 x 112 x 112 x 64 fp16 tensor: the fused
operator (forward: one statistics + one pooling pass; backward: two gather passes) against BatchNorm+ReLU
followed by the pooling operator, forward and backward timed separately (ms)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxnet_maintenance_amd.ops import kernel_fns as KF  # noqa: E402
from mxnet_maintenance_amd.ops import hip_ops as H  # noqa: E402


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / iters


def main():
    C = 64
    x = (torch.randn(256, 112, 112, C, device='cuda') * 2).half().requires_grad_()
    g = (torch.rand(C, device='cuda') + 0.5).requires_grad_()
    b = torch.randn(C, device='cuda').requires_grad_()
    rm, rv = torch.zeros(C, device='cuda'), torch.ones(C, device='cuda')
    dy = torch.randn(256, 56, 56, C, device='cuda').half()

    def fused():
        return H.batch_norm_relu_maxpool(x, g, b, rm, rv, 1e-5, 0.9, False, True, 3, (3, 3), (2, 2), (1, 1))[0]

    def unfused():
        y = H.batch_norm(x, g, b, rm, rv, 1e-5, 0.9, False, True, 3, 'relu')[0]
        return H.pool(y, 'max', (3, 3), (2, 2), (1, 1), 'valid', True, True)

    for name, fn in (('fused', fused), ('bn+pool', unfused)):
        for fb in ((True, False) if name == 'fused' else (None,)):
            if fb is not None:
                KF._BN_POOL_BWD[0] = fb
            tf = timeit(lambda: fn().detach())
            y = fn()
            tb = timeit(lambda: torch.autograd.grad(fn(), (x, g, b), dy)) - tf
            print('%-8s %-14s fwd %.3f ms  bwd %.3f ms' % (name, '' if fb is None else ('gather-bwd' if fb else
                                                                                       'dense-bwd'), tf, tb),
                  flush=True)
            del y
    KF._BN_POOL_BWD[0] = True


if __name__ == '__main__':
    main()
