"""GELU backward with bias partials (gelu_bwd_colpart_kernel + column_sum_partials) against the plain GELU
backward + the two-pass column sum it replaces, on BERT's FFN-1 shape (4096 x 3072 bf16)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxnet_maintenance_amd.ops import kernels as _K  # noqa: E402
from mxnet_maintenance_amd.ops import nlp_fns as NF  # noqa: E402


def timeit(fn, iters=50):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    lib = _K.lib()
    st = torch.cuda.current_stream().cuda_stream
    for M, N in ((4096, 3072), (4096, 768), (640, 768)):
        x = torch.randn(M, N, device='cuda', dtype=torch.bfloat16)
        gy = torch.randn(M, N, device='cuda', dtype=torch.bfloat16)
        dx = torch.empty_like(x)
        nb = lib.gelu_colpart_blocks(M, N)
        part = torch.empty(nb, N, device='cuda')
        db = torch.zeros(N, device='cuda', dtype=torch.bfloat16)

        def old():
            lib.gelu_backward(2, x.data_ptr(), gy.data_ptr(), dx.data_ptr(), x.numel(), st)
            NF.bias_grad(dx, None, torch.bfloat16)

        def gel():
            lib.gelu_backward(2, x.data_ptr(), gy.data_ptr(), dx.data_ptr(), x.numel(), st)

        def colp():
            lib.gelu_backward_colpart(2, x.data_ptr(), gy.data_ptr(), dx.data_ptr(), part.data_ptr(), M, N, st)

        def new():
            colp()
            lib.column_sum_partials(2, part.data_ptr(), nb, N, db.data_ptr(), 0, st)
        print('M%d N%d: gelu_bwd %.1f us, gelu_bwd+bias_grad %.1f us | colpart %.1f us, colpart+column_sum %.1f us'
              % (M, N, timeit(gel), timeit(old), timeit(colp), timeit(new)), flush=True)


if __name__ == '__main__':
    main()
