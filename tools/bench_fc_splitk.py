"""BERT FullyConnected weight-gradient GEMMs (dW = dY^T X, M = B*S rows) on one MI355X:
hipBLASLt torch.mm into the bf16 .grad (beta = 1) vs split-K batched GEMMs with fp32 partials
summed by the in-tree slab_reduce kernel (which accumulates into the .grad)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from mxnet_maintenance_amd.ops import kernels as K  # noqa: E402


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / it


def main():
    lib = K.lib()
    M = 4096
    st = torch.cuda.current_stream().cuda_stream
    for N, Kd in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
        dy = torch.randn(M, N, device='cuda', dtype=torch.bfloat16)
        x = torch.randn(M, Kd, device='cuda', dtype=torch.bfloat16)
        g = torch.zeros(N, Kd, device='cuda', dtype=torch.bfloat16)
        t_mm = timeit(lambda: g.addmm_(dy.t(), x))
        res = ['N=%d K=%d  mm %.1f us (%.0f TF/s)' % (N, Kd, t_mm * 1e3, 2 * M * N * Kd / t_mm / 1e9)]
        for S in (2, 4, 8):
            a = dy.view(S, M // S, N).transpose(1, 2)
            b = x.view(S, M // S, Kd)
            slab = torch.empty(S, N, Kd, device='cuda', dtype=torch.float32)

            def sk():
                torch.bmm(a, b, out_dtype=torch.float32, out=slab)
                lib.slab_reduce(2, slab.data_ptr(), S, N * Kd, g.data_ptr(), 1, st)
            ref = dy.float().t() @ x.float()
            g.zero_()
            sk()
            err = ((g.float() - ref).abs().max() / ref.abs().max()).item()
            t = timeit(sk)
            res.append('sk%d %.1f us (err %.1e)' % (S, t * 1e3, err))
        print(' | '.join(res), flush=True)


if __name__ == '__main__':
    main()
