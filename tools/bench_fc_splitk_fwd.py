"""BERT FullyConnected GEMMs with a 768-wide output (attention projection / FFN2 forward, QKV / FFN1
data gradient) on one MI355X: hipBLASLt torch.mm vs split-K batched GEMMs over K with fp32 partials
summed by the in-tree slab_reduce kernel."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from mxnet_maintenance_amd.ops import kernels as K  # noqa: E402
from bench_fc_splitk import timeit  # noqa: E402


def main():
    lib = K.lib()
    st = torch.cuda.current_stream().cuda_stream
    for M in (4096, 8192):
        for N, Kd in ((768, 768), (768, 3072), (768, 2304), (3072, 768), (2304, 768)):
            a = torch.randn(M, Kd, device='cuda', dtype=torch.bfloat16)
            w = torch.randn(N, Kd, device='cuda', dtype=torch.bfloat16)
            t_mm = timeit(lambda: torch.mm(a, w.t()))
            res = ['M=%d N=%d K=%d  mm %.1f us (%.0f TF/s)' % (M, N, Kd, t_mm * 1e3, 2 * M * N * Kd / t_mm / 1e9)]
            for S in (2, 3, 4):
                if Kd % S or (Kd // S) % 64:
                    continue
                Kc = Kd // S
                av = a.view(M, S, Kc).transpose(0, 1)
                wv = w.view(N, S, Kc).transpose(0, 1).transpose(1, 2)
                slab = torch.empty(S, M, N, device='cuda', dtype=torch.float32)
                out = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)

                def sk():
                    torch.bmm(av, wv, out_dtype=torch.float32, out=slab)
                    lib.slab_reduce(2, slab.data_ptr(), S, M * N, out.data_ptr(), 0, st)
                sk()
                ref = a.float() @ w.float().t()
                err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
                t = timeit(sk)
                res.append('sk%d %.1f us (err %.1e)' % (S, t * 1e3, err))
            print(' | '.join(res), flush=True)


if __name__ == '__main__':
    main()
