"""gemm.hip on the BERT FFN shape (M=4096, N=3072, K=768), a few launches per tile config, for
rocprofv3 counter passes (L2 hit rate, waits)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from mxnet_maintenance_amd.ops import gemm as G  # noqa: E402

M, K, N = 4096, 768, 3072
x = torch.randn(M, K, device='cuda', dtype=torch.bfloat16)
w = torch.randn(N, K, device='cuda', dtype=torch.bfloat16) * 0.05
for cfg in ((0, 1), (1, 1), (5, 1)):
    for _ in range(3):
        G.gemm_nt(x, w, cfg=cfg)
for _ in range(3):
    torch.nn.functional.linear(x, w)
torch.cuda.synchronize()
print('ok')
