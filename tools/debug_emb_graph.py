"""Embedding fwd+bwd captured in a HIP graph vs eager (debug aid)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mxnet_maintenance_amd.ops import nlp_fns

torch.manual_seed(int(sys.argv[1]) if len(sys.argv) > 1 else 0)
V, C, B, S = 30528, 768, 8, 128
idx = torch.randint(0, V, (B, S), device='cuda').float()
w = (torch.randn(V, C, device='cuda') * 0.02).to(torch.bfloat16).requires_grad_()
w.grad = torch.zeros_like(w)
dy = torch.randn(B, S, C, device='cuda').to(torch.bfloat16)
out = {}


def step():
    w.grad.zero_()
    y = nlp_fns.Embedding.apply(idx, w)
    y.backward(dy)
    out['y'] = y


s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        step()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
ref_y = out['y'].float().clone()
ref_g = w.grad.float().clone()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    step()
y = out['y']
for i in range(5):
    g.replay()
    torch.cuda.synchronize()
    print('replay', i, 'y err', float((y.float() - ref_y).abs().max()),
          'grad err', float((w.grad.float() - ref_g).abs().max()), 'grad max', float(ref_g.abs().max()), flush=True)
