"""GELU backward with the producing Dense's bias gradient as column partials
(nlp_kernels.hip gelu_bwd_colpart_kernel -> Linear.backward via dx._mxamd_bias_part) against a plain
PyTorch fp32 reference of Dense -> GELU."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-6))


@pytest.mark.parametrize('dt', [torch.bfloat16, torch.float16])
@pytest.mark.parametrize('M,N', [(4096, 3072), (300, 768), (37, 96), (5, 2056)])
def test_gelu_backward_colpart_matches_fp32(dt, M, N):
    from mxnet_maintenance_amd.ops import kernels as _K
    lib = _K.lib()
    torch.manual_seed(M + N)
    x = torch.randn(M, N, device='cuda', dtype=dt)
    gy = torch.randn(M, N, device='cuda', dtype=dt)
    dx = torch.empty_like(x)
    nb = lib.gelu_colpart_blocks(M, N)
    part = torch.full((nb, N), float('nan'), device='cuda')
    lib.gelu_backward_colpart({torch.float16: 1, torch.bfloat16: 2}[dt], x.data_ptr(), gy.data_ptr(), dx.data_ptr(),
                              part.data_ptr(), M, N, torch.cuda.current_stream().cuda_stream)
    xr = x.float().requires_grad_()
    torch.nn.functional.gelu(xr).backward(gy.float())
    assert _rel(dx, xr.grad) < 1e-2
    assert _rel(part.sum(0), xr.grad.sum(0)) < 1e-3


def test_dense_gelu_bias_gradient_from_partials():
    """Dense -> GELU on the HIP path: the Dense's bias gradient comes from the GELU backward's partials
    and matches fp32 autograd."""
    from mxnet_maintenance_amd.ops import hip_ops as H
    torch.manual_seed(3)
    dt = torch.bfloat16
    x = torch.randn(512, 256, device='cuda', dtype=dt)
    w = (torch.randn(1024, 256, device='cuda') * 0.05).to(dt).requires_grad_()
    b = (torch.randn(1024, device='cuda') * 0.1).to(dt).requires_grad_()
    gy = torch.randn(512, 1024, device='cuda', dtype=dt)
    y = H.gelu(H.linear(x, w, b))
    y.backward(gy)
    wr = w.detach().float().requires_grad_()
    br = b.detach().float().requires_grad_()
    torch.nn.functional.gelu(torch.nn.functional.linear(x.float(), wr, br)).backward(gy.float())
    assert _rel(b.grad, br.grad) < 2e-2
    assert _rel(w.grad, wr.grad) < 2e-2
