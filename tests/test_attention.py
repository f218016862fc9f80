"""Fused self-attention kernels (src/kernels/attention.hip) vs a plain PyTorch fp32 reference (GPU only)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _fns():
    from mxnet_maintenance_amd.ops import kernels
    assert kernels.available(), 'HIP kernel extension not loaded: %s' % kernels.load_error()
    from mxnet_maintenance_amd.ops import attention_fns
    return attention_fns


def _ref(qkv, heads, mask=None, keep=None, p=0.0):
    """fp32 attention on the interleaved (S, B, H*3*D) layout; keep: (B, H, S, S) dropout mask."""
    S, B, C = qkv.shape
    D = C // (3 * heads)
    t = qkv.float().reshape(S, B, heads, 3, D).permute(3, 1, 2, 0, 4)
    q, k, v = t[0], t[1], t[2]
    s = q @ k.transpose(-1, -2) / math.sqrt(D)
    if mask is not None:
        s = s.masked_fill(mask.reshape(B, 1, 1, S) == 0, float('-inf'))
    a = torch.softmax(s, -1)
    if keep is not None:
        a = a * keep / (1 - p)
    o = a @ v
    return o.permute(2, 0, 1, 3).reshape(S, B, heads * D)


def _qkv(S, B, H, dtype, seed=0):
    g = torch.Generator(device='cpu').manual_seed(seed)
    return (torch.randn(S, B, H * 3 * 64, generator=g) * 0.8).to('cuda', dtype).requires_grad_()


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
@pytest.mark.parametrize('S,B,H', [(128, 4, 3), (32, 2, 2), (96, 3, 1), (256, 2, 2)])
@pytest.mark.parametrize('masked', [False, True])
def test_attention_fwd_bwd_matches_fp32(dtype, S, B, H, masked):
    A = _fns()
    qkv = _qkv(S, B, H, dtype)
    assert A.attention_ok(qkv, H)
    mask = None
    if masked:
        vl = torch.tensor([S - 7 * (i + 1) for i in range(B)])
        mask = (torch.arange(S).reshape(1, S) < vl.reshape(B, 1)).float().cuda()
    out = A.SelfAttention.apply(qkv, mask, H, 0.0)
    gy = torch.randn(out.shape, device='cuda').to(dtype)
    out.backward(gy)
    x32 = qkv.detach().float().requires_grad_()
    ref = _ref(x32, H, mask)
    ref.backward(gy.float())
    tol = 2e-2 if dtype == torch.bfloat16 else 4e-3
    torch.testing.assert_close(out.float(), ref, atol=tol, rtol=tol)
    gref = x32.grad
    scale = gref.abs().max().item()
    torch.testing.assert_close(qkv.grad.float(), gref, atol=tol * max(scale, 1.0), rtol=tol * 2)


def test_attention_dropout_mask_consistent_fwd_bwd():
    """Recover the kernel's dropout mask with V = identity, then check fwd/bwd against fp32 with that mask."""
    A = _fns()
    S, B, H, p, dtype = 64, 2, 2, 0.3, torch.bfloat16
    base = _qkv(S, B, H, dtype, seed=3).detach()
    probe = base.clone().reshape(S, B, H, 3, 64)
    probe[:, :, :, 2, :] = torch.eye(S, device='cuda', dtype=dtype).reshape(S, 1, 1, S)
    probe = probe.reshape(S, B, H * 192)
    torch.manual_seed(11)
    pd = A.SelfAttention.apply(probe, None, H, p)                     # (S_q, B, H*S_k) = P∘Z/(1-p)
    keep = (pd.float().reshape(S, B, H, S).permute(1, 2, 0, 3) != 0).float()
    rate = 1 - keep.mean().item()
    assert abs(rate - p) < 0.03, rate
    qkv = base.clone().requires_grad_()
    torch.manual_seed(11)
    out = A.SelfAttention.apply(qkv, None, H, p)
    gy = torch.randn(out.shape, device='cuda').to(dtype)
    out.backward(gy)
    x32 = base.float().requires_grad_()
    ref = _ref(x32, H, keep=keep, p=p)
    ref.backward(gy.float())
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(qkv.grad.float(), x32.grad, atol=3e-2 * max(x32.grad.abs().max().item(), 1.0),
                               rtol=5e-2)


def test_sdp_attention_op_dispatches_to_hip_kernel():
    from mxnet_maintenance_amd import nd
    import mxnet_maintenance_amd as mx
    S, B, H = 128, 2, 4
    x = torch.randn(S, B, H * 192).to('cuda', torch.bfloat16)
    X = nd.array(x.float().cpu().numpy(), ctx=mx.gpu(0)).astype('bfloat16')
    calls = []
    from mxnet_maintenance_amd.ops import attention_fns
    orig = attention_fns.SelfAttention.apply

    def spy(*a):
        calls.append(1)
        return orig(*a)
    attention_fns.SelfAttention.apply = spy
    try:
        out = nd.contrib.sdp_attention(X, heads=H)
    finally:
        attention_fns.SelfAttention.apply = orig
    assert calls, 'fused HIP attention was not used'
    ref = _ref(x, H)
    torch.testing.assert_close(torch.from_numpy(out.astype('float32').asnumpy()), ref.cpu(), atol=2e-2, rtol=2e-2)
