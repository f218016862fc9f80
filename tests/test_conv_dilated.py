"""Dilated (atrous) NHWC convolutions on the in-tree MFMA kernels: conv_big.hip with dilated taps
(forward; stride-1 data gradient through the flipped weight) and conv_wgrad.hip with dilated taps,
against an fp32 torch reference."""
import pytest
import torch


def _ref(x, w, stride, pad, dil):
    xr = x.float().cpu().permute(0, 3, 1, 2).requires_grad_()
    wr = w.float().cpu().permute(0, 3, 1, 2).requires_grad_()
    y = torch.nn.functional.conv2d(xr, wr, None, stride, pad, dil)
    return xr, wr, y


def _rel(a, b):
    return float((a.float().cpu() - b).norm() / b.norm().clamp_min(1e-12))


@pytest.mark.gpu
@pytest.mark.parametrize('C,K,H,stride,dil', [(64, 128, 20, 1, 2), (128, 64, 17, 1, 4), (64, 64, 19, 2, 2)])
def test_dilated_kernels_match_fp32_reference(C, K, H, stride, dil):
    from mxnet_maintenance_amd.ops import kernel_fns as KF
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, H, H, C, generator=g).to('cuda', torch.float16)
    w = (torch.randn(K, 3, 3, C, generator=g) * 0.05).to('cuda', torch.float16)
    pad = (dil, dil)
    xr, wr, yr = _ref(x, w, (stride, stride), pad, (dil, dil))
    gy = torch.randn(yr.shape, generator=g)
    yr.backward(gy)
    dy = gy.permute(0, 2, 3, 1).contiguous().to('cuda', torch.float16)
    for v, (bco, _bpix) in sorted(KF._BIG_VARIANTS.items()):
        if K % bco or v in KF._BIG_SKINNY:
            continue
        y = KF.conv_fwd(x, w, (stride, stride), pad, None, v, dil=(dil, dil))
        assert _rel(y.permute(0, 3, 1, 2), yr.detach()) < 1e-2, ('fwd', v)
    if stride == 1:
        for v, (bco, _bpix) in sorted(KF._BIG_VARIANTS.items()):
            if C % bco or v in KF._BIG_SKINNY:
                continue
            dx = KF.conv_fwd(dy, KF._dgrad_weight(w), (1, 1), (2 * dil - dil, 2 * dil - dil), None, v,
                             dil=(dil, dil))
            assert _rel(dx.permute(0, 3, 1, 2), xr.grad) < 1e-2, ('dgrad', v)
    dw = KF.conv_wgrad(x, dy, w.shape, (stride, stride), pad, dil=(dil, dil))
    assert _rel(dw.permute(0, 3, 1, 2), wr.grad) < 1e-2, 'wgrad'
    lib = KF._K.lib()
    for ring in range(1, 10):
        if lib.conv_nhwc_wgrad_ring_ok(C, K, 3, 3, ring):
            dw = KF.conv_wgrad(x, dy, w.shape, (stride, stride), pad, ring=ring, dil=(dil, dil))
            assert _rel(dw.permute(0, 3, 1, 2), wr.grad) < 1e-2, ('wgrad ring', ring)


@pytest.mark.gpu
def test_dilated_conv_op_autograd_matches_reference():
    """The Convolution op with dilate=(2, 2) routes to ConvDilNHWC and all gradients match."""
    from mxnet_maintenance_amd.ops import hip_ops
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, 64, 24, 24, generator=g)
    w = torch.randn(64, 64, 3, 3, generator=g) * 0.05
    b = torch.randn(64, generator=g)
    xd, wd, bd = (t.to('cuda', torch.float16).requires_grad_() for t in (x, w, b))
    xl = xd.permute(0, 2, 3, 1).contiguous().permute(0, 3, 1, 2)
    y = hip_ops.conv(xl, wd, bd, (1, 1), (2, 2), (2, 2), 1, False)
    fns = [y.grad_fn] + [f for f, _ in y.grad_fn.next_functions if f is not None]
    assert any('ConvDilNHWC' in type(f).__name__ for f in fns), [type(f).__name__ for f in fns]
    gy = torch.linspace(-1, 1, y.numel()).reshape(y.shape)
    y.backward(gy.to('cuda', torch.float16))
    xr, wr, br = (t.clone().requires_grad_() for t in (x, w, b))
    yr = torch.nn.functional.conv2d(xr, wr, br, 1, 2, 2)
    yr.backward(gy)
    assert _rel(y.detach(), yr.detach()) < 1e-2
    for a, r in ((xd.grad, xr.grad), (wd.grad, wr.grad), (bd.grad, br.grad)):
        assert _rel(a, r) < 1e-2
