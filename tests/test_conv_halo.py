"""Halo-tile 3x3 conv (src/kernels/conv_halo.hip): C = K = 64, stride 1, pad 1 -- forward against
fp32 PyTorch (image heights that are not multiples of the 4-row tile, widths up to 57, more tiles than
workgroups so the persistent loop and the double-buffered patches are exercised), the BatchNorm
statistics epilogue, the stride-1 data gradient on the flipped weight, and its BatchNorm-backward
statistics (modes 0 / 2)."""
import pytest
import torch
import torch.nn.functional as F

from mxnet_maintenance_amd.ops import kernel_fns as KF

pytestmark = pytest.mark.gpu


def _relnorm(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


@pytest.mark.parametrize('dt', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('shape', [(2, 13, 56), (300, 4, 7), (3, 9, 57), (1, 1, 1), (5, 56, 56)])
def test_halo_forward_and_bn_stats(dt, shape):
    N, H, W = shape
    torch.manual_seed(1)
    x = torch.randn(N, H, W, 64, device='cuda').to(dt)
    w = (torch.randn(64, 3, 3, 64, device='cuda') / 24.0).to(dt)
    assert KF.halo_ok(x, w, (1, 1), (1, 1))
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), None, 1, 1).permute(0, 2, 3, 1)
    y = KF.conv_halo(x, w, bn_stats=True)
    assert y.shape == ref.shape
    tol = 2e-3 if dt == torch.float16 else 1e-2
    assert _relnorm(y, ref) < tol, _relnorm(y, ref)
    part, nparts = y._mxamd_bn_part
    p = part.view(2, 64, nparts).sum(-1)
    yf = y.float()
    stol = 2e-3 if dt == torch.float16 else 1e-2     # the partials sum the fp32 accumulators, y is rounded
    assert _relnorm(p[0], yf.sum((0, 1, 2))) < stol
    assert _relnorm(p[1], (yf * yf).sum((0, 1, 2))) < stol
    y2 = KF.conv_halo(x, w)
    assert torch.equal(y2, y)            # deterministic, statistics epilogue does not change y


@pytest.mark.parametrize('relu', [True, False])
@pytest.mark.parametrize('dt', [torch.float16, torch.bfloat16])
def test_halo_dgrad_and_bn_backward_stats(dt, relu):
    N, H, W = 6, 14, 56
    torch.manual_seed(2)
    dy = torch.randn(N, H, W, 64, device='cuda').to(dt)
    w = (torch.randn(64, 3, 3, 64, device='cuda') / 24.0).to(dt)
    x = torch.randn(N, H, W, 64, device='cuda').to(dt).requires_grad_(False)
    ref = torch.nn.grad.conv2d_input((N, 64, H, W), w.float().permute(0, 3, 1, 2), dy.float().permute(0, 3, 1, 2),
                                     1, 1).permute(0, 2, 3, 1)
    z = torch.randn(N, H, W, 64, device='cuda').to(dt)
    mean = z.float().mean(dim=(0, 1, 2)).contiguous()
    scale = (torch.rand(64, device='cuda') + 0.5) if relu else None
    shift = (torch.randn(64, device='cuda') * 0.3) if relu else None
    src = (z, mean, scale, shift, None, 2 if relu else 0, object())
    dx = KF.conv_halo(dy, KF._dgrad_weight(w), bn_bwd=src)
    tol = 2e-3 if dt == torch.float16 else 1e-2
    assert _relnorm(dx, ref) < tol
    part, nparts, token, ver = dx._mxamd_bn_bwd
    assert token is src[6] and ver == dx._version
    p = part.view(2, 64, nparts).sum(-1)
    d = dx.float()
    if relu:
        d = d * ((z.float() * scale + shift) > 0)
    assert _relnorm(p[0], d.sum((0, 1, 2))) < 1e-3
    assert _relnorm(p[1], (d * (z.float() - mean)).sum((0, 1, 2))) < 1e-3
    # the dgrad candidates offer the halo kernel for this shape
    names = [n for n, _ in KF._dgrad_candidates(dy, x, w, (1, 1), (1, 1))]
    assert 'halo' in names
