"""1x1 stride-2 data gradient in one big-tile pass (conv_big.hip GeomB::up = 2): dY . W written to the
even pixels of dX, the other three pixels of every 2x2 block zeroed by the same epilogue; checked
against fp32 PyTorch, with and without the BatchNorm-backward statistics epilogue."""
import pytest
import torch

from mxnet_maintenance_amd.ops import kernel_fns as KF

pytestmark = pytest.mark.gpu


def _relnorm(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


@pytest.mark.parametrize('dt', [torch.float16, torch.bfloat16])
@pytest.mark.parametrize('shape', [(3, 7, 9, 128, 256), (2, 14, 14, 256, 512)])
def test_up2_dgrad_matches_torch(dt, shape):
    N, Ho, Wo, C, K = shape
    torch.manual_seed(3)
    dy = torch.randn(N, Ho, Wo, K, device='cuda').to(dt)
    w = (torch.randn(K, 1, 1, C, device='cuda') / K ** 0.5).to(dt)
    xshape = (N, 2 * Ho, 2 * Wo, C)
    assert KF.conv_up2_ok(dy, w, (2, 2), (0, 0), xshape)
    ref = torch.nn.grad.conv2d_input((N, C, 2 * Ho, 2 * Wo), w.float().permute(0, 3, 1, 2),
                                     dy.float().permute(0, 3, 1, 2), 2, 0).permute(0, 2, 3, 1)
    tol = 2e-3 if dt == torch.float16 else 1e-2
    for v, (bco, _) in sorted(KF._BIG_VARIANTS.items()):
        if C % bco or v in KF._BIG_SKINNY:
            continue
        torch.cuda.synchronize()
        dx = torch.full(xshape, float('nan'), device='cuda').to(dt)   # poison: every pixel must be written
        dx = KF.conv_dgrad_up2(dy, w, v)
        assert dx.shape == xshape
        assert torch.isfinite(dx.float()).all()
        assert _relnorm(dx, ref) < tol, (v, _relnorm(dx, ref))
        assert float(dx[:, 1::2].float().abs().max()) == 0 and float(dx[:, :, 1::2].float().abs().max()) == 0
    # BN-backward statistics of dX (mode 2: ReLU mask from z)
    z = torch.randn(xshape, device='cuda').to(dt)
    mean = z.float().mean((0, 1, 2)).contiguous()
    scale = torch.rand(C, device='cuda') + 0.5
    shift = torch.randn(C, device='cuda') * 0.3
    src = (z, mean, scale, shift, None, 2, object())
    dx = KF.conv_dgrad_up2(dy, w, 10 if C % 256 == 0 else 11, bn_bwd=src)
    part, nparts, token, _ver = dx._mxamd_bn_bwd
    p = part.view(2, C, nparts).sum(-1)
    d = dx.float() * ((z.float() * scale + shift) > 0)
    assert _relnorm(p[0], d.sum((0, 1, 2))) < 1e-3
    assert _relnorm(p[1], (d * (z.float() - mean)).sum((0, 1, 2))) < 1e-3
