"""BatchNorm-backward statistics from the LDS-DMA dgrad epilogues (src/kernels/conv_glds.hip BnbG):
the stride-1 glds kernel (conv_fwd variants 5 / 6 on the flipped weight) and the strided phase kernel
emit per-channel (sum dz, sum dz*(z - mean)) of their output, dz = dX masked by z*scale + shift > 0
(or unmasked for a BN without ReLU).  Checked against fp32 PyTorch sums over the kernel's own dX."""
import pytest
import torch

from mxnet_maintenance_amd.ops import kernel_fns as KF

pytestmark = pytest.mark.gpu


def _src(shape, dt, relu):
    C = shape[-1]
    z = torch.randn(shape, device='cuda').to(dt)
    mean = z.float().mean(dim=(0, 1, 2)).contiguous()
    scale = (torch.rand(C, device='cuda') + 0.5) if relu else None
    shift = (torch.randn(C, device='cuda') * 0.3) if relu else None
    return (z, mean, scale, shift, None, 2 if relu else 0, object())


def _check(dx, src):
    part, nparts, token, ver = dx._mxamd_bn_bwd
    assert token is src[6] and ver == dx._version
    C = dx.shape[-1]
    p = part.view(2, C, nparts).sum(-1)
    z = src[0].float()
    d = dx.float()
    if src[2] is not None:
        d = d * ((z * src[2] + src[3]) > 0)
    s1 = d.sum(dim=(0, 1, 2))
    s2 = (d * (z - src[1])).sum(dim=(0, 1, 2))
    for got, ref in ((p[0], s1), (p[1], s2)):
        err = float((got - ref).norm() / ref.norm())
        assert err < 1e-3, err


@pytest.mark.parametrize('relu', [True, False])
@pytest.mark.parametrize('variant', [5, 6])
@pytest.mark.parametrize('dt', [torch.float16, torch.bfloat16])
def test_glds_stride1_dgrad_bn_stats(variant, dt, relu):
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')
    torch.manual_seed(0)
    N, H, W, C, K = 4, 14, 14, 128, 128
    dy = torch.randn(N, H, W, K, device='cuda').to(dt)
    w = (torch.randn(K, 3, 3, C, device='cuda') / (9 * K) ** 0.5).to(dt)
    src = _src((N, H, W, C), dt, relu)
    assert KF.glds_bnb_ok(src)
    dx = KF.conv_fwd(dy, KF._dgrad_weight(w), (1, 1), (1, 1), None, variant, bn_bwd=src)
    plain = KF.conv_fwd(dy, KF._dgrad_weight(w), (1, 1), (1, 1), None, variant)
    torch.testing.assert_close(dx, plain, rtol=0, atol=0)
    _check(dx, src)


@pytest.mark.parametrize('relu', [True, False])
@pytest.mark.parametrize('bco', [128, 64])
@pytest.mark.parametrize('case', [(4, 28, 28, 128, 128, 3, 1), (2, 14, 14, 256, 128, 1, 0)])
def test_phase_dgrad_bn_stats(case, bco, relu):
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')
    torch.manual_seed(1)
    N, H, W, C, K, R, p = case
    dt = torch.float16
    Ho, Wo = (H + 2 * p - R) // 2 + 1, (W + 2 * p - R) // 2 + 1
    dy = torch.randn(N, Ho, Wo, K, device='cuda').to(dt)
    w = (torch.randn(K, R, R, C, device='cuda') / (K * R * R) ** 0.5).to(dt)
    src = _src((N, H, W, C), dt, relu)
    assert KF.conv_dgrad_strided_ok(dy, w, (2, 2), (p, p), (N, H, W, C), bco)
    dx = KF.conv_dgrad_strided(dy, w, (2, 2), (p, p), (N, H, W, C), bco, bn_bwd=src)
    plain = KF.conv_dgrad_strided(dy, w, (2, 2), (p, p), (N, H, W, C), bco)
    torch.testing.assert_close(dx, plain, rtol=0, atol=0)
    _check(dx, src)
