"""Few-channel stride-2 stem convolution kernels (src/kernels/conv_stem.hip) against fp32 torch:
forward, fused BatchNorm statistics partials, and the deterministic slab-reduced weight gradient."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _kf():
    from mxnet_maintenance_amd.ops import kernel_fns as KF
    return KF


def _rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))


def _ref_fwd(x, w, pad):
    return torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), None, 2,
                                      pad).permute(0, 2, 3, 1)


SHAPES = [  # (N, H, W, C, R, S, pad)
    (4, 224, 224, 3, 7, 7, (3, 3)),     # ResNet stem
    (2, 37, 45, 3, 7, 7, (3, 3)),       # partial tiles in both directions
    (3, 64, 64, 3, 3, 3, (1, 1)),       # MobileNet / Inception-style 3x3/2
    (2, 50, 30, 1, 5, 5, (2, 2)),
    (2, 33, 33, 4, 8, 8, (3, 3)),
]


@pytest.mark.parametrize('shape', SHAPES)
@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
def test_stem_forward_and_bn_partials(shape, dtype):
    KF = _kf()
    N, H, W, C, R, S, pad = shape
    torch.manual_seed(0)
    x = torch.randn(N, H, W, C, device='cuda').to(dtype)
    w = (torch.randn(64, R, S, C, device='cuda') * 0.1).to(dtype)
    assert KF.stem_ok(x, w, (2, 2), pad)
    y = KF.conv_stem_fwd(x, w, pad, bn_stats=True)
    ref = _ref_fwd(x, w, pad)
    assert y.shape == ref.shape
    assert _rel(y, ref) < (5e-3 if dtype == torch.float16 else 2e-2)
    # the partials come from the fp32 accumulators: compare with the fp32 reference, to within the
    # accumulated difference of the operands' rounding
    part, nparts = y._mxamd_bn_part
    p = part.view(2, 64, nparts)
    rf = ref.float().reshape(-1, 64)
    scale = rf.abs().sum(0) * (2e-3 if dtype == torch.float16 else 1e-2) + 1e-2
    assert ((p[0].sum(1) - rf.sum(0)).abs() <= scale).all()
    sq = (rf * rf).sum(0)
    assert ((p[1].sum(1) - sq).abs() <= sq * (4e-3 if dtype == torch.float16 else 2e-2) + 1e-2).all()


@pytest.mark.parametrize('shape', SHAPES)
def test_stem_wgrad_matches_fp32_and_is_deterministic(shape):
    KF = _kf()
    N, H, W, C, R, S, pad = shape
    torch.manual_seed(1)
    x = torch.randn(N, H, W, C, device='cuda').half()
    w = (torch.randn(64, R, S, C, device='cuda') * 0.1).half()
    Ho, Wo = (H + 2 * pad[0] - R) // 2 + 1, (W + 2 * pad[1] - S) // 2 + 1
    dy = torch.randn(N, Ho, Wo, 64, device='cuda').half()
    xf = x.permute(0, 3, 1, 2).float().requires_grad_(False)
    wf = w.permute(0, 3, 1, 2).float().requires_grad_(True)
    yf = torch.nn.functional.conv2d(xf, wf, None, 2, pad)
    yf.backward(dy.permute(0, 3, 1, 2).float())
    ref = wf.grad.permute(0, 2, 3, 1)
    dw = KF.conv_stem_wgrad(x, dy, w.shape, pad, out=torch.empty(64, R, S, C, device='cuda'))
    assert _rel(dw, ref) < 2e-3
    dw2 = KF.conv_stem_wgrad(x, dy, w.shape, pad, out=torch.empty(64, R, S, C, device='cuda'))
    assert torch.equal(dw, dw2)
    acc = torch.ones(64, R, S, C, device='cuda').half()
    KF.conv_stem_wgrad(x, dy, w.shape, pad, out=acc, accum=True)
    assert _rel(acc.float() - 1.0, ref) < 5e-3
