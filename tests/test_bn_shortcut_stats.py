"""Residual tail fed by a projection-shortcut BatchNorm: the tail's backward apply also reduces the
shortcut BN's backward statistics (bn_nhwc.hip bn_tail_bwd_ds_kernel), so the shortcut BN skips its
own reduction pass.  Gradients against a plain fp32 PyTorch reference of the same block tail."""
import pytest
import torch
import torch.nn.functional as F

from mxnet_maintenance_amd.ops import kernel_fns as KF

pytestmark = pytest.mark.gpu


def _ref_bn(x, g, b, eps):
    """Training-mode BatchNorm over the channel-last axis in fp32."""
    dims = tuple(range(x.dim() - 1))
    mean = x.mean(dims)
    var = x.var(dims, unbiased=False)
    return (x - mean) / torch.sqrt(var + eps) * g + b


@pytest.mark.parametrize('shape,dt', [((8, 14, 14, 256), torch.float16), ((4, 7, 7, 512), torch.bfloat16),
                                      ((16, 28, 28, 128), torch.float16)])
def test_tail_backward_carries_shortcut_bn_statistics(shape, dt):
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')
    torch.manual_seed(0)
    C = shape[-1]
    dev = 'cuda'
    x3 = torch.randn(shape, device=dev).to(dt).requires_grad_(True)
    xd = torch.randn(shape, device=dev).to(dt).requires_grad_(True)
    g1, b1 = (torch.rand(C, device=dev) + 0.5).requires_grad_(True), (torch.randn(C, device=dev) * 0.1).requires_grad_(True)
    g2, b2 = (torch.rand(C, device=dev) + 0.5).requires_grad_(True), (torch.randn(C, device=dev) * 0.1).requires_grad_(True)
    w = torch.randn(shape, device=dev)
    eps = 1e-5
    calls = []
    orig = KF._K.lib().bn_nhwc_backward

    def spy(*a, **k):
        calls.append(bool(k.get('ds_z')))
        return orig(*a, **k)
    lib = KF._K.lib()
    try:
        lib.bn_nhwc_backward = spy
    except (AttributeError, TypeError):
        lib = None
    yd = KF.BatchNormNHWC.apply(xd, g2, b2, None, eps, True, False, torch.zeros(C, device=dev),
                                torch.ones(C, device=dev), 0.9)[0]
    y = KF.BatchNormNHWC.apply(x3, g1, b1, yd, eps, True, True, torch.zeros(C, device=dev),
                               torch.ones(C, device=dev), 0.9)[0]
    (y.float() * w).sum().backward()
    if lib is not None:
        lib.bn_nhwc_backward = orig
        assert any(calls), 'the fused tail kernel did not run'
    # fp32 reference
    x3f = x3.detach().float().requires_grad_(True)
    xdf = xd.detach().float().requires_grad_(True)
    g1f, b1f, g2f, b2f = [t.detach().clone().requires_grad_(True) for t in (g1, b1, g2, b2)]
    ydf = _ref_bn(xdf, g2f, b2f, eps)
    yf = F.relu(_ref_bn(x3f, g1f, b1f, eps) + ydf.to(dt).float())
    (yf * w).sum().backward()

    def rel(a, b):
        return float((a.float() - b).norm() / b.norm())
    assert rel(y, yf.detach()) < 2e-2
    for got, ref in ((xd.grad, xdf.grad), (g2.grad, g2f.grad), (b2.grad, b2f.grad), (x3.grad, x3f.grad),
                     (g1.grad, g1f.grad), (b1.grad, b1f.grad)):
        assert rel(got, ref) < 3e-2, rel(got, ref)
