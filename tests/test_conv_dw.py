"""Depthwise NHWC convolution (src/kernels/conv_dw.hip) against fp32 torch ``conv2d(groups=C)``:
forward, data gradient and weight gradient, strides 1/2, dilation, 3x3 and 5x5, fp32/fp16/bf16."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [
    # N, H, W, C, R, stride, pad, dilate
    (4, 28, 28, 32, 3, 1, 1, 1),
    (2, 15, 17, 96, 3, 2, 1, 1),
    (2, 14, 14, 144, 5, 1, 2, 1),
    (3, 16, 16, 64, 3, 1, 2, 2),
    (2, 9, 9, 960, 3, 2, 1, 1),
]


def _ref(x, w, b, st, p, d):
    """fp32 NCHW torch reference on NHWC inputs; returns NHWC output and grads."""
    xr = x.detach().float().cpu().permute(0, 3, 1, 2).requires_grad_()
    wr = w.detach().float().cpu().permute(0, 3, 1, 2).requires_grad_()
    br = b.detach().float().cpu().requires_grad_()
    y = F.conv2d(xr, wr, br, stride=st, padding=p, dilation=d, groups=xr.shape[1])
    gy = torch.linspace(-1, 1, y.numel()).reshape(y.shape)
    y.backward(gy)
    return (y.detach().permute(0, 2, 3, 1), xr.grad.permute(0, 2, 3, 1), wr.grad.permute(0, 2, 3, 1), br.grad,
            gy.permute(0, 2, 3, 1).contiguous())


@pytest.mark.parametrize('shape', SHAPES)
@pytest.mark.parametrize('dtype', [torch.float32, torch.float16, torch.bfloat16])
def test_depthwise_matches_fp32_torch(shape, dtype):
    from mxnet_maintenance_amd.ops import kernels
    from mxnet_maintenance_amd.ops.conv_dw import ConvDwNHWC, dw_ok
    assert kernels.available(), kernels.load_error()
    N, H, W, C, R, st, p, d = shape
    g = torch.Generator().manual_seed(C + R)
    x = torch.randn(N, H, W, C, generator=g).to('cuda', dtype)
    w = (torch.randn(C, R, R, 1, generator=g) * 0.3).to('cuda', dtype)
    b = torch.randn(C, generator=g).to('cuda', torch.float32)
    assert dw_ok(x, w, C, (d, d))
    y_ref, dx_ref, dw_ref, db_ref, gy = _ref(x, w, b, st, p, d)
    xg, wg, bg = (t.clone().requires_grad_() for t in (x, w, b))
    y = ConvDwNHWC.apply(xg, wg, bg, (R, R), (st, st), (p, p), (d, d))
    y.backward(gy.to('cuda', dtype))
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    for name, a, r in (('y', y, y_ref), ('dx', xg.grad, dx_ref), ('dw', wg.grad, dw_ref), ('db', bg.grad, db_ref)):
        err = (a.detach().float().cpu() - r).norm() / r.norm().clamp_min(1e-12)
        assert err < tol, (name, float(err))


def test_depthwise_wgrad_is_deterministic():
    from mxnet_maintenance_amd.ops.conv_dw import ConvDwNHWC
    x = torch.randn(8, 28, 28, 64, device='cuda', dtype=torch.float16)
    w = torch.randn(64, 3, 3, 1, device='cuda', dtype=torch.float16, requires_grad=True)
    gy = torch.randn(8, 28, 28, 64, device='cuda', dtype=torch.float16)
    grads = []
    for _ in range(2):
        w.grad = None
        ConvDwNHWC.apply(x, w, None, (3, 3), (1, 1), (1, 1), (1, 1)).backward(gy)
        grads.append(w.grad.clone())
    assert torch.equal(grads[0], grads[1])


def test_mobilenet_v2_trains_through_depthwise_kernels(monkeypatch):
    import mxnet_maintenance_amd as mx
    from mxnet_maintenance_amd import gluon, autograd
    from mxnet_maintenance_amd.ops import conv_dw
    calls = []
    real = conv_dw.ConvDwNHWC.apply
    monkeypatch.setattr(conv_dw.ConvDwNHWC, 'apply', lambda *a: calls.append(1) or real(*a))
    ctx = mx.gpu(0)
    net = gluon.model_zoo.vision.get_model('mobilenetv2_1.0', classes=10)
    net.initialize(mx.init.Xavier(), ctx=ctx)
    net.cast('float16')
    tr = gluon.Trainer(net.collect_params(), 'sgd', {'learning_rate': 0.05, 'multi_precision': True})
    x = mx.nd.random.uniform(shape=(8, 3, 64, 64), ctx=ctx).astype('float16')
    y = mx.nd.array(np.arange(8) % 10, ctx=ctx)
    losses = []
    for _ in range(3):
        with autograd.record():
            loss = gluon.loss.SoftmaxCrossEntropyLoss()(net(x), y)
        loss.backward()
        tr.step(8)
        losses.append(float(loss.mean().asscalar()))
    assert len(calls) >= 17 * 3, len(calls)          # every inverted-residual block's depthwise conv
    assert np.isfinite(losses).all()
