"""SSD-ResNet50 detector (models/ssd.py) and the gfx950 MultiBoxTarget kernel.

CPU tests: model shapes/anchors vs the reference's SSD layout (example/ssd/symbol/
symbol_factory.py 'resnet50'), one training step.  GPU tests: the HIP MultiBoxTarget
(src/kernels/detection.hip) against the CPU reference implementation of the op
(src/operator/contrib/multibox_target.cc semantics), exact match.
"""
import numpy as np
import pytest
import torch

import mxnet_maintenance_amd as mx
from mxnet_maintenance_amd import nd, gluon
from mxnet_maintenance_amd.models import ssd
from mxnet_maintenance_amd.ops import detection


def _labels(B, L, classes, seed):
    g = torch.Generator().manual_seed(seed)
    lab = torch.full((B, L, 5), -1.0)
    for b in range(B):
        n = int(torch.randint(0, L + 1, (1,), generator=g))
        xy = torch.rand(n, 2, generator=g) * 0.7
        wh = 0.03 + torch.rand(n, 2, generator=g) * 0.3
        lab[b, :n, 0] = torch.randint(0, classes, (n,), generator=g).float()
        lab[b, :n, 1:3] = xy
        lab[b, :n, 3:5] = torch.clamp(xy + wh, max=1.0)
    return lab


def _anchors(h, w, sizes, ratios):
    return nd.contrib.MultiBoxPrior(nd.zeros((1, 1, h, w)), sizes=sizes, ratios=ratios).reshape((1, -1, 4))


def test_ssd_anchor_count_matches_reference_layout():
    net = ssd.ssd_512_resnet50_v1(classes=20)
    shapes = net.feature_shapes((512, 512))
    assert shapes == [(32, 32), (16, 16), (8, 8), (4, 4), (2, 2), (1, 1)]
    assert net.num_anchors == [4, 6, 6, 6, 4, 4]
    assert net.anchors((512, 512)).shape == (1, 6132, 4)


def test_ssd_forward_backward_step_cpu():
    net = ssd.SSD(classes=3, layout='NHWC', fuse=True)
    net.initialize(mx.init.Xavier(magnitude=2))
    net.hybridize()
    trainer = gluon.Trainer(net.collect_params(), 'sgd', {'learning_rate': 1e-3, 'momentum': 0.9})
    step = ssd.SSDTrainStep(net, trainer, (96, 96))
    x = nd.random.uniform(-1, 1, shape=(2, 96, 96, 3))
    lab = nd.array(_labels(2, 4, 3, 0).numpy())
    cls, loc = net(x)
    A = net.anchors((96, 96)).shape[1]
    assert cls.shape == (2, A, 4) and loc.shape == (2, A * 4)
    w0 = net.cls_preds[0].weight.data().asnumpy().copy()
    losses = [float(step(x, lab, 1).asscalar()) for _ in range(2)]
    assert all(np.isfinite(losses))
    assert not np.allclose(w0, net.cls_preds[0].weight.data().asnumpy())


def test_multibox_target_cpu_reference_semantics():
    # one gt: the greedy stage claims the best anchor even below the threshold
    anchors = nd.array([[[0.0, 0.0, 0.5, 0.5], [0.5, 0.5, 1.0, 1.0], [0.0, 0.0, 0.2, 0.2]]])
    lab = nd.array([[[1, 0.3, 0.3, 0.55, 0.55], [-1, -1, -1, -1, -1]]])
    cls = nd.zeros((1, 3, 3))
    lt, lm, ct = nd.contrib.MultiBoxTarget(anchors, lab, cls, overlap_threshold=0.9)
    assert ct.asnumpy().tolist() == [[2.0, 0.0, 0.0]]
    assert lm.asnumpy()[0, :4].tolist() == [1, 1, 1, 1] and lm.asnumpy()[0, 4:].sum() == 0


@pytest.mark.gpu
@pytest.mark.parametrize('ratio', [-1.0, 3.0])
@pytest.mark.parametrize('dtype', [torch.float32, torch.float16])
@pytest.mark.parametrize('thr', [0.5, 0.0])
def test_multibox_target_hip_matches_cpu(ratio, dtype, thr):
    from mxnet_maintenance_amd.ops import kernels
    assert kernels.available(), kernels.load_error()
    parts = [_anchors(16, 16, [.1, .141], [1, 2, .5]), _anchors(8, 8, [.2, .272], [1, 2, .5, 3, 1. / 3]),
             _anchors(4, 4, [.37, .447], [1, 2, .5, 3, 1. / 3]), _anchors(1, 1, [.88, .961], [1, 2, .5])]
    anchors = torch.cat([p._data for p in parts], 1)          # [1, A, 4]
    A = anchors.shape[1]
    B, L, C = 6, 12, 8
    lab = _labels(B, L, C - 1, 3)
    lab[0] = -1                                                 # an image without objects
    g = torch.Generator().manual_seed(5)
    cls = (torch.randn(B, C, A, generator=g) * 2).to(dtype)
    ref = detection.multibox_target(anchors, lab, cls, overlap_threshold=thr, negative_mining_ratio=ratio,
                                    minimum_negative_samples=2)
    got = detection.multibox_target(anchors.cuda(), lab.cuda(), cls.cuda(), overlap_threshold=thr,
                                    negative_mining_ratio=ratio, minimum_negative_samples=2)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got[2].cpu().numpy(), ref[2].numpy())      # cls target (incl. mined negatives)
    np.testing.assert_array_equal(got[1].cpu().numpy(), ref[1].numpy())      # loc mask
    np.testing.assert_allclose(got[0].cpu().numpy(), ref[0].numpy(), rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_ssd_train_step_gpu():
    from mxnet_maintenance_amd.ops import kernels
    assert kernels.available(), kernels.load_error()
    ctx = mx.gpu(0)
    net = ssd.ssd_512_resnet50_v1(classes=20)
    net.initialize(mx.init.Xavier(magnitude=2), ctx=ctx)
    net.cast('float16')
    net.hybridize(static_alloc=True, static_shape=True)
    trainer = gluon.Trainer(net.collect_params(), 'sgd', {'learning_rate': 1e-3, 'momentum': 0.9,
                                                          'multi_precision': True})
    step = ssd.SSDTrainStep(net, trainer, (256, 256))
    x = nd.random.uniform(-1, 1, shape=(4, 256, 256, 3), ctx=ctx).astype('float16')
    lab = nd.array(_labels(4, 8, 20, 1).numpy(), ctx=ctx)
    losses = [float(step(x, lab, 1).asscalar()) for _ in range(3)]
    assert all(np.isfinite(losses)), losses


def _loss_inputs(dev, dt, B=3, A=997, C1=21):
    import torch
    g = torch.Generator().manual_seed(5)
    cls = (torch.randn(B, A, C1, generator=g) * 2).to(dev).to(dt)
    loc = torch.randn(B, A * 4, generator=g).to(dev).to(dt)
    ct = torch.randint(-1, C1, (B, A), generator=g).float().to(dev)
    ct[0, :5] = -1
    lt = (torch.randn(B, A * 4, generator=g) * 1.5).to(dev)
    lm = (torch.rand(B, A * 4, generator=g) > 0.6).float().to(dev)
    return cls, loc, ct, lt, lm


def test_ssd_loss_op_cpu_matches_composition():
    import torch
    from mxnet_maintenance_amd.ops import detection as D
    cls, loc, ct, lt, lm = _loss_inputs('cpu', torch.float32)
    v = D.ssd_multibox_loss(cls, loc, ct, lt, lm, lambd=0.7)
    logp = torch.log_softmax(cls, -1)
    valid = ct >= 0
    ce = -(logp.gather(-1, ct.clamp(min=0).long()[..., None])[..., 0] * valid).sum() / valid.sum()
    d = (loc - lt) * lm
    sl1 = torch.nn.functional.smooth_l1_loss(d, torch.zeros_like(d), reduction='sum', beta=1.0)
    assert abs(float(v) - float(ce + 0.7 * sl1 / (ct > 0).sum())) < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', ['float16', 'bfloat16', 'float32'])
def test_ssd_loss_fused_kernel_matches_fp32_reference(dtype):
    """Fused SSD loss (detection.hip ssd_loss_*): loss and both gradients against the fp32 autograd
    composition of the same inputs."""
    import torch
    from mxnet_maintenance_amd.ops import detection as D
    dt = getattr(torch, dtype)
    cls, loc, ct, lt, lm = _loss_inputs('cuda', dt)
    cls.requires_grad_(True)
    loc.requires_grad_(True)
    v = D.ssd_multibox_loss(cls, loc, ct, lt, lm, lambd=0.7)
    (v * 1.5).backward()
    c32 = cls.detach().float().requires_grad_(True)
    l32 = loc.detach().float().requires_grad_(True)
    r = D._ssd_loss_reference(c32, l32, ct, lt, lm, 0.7)
    (r * 1.5).backward()
    assert abs(float(v) - float(r)) < 1e-3 * max(1.0, abs(float(r)))
    tol = 1e-5 if dt == torch.float32 else (2e-3 if dt == torch.float16 else 1e-2)
    for a, b in ((cls.grad, c32.grad), (loc.grad, l32.grad)):
        err = float((a.float() - b).norm() / b.norm())
        assert err < tol, err
