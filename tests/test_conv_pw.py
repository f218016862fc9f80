"""Streaming 1x1 convolution (src/kernels/conv_pw.hip) vs fp32 PyTorch: outputs and the fused BatchNorm
statistics partials."""
import numpy as np
import pytest
import torch

from mxnet_maintenance_amd.ops import kernel_fns as KF

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('kin,nout,M,dt', [(64, 256, 3136 * 2 + 40, torch.float16), (256, 64, 5000, torch.bfloat16),
                                           (64, 64, 777, torch.float16), (512, 128, 1568, torch.float16),
                                           (256, 128, 2049, torch.bfloat16), (128, 128, 100, torch.float16),
                                           (128, 256, 3000, torch.bfloat16), (64, 128, 1000, torch.float16),
                                           (128, 512, 1600, torch.float16), (256, 512, 900, torch.bfloat16),
                                           (512, 256, 2500, torch.float16), (256, 1024, 1700, torch.float16),
                                           (1024, 256, 1000, torch.bfloat16), (512, 2048, 300, torch.float16)])
def test_conv_pw_matches_fp32(kin, nout, M, dt):
    dev = torch.device('cuda', 0)
    assert KF.pw_ok(torch.empty(1, kin, dtype=dt, device=dev), kin, nout)
    g = torch.Generator().manual_seed(kin + nout)
    x = (torch.rand(M, kin, generator=g) * 2 - 1).to(dev, dt).view(1, 1, M, kin)
    w = ((torch.rand(nout, kin, generator=g) * 2 - 1) / kin ** 0.5).to(dev, dt)
    y = KF.conv_pw(x, w, bn_stats=True)
    ref = x.float().reshape(M, kin) @ w.float().t()
    err = float((y.float().reshape(M, nout) - ref).norm() / ref.norm())
    assert err < 1e-2, err
    part, nparts = y._mxamd_bn_part
    p = part.view(2, nout, nparts).sum(-1)
    yr = y.float().reshape(M, nout)
    assert float((p[0] - yr.sum(0)).abs().max()) < 1e-2 * float(yr.abs().sum(0).max() + 1)
    assert float((p[1] - (yr * yr).sum(0)).abs().max()) < 1e-3 * float((yr * yr).sum(0).max() + 1)
    # no statistics requested: same output
    y2 = KF.conv_pw(x, w)
    assert torch.equal(y2, y)


@pytest.mark.parametrize('kin,nout,M,dt', [(64, 256, 3136 * 3 + 17, torch.float16), (128, 256, 4000, torch.bfloat16),
                                           (256, 64, 2001, torch.float16), (64, 64, 65, torch.bfloat16),
                                           (512, 128, 3000, torch.float16), (128, 512, 3136 + 5, torch.float16),
                                           (256, 512, 1000, torch.bfloat16), (256, 1024, 1568 + 3, torch.float16),
                                           (512, 2048, 200, torch.bfloat16)])
def test_conv_pw_addend_epilogue(kin, nout, M, dt):
    """y = x . w^T + addend (the identity-shortcut gradient of a tee dgrad) in the epilogue."""
    dev = torch.device('cuda', 0)
    g = torch.Generator().manual_seed(3 * kin + nout)
    x = (torch.rand(M, kin, generator=g) * 2 - 1).to(dev, dt).view(1, 1, M, kin)
    w = ((torch.rand(nout, kin, generator=g) * 2 - 1) / kin ** 0.5).to(dev, dt)
    a = (torch.rand(M, nout, generator=g) * 2 - 1).to(dev, dt).view(1, 1, M, nout)
    y = KF.conv_pw(x, w, addend=a)
    ref = x.float().reshape(M, kin) @ w.float().t() + a.float().reshape(M, nout)
    err = float((y.float().reshape(M, nout) - ref).norm() / ref.norm())
    assert err < 1e-2, err
    # with statistics as well (they cover the summed output)
    y2 = KF.conv_pw(x, w, bn_stats=True, addend=a)
    assert torch.equal(y2, y)
    part, nparts = y2._mxamd_bn_part
    yr = y.float().reshape(M, nout)
    assert float((part.view(2, nout, nparts).sum(-1)[0] - yr.sum(0)).abs().max()) < \
        1e-2 * float(yr.abs().sum(0).max() + 1)


def test_tee_dgrad_pw_candidate_matches_mm():
    """The tee dgrad's streaming-kernel candidate equals dY . W + dShortcut."""
    dev = torch.device('cuda', 0)
    dt = torch.float16
    N, H, W, C, K = 2, 28, 28, 256, 64
    gy = (torch.randn(N, H, W, K, device=dev) * 0.1).to(dt)
    gpass = (torch.randn(N, H, W, C, device=dev) * 0.1).to(dt)
    w = (torch.randn(K, 1, 1, C, device=dev) / C ** 0.5).to(dt)
    y = KF.conv_pw(gy, w.reshape(K, C).t(), addend=gpass)
    ref = gy.float().reshape(-1, K) @ w.float().reshape(K, C) + gpass.float().reshape(-1, C)
    assert float((y.float().reshape(-1, C) - ref).abs().max()) < 2e-2


@pytest.mark.parametrize('kin,nout,M,dt', [(64, 256, 3136 + 40, torch.float16), (256, 64, 2000, torch.bfloat16),
                                           (64, 64, 777, torch.float16), (512, 128, 1568, torch.float16),
                                           (128, 512, 1600, torch.float16), (512, 256, 900, torch.bfloat16),
                                           (256, 1024, 1700, torch.float16), (512, 2048, 300, torch.float16),
                                           (1024, 256, 500, torch.bfloat16)])
@pytest.mark.parametrize('add', [False, True])
def test_conv_pw_transposed_weight_view(kin, nout, M, dt, add):
    """A dgrad passes w2 as the transpose of a contiguous [Cin][Cout] weight; the kernel transposes it
    while loading its resident fragments and must equal the run on the materialised transpose."""
    dev = torch.device('cuda', 0)
    g = torch.Generator().manual_seed(5 * kin + nout)
    x = (torch.rand(M, kin, generator=g) * 2 - 1).to(dev, dt).view(1, 1, M, kin)
    wk = ((torch.rand(kin, nout, generator=g) * 2 - 1) / kin ** 0.5).to(dev, dt)   # [Cin][Cout]
    a = (torch.rand(M, nout, generator=g) * 2 - 1).to(dev, dt).view(1, 1, M, nout) if add else None
    y_view = KF.conv_pw(x, wk.t(), addend=a)
    y_copy = KF.conv_pw(x, wk.t().contiguous(), addend=a)
    assert torch.equal(y_view, y_copy)
    ref = x.float().reshape(M, kin) @ wk.float() + (a.float().reshape(M, nout) if add else 0)
    err = float((y_view.float().reshape(M, nout) - ref).norm() / ref.norm())
    assert err < 1e-2, err


def _bnb_ref(y, z, mean, scale=None, shift=None, mask=None):
    yf, zf = y.float().reshape(-1, y.shape[-1]), z.float().reshape(-1, z.shape[-1])
    if mask is not None:
        bits = ((mask.view(-1, 1).int() >> torch.arange(8, device=y.device)) & 1).reshape(yf.shape)
        keep = bits.bool()
    else:
        keep = zf * scale + shift > 0
    dz = torch.where(keep, yf, torch.zeros_like(yf))
    return dz.sum(0), (dz * (zf - mean)).sum(0)


@pytest.mark.parametrize('kin,nout,M,dt', [(512, 128, 3000, torch.float16), (256, 64, 2001, torch.bfloat16),
                                           (512, 256, 1568, torch.float16), (128, 128, 777, torch.float16)])
def test_conv_pw_bn_backward_stats_from_z(kin, nout, M, dt):
    """dgrad feeding BN+ReLU: the epilogue's (sum dz, sum dz*(z-mean)) partials, the ReLU mask recomputed
    from the BN input z and the forward's scale/shift; the output itself is unchanged."""
    dev = torch.device('cuda', 0)
    g = torch.Generator().manual_seed(7 * kin + nout)
    x = (torch.rand(M, kin, generator=g) * 2 - 1).to(dev, dt).view(1, 1, M, kin)
    wk = ((torch.rand(kin, nout, generator=g) * 2 - 1) / kin ** 0.5).to(dev, dt)
    z = (torch.rand(M, nout, generator=g) * 2 - 1).to(dev, dt).view(1, 1, M, nout)
    mean = (torch.rand(nout, generator=g) * 0.2 - 0.1).to(dev)
    scale = (torch.rand(nout, generator=g) + 0.5).to(dev)
    shift = (torch.rand(nout, generator=g) - 0.5).to(dev)
    assert KF.pw_bnb_ok(kin, nout, False, (z, mean, scale, shift, None, 2, None))
    y = KF.conv_pw(x, wk.t(), bn_bwd=(z, mean, scale, shift, None, 2, 'tok'))
    assert torch.equal(y, KF.conv_pw(x, wk.t()))
    part, nparts, tok, ver = y._mxamd_bn_bwd
    assert tok == 'tok' and ver == y._version
    s1, s2 = part.view(2, nout, nparts).sum(-1)
    r1, r2 = _bnb_ref(y, z, mean, scale, shift)
    torch.testing.assert_close(s1, r1, rtol=1e-3, atol=1e-2 * float(r1.abs().max() + 1))
    torch.testing.assert_close(s2, r2, rtol=1e-3, atol=1e-2 * float(r2.abs().max() + 1))


@pytest.mark.parametrize('kin,nout,M,dt', [(128, 256, 3136 + 5, torch.float16), (128, 512, 1600, torch.bfloat16),
                                           (256, 512, 1000, torch.float16), (256, 1024, 1568 + 3, torch.float16),
                                           (512, 2048, 200, torch.bfloat16)])
def test_conv_pw_tee_bn_backward_stats_mask(kin, nout, M, dt):
    """Tee dgrad feeding the previous block's residual tail: y = conv + addend, with the tail's backward
    statistics from its 1-bit forward ReLU mask."""
    dev = torch.device('cuda', 0)
    g = torch.Generator().manual_seed(11 * kin + nout)
    x = (torch.rand(M, kin, generator=g) * 2 - 1).to(dev, dt).view(1, 1, M, kin)
    wk = ((torch.rand(kin, nout, generator=g) * 2 - 1) / kin ** 0.5).to(dev, dt)
    a = (torch.rand(M, nout, generator=g) * 2 - 1).to(dev, dt).view(1, 1, M, nout)
    z = (torch.rand(M, nout, generator=g) * 2 - 1).to(dev, dt).view(1, 1, M, nout)
    mask = torch.randint(0, 256, (M * nout // 8,), generator=g, dtype=torch.int32).to(torch.uint8).to(dev)
    mean = (torch.rand(nout, generator=g) * 0.2 - 0.1).to(dev)
    src = (z, mean, None, None, mask, 3, 'tok')
    assert KF.pw_bnb_ok(kin, nout, True, src)
    y = KF.conv_pw(x, wk.t(), addend=a, bn_bwd=src)
    assert torch.equal(y, KF.conv_pw(x, wk.t(), addend=a))
    part, nparts, _tok, _ver = y._mxamd_bn_bwd
    s1, s2 = part.view(2, nout, nparts).sum(-1)
    r1, r2 = _bnb_ref(y, z, mean, mask=mask)
    torch.testing.assert_close(s1, r1, rtol=1e-3, atol=1e-2 * float(r1.abs().max() + 1))
    torch.testing.assert_close(s2, r2, rtol=1e-3, atol=1e-2 * float(r2.abs().max() + 1))


@pytest.mark.parametrize('kin,nout,M,dt', [(128, 256, 3136 + 5, torch.float16), (256, 1024, 1568 + 3, torch.float16),
                                           (512, 2048, 200, torch.bfloat16)])
def test_conv_pw_tee_masked_addend(kin, nout, M, dt):
    """The tee dgrad's addend as dy * (a residual tail's ReLU bits), the product never materialised: output and
    the BN-backward statistics equal the materialised-addend launch bit for bit."""
    dev = torch.device('cuda', 0)
    g = torch.Generator().manual_seed(7 * kin + nout)
    x = (torch.rand(M, kin, generator=g) * 2 - 1).to(dev, dt).view(1, 1, M, kin)
    wk = ((torch.rand(kin, nout, generator=g) * 2 - 1) / kin ** 0.5).to(dev, dt)
    dy = (torch.rand(M, nout, generator=g) * 2 - 1).to(dev, dt).view(1, 1, M, nout)
    amask = torch.randint(0, 256, (M * nout // 8,), generator=g, dtype=torch.int32).to(torch.uint8).to(dev)
    z = (torch.rand(M, nout, generator=g) * 2 - 1).to(dev, dt).view(1, 1, M, nout)
    mask = torch.randint(0, 256, (M * nout // 8,), generator=g, dtype=torch.int32).to(torch.uint8).to(dev)
    mean = (torch.rand(nout, generator=g) * 0.2 - 0.1).to(dev)
    src = (z, mean, None, None, mask, 3, 'tok')
    dz = KF._materialize_dz(dy, amask)
    ref = KF.conv_pw(x, wk.t(), addend=dz, bn_bwd=src)
    y = KF.conv_pw(x, wk.t(), addend=dy, bn_bwd=src, addend_mask=amask)
    assert torch.equal(y, ref)
    assert torch.equal(y._mxamd_bn_bwd[0], ref._mxamd_bn_bwd[0])


def test_resnet_lazy_shortcut_gradient_matches_materialised():
    """ResNet-50 (fused NHWC): with the tee data gradients on the masked-addend streaming kernel, the
    residual tails hand their shortcut gradient over unmaterialised; every parameter gradient equals
    the materialised run's."""
    import mxnet_maintenance_amd as mx
    from mxnet_maintenance_amd import autograd, gluon, nd
    ctx = mx.gpu(0)
    mx.random.seed(3)
    net = gluon.model_zoo.vision.get_model('resnet50_v1b', layout='NHWC', fuse=True, classes=10)
    net.initialize(mx.init.Xavier(), ctx=ctx)
    net.cast('float16')
    net.hybridize(static_alloc=True, static_shape=True)
    x = nd.random.uniform(-1, 1, shape=(8, 64, 64, 3), ctx=ctx).astype('float16')
    y = nd.array([1, 2, 3, 4, 5, 6, 7, 8], ctx=ctx)
    loss_fn = gluon.loss.SoftmaxCrossEntropyLoss()
    params = [p for p in net.collect_params().values() if p.grad_req != 'null']

    def grads():
        with autograd.record():
            loss = loss_fn(net(x), y)
        loss.backward()
        return [p.grad(ctx).astype('float32').asnumpy().copy() for p in params]
    grads()                                   # autotune every shape
    forced = 0
    for k in list(KF._ALGO):
        if (k[0] == 'teedgrad' and 'bnbwd' in k
                and KF.pw_ok(torch.empty(1, 1, 8, k[2][0], dtype=k[3], device='cuda'), k[2][0], k[2][3])
                and KF._K.lib().conv_pw_stream_bnb_ok(k[2][0], k[2][3], 1, 3)):
            KF._ALGO[k] = 'pw+bn'
            forced += 1
    assert forced > 0
    KF._LAZY_DZ[0] = False
    ref = grads()
    ref2 = grads()
    KF._LAZY_DZ[0] = True
    used = KF._LAZY_USED[0]
    got = grads()
    assert KF._LAZY_USED[0] > used
    # fp16 forward kernels picked by the autotuner (split-K reductions) are not bitwise reproducible, so
    # compare in relative norm against the materialised path's own run-to-run spread; a wrong shortcut
    # gradient (e.g. the mask not applied) is off by tens of percent
    for a, b, c in zip(got, ref, ref2):
        nb = float(np.linalg.norm(b)) + 1e-6
        noise = float(np.linalg.norm(c - b)) / nb
        assert float(np.linalg.norm(a - b)) / nb <= max(3 * noise, 1e-2)


@pytest.mark.parametrize('second_consumer', [False, True])
def test_projection_shortcut_lazy_gradient(second_consumer):
    """relu(BN1(x) + BN2(s)) with BN2 the projection shortcut: the tail hands BN2 its dy and ReLU mask
    instead of d_addend; with a second consumer of BN2's output autograd sums the gradients and BN2
    corrects the sum. Gradients equal the materialised path's."""
    from mxnet_maintenance_amd.ops import hip_ops as H
    dev = torch.device('cuda', 0)
    torch.manual_seed(5)
    N, Hh, W, C = 4, 14, 14, 256
    x0 = torch.randn(N, Hh, W, C, device=dev).half()
    s0 = torch.randn(N, Hh, W, C, device=dev).half()
    wl = torch.randn(N, Hh, W, C, device=dev)
    w2 = torch.randn(N, Hh, W, C, device=dev)

    def run(lazy):
        KF._LAZY_DZ[0] = lazy
        x = x0.clone().requires_grad_()
        s = s0.clone().requires_grad_()
        g1 = (torch.rand(C, device=dev) + 0.5).requires_grad_()
        b1 = torch.zeros(C, device=dev).requires_grad_()
        g2 = (torch.rand(C, device=dev) + 0.5).requires_grad_()
        b2 = torch.zeros(C, device=dev).requires_grad_()
        torch.manual_seed(9)
        g1.data.uniform_(0.5, 1.5)
        g2.data.uniform_(0.5, 1.5)
        rm1, rv1, rm2, rv2 = (torch.zeros(C, device=dev), torch.ones(C, device=dev),
                              torch.zeros(C, device=dev), torch.ones(C, device=dev))
        sc = H.batch_norm(s, g2, b2, rm2, rv2, 1e-5, 0.9, False, True, 3, None)[0]
        out = H.batch_norm(x, g1, b1, rm1, rv1, 1e-5, 0.9, False, True, 3, 'relu', addend=sc)[0]
        loss = (out.float() * wl).sum()
        if second_consumer:
            loss = loss + (sc.float() * w2).sum()
        loss.backward()
        KF._LAZY_DZ[0] = True
        return [t.grad.float() for t in (x, s, g1, b1, g2, b2)]
    ref = run(False)
    got = run(True)
    for a, b in zip(got, ref):
        torch.testing.assert_close(a, b, rtol=2e-3, atol=2e-3 * float(b.abs().max() + 1e-6))
