"""gluon.contrib (parity: tests/python/unittest/test_gluon_contrib.py, test_gluon_estimator.py,
test_gluon_event_handler.py, tests/python/gpu/test_gluon_contrib sync-BN)."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as tmp
import torch.nn.functional as F

import mxnet_maintenance_amd as mx
from mxnet_maintenance_amd import nd, gluon, autograd
from mxnet_maintenance_amd.gluon.contrib import nn as cnn, cnn as dconv, rnn as crnn, estimator as est
from mxnet_maintenance_amd.ops import contrib_ops


def test_concurrent_identity_pixelshuffle():
    hc = cnn.HybridConcurrent(axis=1)
    hc.add(gluon.nn.Dense(3, in_units=6), cnn.Identity())
    hc.initialize()
    assert hc(nd.ones((2, 6))).shape == (2, 9)
    c = cnn.Concurrent(axis=1)
    c.add(gluon.nn.Dense(2, in_units=6), gluon.nn.Dense(1, in_units=6))
    c.initialize()
    assert c(nd.ones((2, 6))).shape == (2, 3)
    x = nd.arange(2 * 8 * 3 * 3).reshape((2, 8, 3, 3))
    y = cnn.PixelShuffle2D(2)(x)
    ref = F.pixel_shuffle(torch.as_tensor(x.asnumpy()), 2).numpy()
    np.testing.assert_array_equal(y.asnumpy(), ref)
    assert cnn.PixelShuffle1D(3)(nd.ones((1, 6, 4))).shape == (1, 2, 12)
    assert cnn.PixelShuffle3D(2)(nd.ones((1, 16, 2, 2, 2))).shape == (1, 2, 4, 4, 4)


def test_deformable_conv_zero_offset_is_conv():
    x = torch.randn(2, 4, 7, 7, dtype=torch.float64)
    w = torch.randn(6, 4, 3, 3, dtype=torch.float64)
    off = torch.zeros(2, 18, 7, 7, dtype=torch.float64)
    y = contrib_ops.deformable_convolution(x, off, w, None, kernel=(3, 3), pad=(1, 1), num_filter=6, no_bias=True)
    torch.testing.assert_close(y, F.conv2d(x, w, padding=1))
    off[:, 1::2] = 1.0   # every tap sampled one column to the right
    y2 = contrib_ops.deformable_convolution(x, off, w, None, kernel=(3, 3), pad=(1, 1), num_filter=6, no_bias=True)
    torch.testing.assert_close(y2, F.conv2d(F.pad(x, (0, 2, 1, 1)), w))
    m = torch.full((2, 9, 7, 7), 0.5, dtype=torch.float64)
    y3 = contrib_ops.modulated_deformable_convolution(x, torch.zeros_like(off), m, w, None, kernel=(3, 3),
                                                      pad=(1, 1), num_filter=6, no_bias=True)
    torch.testing.assert_close(y3, 0.5 * F.conv2d(x, w, padding=1))
    blk = dconv.DeformableConvolution(4, kernel_size=3, padding=1, in_channels=3)
    blk.initialize()
    xx = nd.random.uniform(shape=(1, 3, 5, 5))
    xx.attach_grad()
    with autograd.record():
        out = blk(xx)
    out.backward()
    assert out.shape == (1, 4, 5, 5) and xx.grad.shape == xx.shape
    m2 = dconv.ModulatedDeformableConvolution(4, kernel_size=3, padding=1, in_channels=3)
    m2.initialize()
    assert m2(xx).shape == (1, 4, 5, 5)


def test_conv_rnn_cells():
    c = crnn.Conv2DLSTMCell((3, 8, 8), 4, 3, 3, i2h_pad=1)
    c.initialize()
    o, s = c.unroll(2, nd.ones((2, 2, 3, 8, 8)), merge_outputs=True)
    assert o.shape == (2, 2, 4, 8, 8) and s[0].shape == (2, 4, 8, 8) and len(s) == 2
    g = crnn.Conv1DGRUCell((3, 10), 5, 3, 3)
    g.initialize()
    out, _ = g(nd.ones((2, 3, 10)), g.begin_state(2))
    assert out.shape == (2, 5, 8)
    r = crnn.Conv3DRNNCell((2, 4, 4, 4), 3, 1, 3)
    r.initialize()
    out, _ = r(nd.ones((1, 2, 4, 4, 4)), r.begin_state(1))
    assert out.shape == (1, 3, 4, 4, 4)


def test_estimator_fit_with_handlers():
    X = np.random.rand(64, 6).astype('float32')
    y = (X.sum(1) > 3).astype('float32')
    dl = gluon.data.DataLoader(gluon.data.ArrayDataset(X, y), batch_size=16)
    net = gluon.nn.Dense(2, in_units=6)
    net.initialize()
    tr = gluon.Trainer(net.collect_params(), 'sgd', {'learning_rate': 0.5})
    acc = mx.metric.Accuracy()
    e = est.Estimator(net, gluon.loss.SoftmaxCrossEntropyLoss(), train_metrics=acc, trainer=tr, context=mx.cpu())
    with tempfile.TemporaryDirectory() as d:
        ck = est.CheckpointHandler(d, model_prefix='m', monitor=e.train_metrics[0], save_best=True)
        es = est.EarlyStoppingHandler(monitor=e.train_metrics[0], patience=100)
        e.fit(dl, val_data=dl, epochs=4, event_handlers=[ck, es])
        files = os.listdir(d)
        assert any(f.startswith('m-epoch3') for f in files) and 'm-best.params' in files
    name, value = e.train_metrics[0].get()
    assert 'training' in name and value > 0.5
    e.evaluate(dl)
    assert 'validation' in e.val_metrics[0].get()[0]
    e2 = est.Estimator(net, gluon.loss.SoftmaxCrossEntropyLoss(), trainer=tr, context=mx.cpu())
    e2.fit(dl, batches=3)


def test_sync_batchnorm_single_process_matches_batchnorm():
    x = nd.random.uniform(shape=(4, 3, 2, 2))
    s = cnn.SyncBatchNorm(in_channels=3)
    s.initialize()
    b = gluon.nn.BatchNorm(in_channels=3)
    b.initialize()
    with autograd.record():
        ys = s(x)
        yb = b(x)
    np.testing.assert_allclose(ys.asnumpy(), yb.asnumpy(), rtol=1e-4, atol=1e-4)


def _sbn_worker(rank, world, port, q):
    os.environ.update({'RANK': str(rank), 'WORLD_SIZE': str(world), 'MASTER_ADDR': '127.0.0.1',
                       'MASTER_PORT': str(port)})
    import torch.distributed as dist
    try:
        dist.init_process_group('gloo', rank=rank, world_size=world)
        import mxnet_maintenance_amd as mx
        from mxnet_maintenance_amd import nd, autograd
        from mxnet_maintenance_amd.gluon.contrib import nn as cnn
        rng = np.random.RandomState(0)
        full = rng.rand(8, 3, 2, 2).astype('float32')
        part = nd.array(full[rank * 4:(rank + 1) * 4])
        s = cnn.SyncBatchNorm(in_channels=3)
        s.initialize()
        with autograd.record():
            y = s(part)
        mean = s.running_mean.data().asnumpy()
        q.put((rank, y.asnumpy().tolist(), mean.tolist()))
    except Exception:
        import traceback
        q.put((rank, 'ERR', traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_sync_batchnorm_two_processes_uses_global_stats():
    ctx = tmp.get_context('spawn')
    q = ctx.Queue()
    port = 29500 + os.getpid() % 400
    ps = [ctx.Process(target=_sbn_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        item = q.get(timeout=240)
        res[item[0]] = item
    for p in ps:
        p.join(timeout=60)
    for r in range(2):
        assert res[r][1] != 'ERR', res[r][2]
    rng = np.random.RandomState(0)
    full = rng.rand(8, 3, 2, 2).astype('float32')
    mean = full.mean(axis=(0, 2, 3))
    var = full.var(axis=(0, 2, 3))
    ref = (full - mean.reshape(1, 3, 1, 1)) / np.sqrt(var.reshape(1, 3, 1, 1) + 1e-5)
    got = np.concatenate([np.array(res[0][1]), np.array(res[1][1])])
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(res[0][2], 0.1 * mean, rtol=1e-4)
