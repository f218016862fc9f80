"""gluon.GraphStep: a whole training step (forward, backward, fused optimizer update) captured in one
HIP graph must train exactly like the eager step; captured dropout must draw fresh masks per replay."""
import numpy as np
import pytest
import torch

import mxnet_maintenance_amd as mx
from mxnet_maintenance_amd import autograd, gluon, nd


def _net(seed, dropout=0.0):
    mx.random.seed(seed)
    net = gluon.nn.HybridSequential()
    net.add(gluon.nn.Dense(256, activation='relu', in_units=128))
    if dropout:
        net.add(gluon.nn.Dropout(dropout))
    net.add(gluon.nn.Dense(64, in_units=256))
    net.initialize(mx.init.Xavier(), ctx=mx.gpu(0))
    net.hybridize(static_alloc=True, static_shape=True)
    return net


def _train(optimizer, opt_params, graph, steps=8, dtype='float32'):
    net = _net(7)
    if dtype != 'float32':
        net.cast(dtype)
    sched = mx.lr_scheduler.FactorScheduler(step=2, factor=0.5, base_lr=opt_params['learning_rate'])
    trainer = gluon.Trainer(net.collect_params(), optimizer, dict(opt_params, lr_scheduler=sched))
    loss_fn = gluon.loss.L2Loss()
    rs = np.random.RandomState(0)
    xs = [nd.array(rs.randn(32, 128), ctx=mx.gpu(0), dtype=dtype) for _ in range(steps)]
    ys = [nd.array(rs.randn(32, 64), ctx=mx.gpu(0), dtype=dtype) for _ in range(steps)]

    def step(x, y):
        with autograd.record():
            loss = loss_fn(net(x), y)
        loss.backward()
        trainer.step(32)
        return loss

    run = gluon.GraphStep(step, trainer, warmup=2) if graph else step
    losses = [float(run(x, y).mean().asscalar()) for x, y in zip(xs, ys)]
    if graph:
        assert run.captured
    return losses, [p.data().asnumpy().astype(np.float32) for p in net.collect_params().values()]


@pytest.mark.gpu
@pytest.mark.parametrize('optimizer,params', [
    ('sgd', {'learning_rate': 0.05, 'momentum': 0.9, 'wd': 1e-4}),
    ('adam', {'learning_rate': 1e-3, 'wd': 1e-4}),
    ('lamb', {'learning_rate': 1e-3, 'wd': 0.01}),
])
def test_graph_step_matches_eager(optimizer, params):
    le, we = _train(optimizer, params, graph=False)
    lg, wg = _train(optimizer, params, graph=True)
    np.testing.assert_allclose(lg, le, rtol=1e-4, atol=1e-5)
    for a, b in zip(wg, we):
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize('optimizer', ['adam', 'lamb', 'sgd'])
def test_graph_step_multi_precision_bf16(optimizer):
    params = {'learning_rate': 1e-3, 'multi_precision': True}
    le, we = _train(optimizer, params, graph=False, dtype='bfloat16')
    lg, wg = _train(optimizer, params, graph=True, dtype='bfloat16')
    np.testing.assert_allclose(lg, le, rtol=2e-2, atol=1e-3)
    for a, b in zip(wg, we):
        np.testing.assert_allclose(a, b, rtol=2e-2, atol=2e-3)


@pytest.mark.gpu
def test_graph_step_dropout_fresh_masks():
    net = _net(3, dropout=0.5)
    net.cast('bfloat16')
    x = nd.ones((64, 128), ctx=mx.gpu(0), dtype='bfloat16')

    def fwd(x):
        with autograd.train_mode():
            return net(x)

    run = gluon.GraphStep(fwd, None, warmup=1)
    run(x)
    outs = [run(x).asnumpy().astype(np.float32).copy() for _ in range(3)]
    assert run.captured
    assert not np.allclose(outs[0], outs[1]) and not np.allclose(outs[1], outs[2])


@pytest.mark.gpu
def test_graph_step_rejects_shape_change():
    net = _net(1)

    def fwd(x):
        return net(x)

    run = gluon.GraphStep(fwd, None, warmup=1)
    x = nd.ones((8, 128), ctx=mx.gpu(0))
    run(x)
    run(x)
    with pytest.raises(ValueError):
        run(nd.ones((4, 128), ctx=mx.gpu(0)))


def test_graph_step_eager_warmup_on_cpu():
    # the warm-up calls run eagerly anywhere; capture needs a HIP device
    calls = []
    run = gluon.GraphStep(lambda x: calls.append(1) or x * 2, None, warmup=2)
    x = nd.ones((2, 2))
    assert (run(x).asnumpy() == 2).all()
    run(x)
    assert len(calls) == 2
    if not torch.cuda.is_available():
        with pytest.raises(RuntimeError):
            run(x)
