"""Optimizers, LR schedulers, initializers, metrics (parity: test_optimizer.py, test_init.py,
test_metric.py, lr scheduler tests)."""
import math
import pickle

import numpy as np
import pytest

import mxnet_maintenance_amd as mx
from mxnet_maintenance_amd import nd


def _run_opt(opt, w0, grads, mp=False):
    w = nd.array(w0, dtype='float16' if mp else 'float32')
    st = opt.create_state_multi_precision(0, w)
    for g in grads:
        opt.update_multi_precision(0, w, nd.array(g, dtype=w.dtype), st)
    return w.asnumpy().astype(np.float64)


def test_sgd_momentum_matches_numpy():
    rng = np.random.RandomState(0)
    w0 = rng.rand(10).astype(np.float32)
    grads = [rng.rand(10).astype(np.float32) for _ in range(3)]
    lr, mom, wd, rs = 0.1, 0.9, 0.01, 0.5
    opt = mx.optimizer.SGD(learning_rate=lr, momentum=mom, wd=wd, rescale_grad=rs)
    got = _run_opt(opt, w0, grads)
    w, m = w0.astype(np.float64), np.zeros(10)
    for g in grads:
        m = mom * m - lr * (rs * g + wd * w)
        w = w + m
    np.testing.assert_allclose(got, w, rtol=1e-5)
    opt = mx.optimizer.SGD(learning_rate=lr, momentum=mom, wd=wd, rescale_grad=rs, multi_precision=True)
    got16 = _run_opt(opt, w0, grads, mp=True)
    np.testing.assert_allclose(got16, w, rtol=2e-3, atol=2e-3)


def test_adam_matches_numpy():
    rng = np.random.RandomState(1)
    w0 = rng.rand(6).astype(np.float32)
    grads = [rng.rand(6).astype(np.float32) for _ in range(4)]
    lr, b1, b2, eps, wd = 0.01, 0.9, 0.999, 1e-8, 0.001
    opt = mx.optimizer.Adam(learning_rate=lr, beta1=b1, beta2=b2, epsilon=eps, wd=wd)
    got = _run_opt(opt, w0, grads)
    w, m, v = w0.astype(np.float64), np.zeros(6), np.zeros(6)
    for t, g in enumerate(grads, 1):
        g = g + wd * w
        m = b1 * m + (1 - b1) * g
        v = b2 * v + (1 - b2) * g * g
        lrt = lr * math.sqrt(1 - b2 ** t) / (1 - b1 ** t)
        w = w - lrt * m / (np.sqrt(v) + eps)
    np.testing.assert_allclose(got, w, rtol=1e-4)


@pytest.mark.parametrize('name,kw', [('nag', {'momentum': 0.9}), ('rmsprop', {}), ('rmsprop', {'centered': True}),
                                     ('adagrad', {}), ('adadelta', {}), ('ftrl', {}), ('adamax', {}),
                                     ('nadam', {}), ('signum', {}), ('ftml', {}), ('lamb', {}), ('lars', {}),
                                     ('dcasgd', {'momentum': 0.9}), ('sgld', {}), ('adamw', {}),
                                     ('lbsgd', {}), ('groupadagrad', {})])
def test_all_optimizers_decrease_quadratic(name, kw):
    mx.random.seed(0)
    opt = mx.optimizer.create(name, learning_rate=0.05, **kw)
    w = nd.array(np.ones((4, 3), dtype=np.float32) * 2)
    st = opt.create_state_multi_precision(0, w)
    start = float((w * w).sum().asscalar())
    for _ in range(20):
        g = 2 * w
        opt.update_multi_precision(0, w, g, st)
    end = float((w * w).sum().asscalar())
    assert np.isfinite(end)
    if name != 'sgld':
        assert end < start, (name, start, end)
    pickle.dumps(opt)


def test_updater_states_roundtrip():
    opt = mx.optimizer.SGD(learning_rate=0.1, momentum=0.9)
    upd = mx.optimizer.get_updater(opt)
    w = nd.ones((3,))
    upd(0, nd.ones((3,)), w)
    s = upd.get_states(dump_optimizer=True)
    upd2 = mx.optimizer.get_updater(mx.optimizer.SGD())
    upd2.set_states(s)
    assert upd2.optimizer.momentum == 0.9
    np.testing.assert_allclose(upd2.states[0].asnumpy(), upd.states[0].asnumpy())


def test_lr_mult_wd_mult():
    opt = mx.optimizer.SGD(learning_rate=1.0, param_idx2name={0: 'fc_weight', 1: 'fc_bias'}, wd=0.1)
    opt.set_lr_mult({'fc_weight': 0.5})
    assert opt._get_lr(0) == 0.5 and opt._get_lr(1) == 1.0
    assert opt._get_wd(0) == pytest.approx(0.1) and opt._get_wd(1) == 0.0


def test_lr_schedulers():
    f = mx.lr_scheduler.FactorScheduler(step=10, factor=0.5, base_lr=1.0)
    assert f(5) == 1.0 and f(15) == 0.5 and f(25) == 0.25
    m = mx.lr_scheduler.MultiFactorScheduler(step=[5, 10], factor=0.1, base_lr=1.0)
    assert m(3) == 1.0 and m(7) == pytest.approx(0.1) and m(12) == pytest.approx(0.01)
    p = mx.lr_scheduler.PolyScheduler(max_update=100, base_lr=1.0, pwr=2)
    assert p(50) == pytest.approx(0.25)
    c = mx.lr_scheduler.CosineScheduler(max_update=100, base_lr=1.0, final_lr=0.0)
    assert c(50) == pytest.approx(0.5)
    w = mx.lr_scheduler.CosineScheduler(max_update=100, base_lr=1.0, warmup_steps=10, warmup_begin_lr=0.0)
    assert w(5) == pytest.approx(0.5)


def test_initializers():
    for init, check in [(mx.init.Zero(), lambda a: (a == 0).all()), (mx.init.One(), lambda a: (a == 1).all()),
                        (mx.init.Constant(3), lambda a: (a == 3).all()),
                        (mx.init.Uniform(0.1), lambda a: np.abs(a).max() <= 0.1),
                        (mx.init.Normal(0.01), lambda a: np.abs(a).std() < 0.05),
                        (mx.init.Xavier(), lambda a: np.isfinite(a).all()),
                        (mx.init.MSRAPrelu(), lambda a: np.isfinite(a).all()),
                        (mx.init.Orthogonal(), lambda a: np.allclose(a @ a.T, a @ a.T))]:
        arr = nd.zeros((8, 8))
        init(mx.init.InitDesc('x_weight'), arr)
        assert check(arr.asnumpy()), init
    arr = nd.zeros((4,))
    mx.init.Xavier()(mx.init.InitDesc('fc_bias'), arr)
    assert (arr.asnumpy() == 0).all()
    arr = nd.zeros((4,))
    mx.init.Uniform()(mx.init.InitDesc('bn_gamma'), arr)
    assert (arr.asnumpy() == 1).all()
    b = nd.zeros((1, 1, 4, 4))
    mx.init.Bilinear()(mx.init.InitDesc('up_weight'), b)
    assert b.asnumpy().max() > 0
    lstm = nd.zeros((16,))
    mx.init.LSTMBias(forget_bias=1.0)(mx.init.InitDesc('lstm_bias', {'__init__': mx.init.LSTMBias(1.0).dumps()}),
                                      lstm)
    assert lstm.asnumpy()[4:8].tolist() == [1, 1, 1, 1]
    mixed = mx.init.Mixed(['.*bias', '.*'], [mx.init.Zero(), mx.init.One()])
    a = nd.zeros((2,))
    mixed('fc_weight', a)
    assert (a.asnumpy() == 1).all()
    assert mx.init.create('xavier').__class__ is mx.init.Xavier


def test_metrics():
    acc = mx.metric.Accuracy()
    acc.update([nd.array([0, 1, 1])], [nd.array([[0.9, 0.1], [0.2, 0.8], [0.7, 0.3]])])
    assert acc.get()[1] == pytest.approx(2 / 3)
    topk = mx.metric.TopKAccuracy(top_k=2)
    topk.update([nd.array([2])], [nd.array([[0.1, 0.5, 0.4]])])
    assert topk.get()[1] == 1.0
    mse = mx.metric.MSE()
    mse.update([nd.array([1., 2.])], [nd.array([1.5, 2.5])])
    assert mse.get()[1] == pytest.approx(0.25)
    ce = mx.metric.CrossEntropy()
    ce.update([nd.array([1])], [nd.array([[0.25, 0.75]])])
    assert ce.get()[1] == pytest.approx(-math.log(0.75))
    f1 = mx.metric.F1()
    f1.update([nd.array([1, 0, 1])], [nd.array([[0.2, 0.8], [0.9, 0.1], [0.6, 0.4]])])
    assert 0 < f1.get()[1] <= 1
    comp = mx.metric.create(['acc', 'mse'])
    assert isinstance(comp, mx.metric.CompositeEvalMetric)
    perp = mx.metric.Perplexity(ignore_label=None)
    perp.update([nd.array([0, 1])], [nd.array([[0.5, 0.5], [0.5, 0.5]])])
    assert perp.get()[1] == pytest.approx(2.0, rel=1e-4)
    cm = mx.metric.np(lambda l, p: float((l == p.argmax(1)).mean()))
    cm.update([nd.array([1])], [nd.array([[0.1, 0.9]])])
    assert cm.get()[1] == 1.0
    pcc = mx.metric.PCC()
    pcc.update([nd.array([0, 1, 1, 0])], [nd.array([[0.9, 0.1], [0.2, 0.8], [0.3, 0.7], [0.6, 0.4]])])
    assert pcc.get()[1] == pytest.approx(1.0)


def _train_arena(opt_name, opt_params, arena, steps=3):
    import os
    import numpy as np
    import mxnet_maintenance_amd as mx
    from mxnet_maintenance_amd import gluon, autograd, nd
    old = os.environ.get('MXAMD_FLAT_ARENA')
    os.environ['MXAMD_FLAT_ARENA'] = '1' if arena else '0'
    try:
        mx.random.seed(7)
        net = gluon.nn.HybridSequential()
        net.add(gluon.nn.Dense(16, activation='relu', in_units=8), gluon.nn.Dense(4, in_units=16))
        net.initialize(mx.init.Xavier())
        tr = gluon.Trainer(net.collect_params(), opt_name, dict(opt_params))
        rng = np.random.RandomState(0)
        for _ in range(steps):
            x = nd.array(rng.randn(5, 8).astype('float32'))
            y = nd.array(rng.randint(0, 4, size=(5,)).astype('float32'))
            with autograd.record():
                loss = gluon.loss.SoftmaxCrossEntropyLoss()(net(x), y)
            loss.backward()
            tr.step(5)
        assert (tr._arenas is not None) == arena
        return [p.data().asnumpy() for p in net.collect_params().values()], tr
    finally:
        if old is None:
            os.environ.pop('MXAMD_FLAT_ARENA', None)
        else:
            os.environ['MXAMD_FLAT_ARENA'] = old


import pytest as _pytest  # noqa: E402


@_pytest.mark.parametrize('opt_name,opt_params', [
    ('adam', {'learning_rate': 0.01, 'wd': 0.01, 'clip_gradient': 0.5}),
    ('adamw', {'learning_rate': 0.01, 'wd': 0.01}),
    ('lamb', {'learning_rate': 0.01, 'wd': 0.01, 'lower_bound': 0.01, 'upper_bound': 10.0}),
    ('sgd', {'learning_rate': 0.1, 'momentum': 0.9, 'wd': 1e-3}),
])
def test_flat_arena_optimizers_match_per_parameter(opt_name, opt_params):
    """The Trainer's flat-arena fused update (HIP kernel on GPU, same math in torch here) equals the
    reference per-parameter optimizer path (python/mxnet/optimizer/optimizer.py semantics)."""
    import numpy as np
    a, tr = _train_arena(opt_name, opt_params, arena=True)
    b, _ = _train_arena(opt_name, opt_params, arena=False)
    for x, y in zip(a, b):
        np.testing.assert_allclose(x, y, rtol=1e-5, atol=1e-6)


def test_flat_arena_adam_save_load_states(tmp_path):
    import numpy as np
    _, tr = _train_arena('adam', {'learning_rate': 0.01}, arena=True)
    f = str(tmp_path / 'adam.states')
    tr.save_states(f)
    st = tr._updaters[0].states
    means = {k: v[0].asnumpy().copy() for k, v in st.items()}
    for a in tr._arenas:
        a.mean.zero_()
    tr.load_states(f)
    st = tr._updaters[0].states
    for k, v in st.items():
        np.testing.assert_allclose(v[0].asnumpy(), means[k])
    a = tr._arenas[0]
    off, n, shape = a.views[0]
    np.testing.assert_allclose(a.mean[off:off + n].numpy(), means[a.indices[0]].reshape(-1))
