"""Regression tests for reference-conformance fixes (reference tests/python/unittest/test_metric.py:34,
test_loss.py:186, test_init.py:22)."""
import json

import numpy as np

import mxnet_maintenance_amd as mx
from mxnet_maintenance_amd import gluon


def test_metric_create_from_config_roundtrip():
    for m in (mx.metric.create('acc', axis=0), mx.metric.create(['acc', 'f1'])):
        cfg = m.get_config()
        assert mx.metric.create(json.dumps(cfg)).get_config() == cfg
        assert mx.metric.create(cfg).get_config() == cfg


def test_ctc_loss_label_lengths_without_pred_lengths():
    loss = gluon.loss.CTCLoss()
    out = loss(mx.nd.ones((2, 20, 4)), mx.nd.array([[2, 1, 2, 2], [3, 2, 2, 2]]), None, mx.nd.array([2, 3]))
    np.testing.assert_allclose(out.asnumpy(), [18.82820702, 16.50581741], rtol=1e-4)


def test_compose_time_default_initializers():
    data = mx.sym.Variable('data')
    mod = mx.mod.Module(mx.sym.LeakyReLU(data=data, act_type='prelu'))
    mod.bind(data_shapes=[('data', (10, 10))])
    mod.init_params()
    assert (list(mod.get_params()[0].values())[0].asnumpy() == 0.25).all()
    attrs = mx.sym.BatchNorm(data, name='bn').attr_dict()
    assert attrs['bn_moving_var']['__init__'] == '["one", {}]'
    assert attrs['bn_moving_mean']['__init__'] == '["zero", {}]'


def test_backward_twice_on_rebound_out_head():
    """A head written with out= under record() gets a fresh graph each iteration: a backward
    without retain_graph per iteration must work (only re-differentiating the SAME recording fails)."""
    import mxnet_maintenance_amd as mx
    from mxnet_maintenance_amd import autograd, nd
    x = nd.array([1.0, 2.0, 3.0])
    x.attach_grad()
    y = nd.zeros((3,))
    for _ in range(3):
        with autograd.record():
            nd.elemwise_mul(x, x, out=y)
        y.backward()
        assert (x.grad.asnumpy() == 2 * x.asnumpy()).all()
    with autograd.record():
        z = x * 3
    z.backward()
    try:
        z.backward()
    except mx.base.MXNetError:
        pass
    else:
        raise AssertionError('second backward through a released graph must fail')
