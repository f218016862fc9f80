"""Reference semantics fixed in round 4 (each mirrors a reference unittest that failed before):
numpy-mode symbols (basic indexing, bool comparisons, mx.np methods), negative-step / mixed
assignment, np-shape file semantics, sparse views and contexts, multinomial log-probability
gradients, recorded symbols of hybridized blocks."""

import numpy as onp
import pytest

import mxnet_maintenance_amd as mx
from mxnet_maintenance_amd import autograd, gluon, nd, np, npx


class _Slice(gluon.HybridBlock):
    def hybrid_forward(self, F, x, y):
        return x[:, -1, 1:3] + y[()][1, 1:3], (x > 0.5), x.max(axis=(), keepdims=True)


def test_numpy_symbol_indexing_comparisons_and_methods():
    npx.set_np()
    try:
        x = np.array(onp.random.RandomState(0).rand(2, 3, 4).astype('float32'))
        y = np.array(onp.arange(8, dtype='float32').reshape(2, 4))
        ref = _Slice()(x, y)
        net = _Slice()
        net.hybridize()
        out = net(x, y)
        for a, b in zip(out, ref):
            assert a.shape == b.shape and a.dtype == b.dtype
            onp.testing.assert_allclose(a.asnumpy().astype('float64'), b.asnumpy().astype('float64'))
        assert out[1].dtype == onp.bool_
        assert out[2].shape == (2, 3, 4)            # axis=() reduces nothing
    finally:
        npx.reset_np()


def test_negative_step_and_mixed_index_assignment():
    a = onp.arange(2 * 3 * 4, dtype='float32').reshape(2, 3, 4)
    x = np.array(a)
    x[:, ::-1, 1] = np.array([10., 20., 30.])
    a[:, ::-1, 1] = [10., 20., 30.]
    x[1, [2], onp.array([[3]]), ...] = 7.
    a[1, [2], onp.array([[3]]), ...] = 7.
    onp.testing.assert_array_equal(x.asnumpy(), a)


def test_np_shape_semantics_of_saved_files(tmp_path):
    f = str(tmp_path / 'a.nd')
    with mx.np_shape(True):
        nd.save(f, [nd.zeros((2, 0))])
    with pytest.raises(mx.base.MXNetError):
        nd.load(f)                                   # saved under numpy shape semantics
    with mx.np_shape(True):
        assert nd.load(f)[0].shape == (2, 0)


def test_row_sparse_index_views_and_cpu_contexts():
    g = nd.sparse.row_sparse_array((onp.ones((2, 3), 'float32'), [0, 2]), shape=(3, 3))
    g[0] = g[0] * 0.5
    onp.testing.assert_array_equal(g[0].asnumpy(), [0.5, 0.5, 0.5])
    c = nd.sparse.csr_matrix(onp.eye(3, dtype='float32'), ctx=mx.cpu(1))
    assert c.context == mx.cpu(1) and c.copy().context == mx.cpu(1)
    assert nd.zeros((2, 2), ctx=mx.Context('cpu_shared', 0)).context == mx.Context('cpu_shared', 0)


def test_multinomial_log_probability_gradient():
    x = nd.array([[0.1, 0.2, 0.3, 0.4]])
    x.attach_grad()
    with autograd.record():
        y, lp = nd.random.multinomial(x, shape=50, get_prob=True)
        lp.sum().backward()
    ys = y.asnumpy().astype(int)[0]
    onp.testing.assert_allclose(lp.asnumpy()[0], onp.log(x.asnumpy()[0][ys]), rtol=1e-5)
    expect = onp.bincount(ys, minlength=4) / x.asnumpy()[0]
    onp.testing.assert_allclose(x.grad.asnumpy()[0], expect, rtol=1e-4)


def test_hybridized_output_symbol_respects_inline_limit():
    import json
    net = gluon.nn.HybridSequential()
    with net.name_scope():
        for _ in range(3):
            net.add(gluon.nn.Dense(4))
    net.initialize()
    counts = []
    for limit in (3, 0):
        net.hybridize(inline_limit=limit)
        with autograd.record():
            y = net(nd.zeros((1, 4)))
        counts.append(len(json.loads(autograd.get_symbol(y).tojson())['nodes']))
        y.backward()
    assert counts[0] == counts[1] + 2                # 3 FullyConnected nodes vs one _CachedOp node


def test_operator_index_errors_are_index_errors():
    with pytest.raises(IndexError):
        nd.gather_nd(nd.array([[0, 1, 2], [3, 4, 5]]), nd.array([[0, 1], [0, 3]])).asnumpy()
