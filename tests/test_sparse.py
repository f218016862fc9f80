"""Compressed sparse storage (csr / row_sparse): constructors, conversions, sparse-native dot, retain,
elementwise, kvstore row_sparse_pull, lazy optimizer updates, save/load.  CPU tests + gfx950 dot kernels."""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

import mxnet_maintenance_amd as mx
from mxnet_maintenance_amd import nd


def _rand_csr(m, n, density, seed=0):
    return sp.random(m, n, density=density, format='csr', random_state=seed, dtype=np.float32)


def test_csr_components_and_roundtrip():
    s = _rand_csr(20, 30, 0.2)
    a = nd.sparse.csr_matrix((s.data, s.indices, s.indptr), shape=s.shape)
    assert a.stype == 'csr' and a.shape == (20, 30)
    np.testing.assert_array_equal(a.indptr.asnumpy(), s.indptr)
    np.testing.assert_array_equal(a.indices.asnumpy(), s.indices)
    np.testing.assert_allclose(a.data.asnumpy(), s.data)
    np.testing.assert_allclose(a.asnumpy(), s.toarray())
    np.testing.assert_allclose(a.asscipy().toarray(), s.toarray())
    d = a.tostype('default')
    assert d.stype == 'default'
    b = d.tostype('csr')
    np.testing.assert_array_equal(b.indptr.asnumpy(), s.indptr)
    # row slices stay compressed
    r = a[3:9]
    assert r.stype == 'csr' and r.shape == (6, 30)
    np.testing.assert_allclose(r.asnumpy(), s.toarray()[3:9])
    a.check_format()


def test_csr_does_not_densify_for_sparse_ops():
    s = _rand_csr(50, 40, 0.1, seed=3)
    a = nd.sparse.csr_matrix(s)
    rhs = nd.array(np.random.RandomState(0).randn(40, 7).astype(np.float32))
    out = nd.sparse.dot(a, rhs)
    assert a._dense is None, 'dot(csr, dense) must not build the dense lhs'
    np.testing.assert_allclose(out.asnumpy(), s @ rhs.asnumpy(), rtol=1e-5, atol=1e-5)
    g = nd.array(np.random.RandomState(1).randn(50, 3).astype(np.float32))
    t = nd.sparse.dot(a, g, transpose_a=True)
    assert t.stype == 'row_sparse' and a._dense is None
    np.testing.assert_array_equal(t.indices.asnumpy(), np.unique(s.indices))
    np.testing.assert_allclose(t.asnumpy(), s.T @ g.asnumpy(), rtol=1e-5, atol=1e-5)


def test_row_sparse_ops():
    u = nd.sparse.row_sparse_array((np.ones((2, 3), np.float32), [4, 1]), shape=(6, 3))
    np.testing.assert_array_equal(u.indices.asnumpy(), [4, 1])          # kept as given ...
    with pytest.raises(mx.base.MXNetError):
        u.check_format()                                                 # ... and reported invalid
    a = nd.sparse.row_sparse_array((np.ones((2, 3), np.float32), [1, 4]), shape=(6, 3))
    b = nd.sparse.row_sparse_array((np.full((2, 3), 2, np.float32), [1, 5]), shape=(6, 3))
    c = a + b
    assert c.stype == 'row_sparse'
    np.testing.assert_array_equal(c.indices.asnumpy(), [1, 4, 5])
    np.testing.assert_allclose(c.asnumpy(), a.asnumpy() + b.asnumpy())
    np.testing.assert_allclose((a - b).asnumpy(), a.asnumpy() - b.asnumpy())
    m = a * b
    np.testing.assert_array_equal(m.indices.asnumpy(), [1])
    np.testing.assert_allclose(m.asnumpy(), a.asnumpy() * b.asnumpy())
    s = a * 3.0
    assert s.stype == 'row_sparse'
    np.testing.assert_allclose(s.asnumpy(), a.asnumpy() * 3)
    r = nd.sparse.retain(c, nd.array([5, 4]))
    np.testing.assert_array_equal(r.indices.asnumpy(), [4, 5])
    z = nd.sparse.zeros('row_sparse', (4, 2))
    assert z.indices.shape == (0,) and z.asnumpy().sum() == 0
    a += b
    np.testing.assert_allclose(a.asnumpy(), c.asnumpy())


def test_dense_writes_resync_compressed_form():
    a = nd.sparse.row_sparse_array((np.ones((1, 2), np.float32), [0]), shape=(3, 2))
    a._data[2] = 5.0           # a generic op writing through the dense view
    np.testing.assert_array_equal(a.indices.asnumpy(), [0, 2])
    x = nd.sparse.zeros('csr', (2, 2))
    nd.array([[0, 1], [2, 0]]).copyto(x)
    np.testing.assert_array_equal(x.indices.asnumpy(), [1, 0])


def test_row_sparse_pull_gathers_rows_only():
    kv = mx.kv.create('local')
    w = np.arange(20, dtype=np.float32).reshape(10, 2)
    kv.init('emb', nd.array(w))
    out = nd.sparse.zeros('row_sparse', (10, 2))
    kv.row_sparse_pull('emb', out=out, row_ids=nd.array([7, 2, 2]))
    np.testing.assert_array_equal(out.indices.asnumpy(), [2, 7])
    np.testing.assert_allclose(out.data.asnumpy(), w[[2, 7]])


@pytest.mark.parametrize('opt', ['sgd', 'adam'])
def test_lazy_update_touches_only_present_rows(opt):
    o = mx.optimizer.create(opt, learning_rate=0.1, wd=0.01, **({'momentum': 0.9} if opt == 'sgd' else {}))
    w = nd.array(np.ones((6, 3), np.float32))
    state = o.create_state(0, w)
    g = nd.sparse.row_sparse_array((np.full((2, 3), 0.5, np.float32), [1, 4]), shape=(6, 3))
    o.update(0, w, g, state)
    wn = w.asnumpy()
    assert np.all(wn[[0, 2, 3, 5]] == 1.0), 'rows absent from the gradient must not move (lazy update)'
    assert np.all(wn[[1, 4]] < 1.0)
    # the same rows with a dense gradient give the same values there
    o2 = mx.optimizer.create(opt, learning_rate=0.1, wd=0.01, **({'momentum': 0.9} if opt == 'sgd' else {}))
    w2 = nd.array(np.ones((6, 3), np.float32))
    o2.update(0, w2, g.tostype('default'), o2.create_state(0, w2))
    np.testing.assert_allclose(wn[[1, 4]], w2.asnumpy()[[1, 4]], rtol=1e-6)


def test_sparse_save_load(tmp_path):
    s = _rand_csr(8, 9, 0.3, seed=5)
    a = nd.sparse.csr_matrix(s)
    r = nd.sparse.row_sparse_array((np.arange(6, dtype=np.float32).reshape(2, 3), [0, 3]), shape=(5, 3))
    f = str(tmp_path / 'sp.params')
    nd.save(f, {'a': a, 'r': r})
    back = nd.load(f)
    assert back['a'].stype == 'csr' and back['r'].stype == 'row_sparse'
    np.testing.assert_allclose(back['a'].asnumpy(), s.toarray())
    np.testing.assert_array_equal(back['r'].indices.asnumpy(), [0, 3])


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize('n', [1, 64, 300])
def test_csr_dot_hip_kernels(dtype, n):
    from mxnet_maintenance_amd.ops import kernels
    assert kernels.available()
    s = _rand_csr(500, 700, 0.02, seed=2)
    a = nd.sparse.csr_matrix(s, ctx=mx.gpu(0), dtype=dtype)
    rhs = torch.randn(700, n, device='cuda').to(dtype)
    out = nd.sparse.dot(a, nd.NDArray(rhs))
    ref = torch.from_numpy(s.toarray()).cuda().to(dtype).float() @ rhs.float()
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    torch.testing.assert_close(out._data.float(), ref, rtol=tol, atol=tol)
    g = torch.randn(500, n, device='cuda').to(dtype)
    t = nd.sparse.dot(a, nd.NDArray(g), transpose_a=True)
    assert t.stype == 'row_sparse'
    reft = torch.from_numpy(s.toarray()).cuda().to(dtype).float().t() @ g.float()
    torch.testing.assert_close(t.todense()._data.float(), reft, rtol=tol, atol=tol * 4)
