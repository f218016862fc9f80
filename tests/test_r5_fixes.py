"""Round-5 regression tests (advisor findings and verdict items)."""
import os

import numpy as np
import pytest

import mxnet_maintenance_amd as mx
from mxnet_maintenance_amd import gluon, nd, autograd


def test_row_sparse_data_does_not_destroy_unpulled_rows(tmp_path):
    """row_sparse_data(subset) outside record() must not zero the replica (save/load keeps every row)."""
    p = gluon.Parameter('emb_weight', shape=(10, 4), stype='row_sparse', grad_stype='row_sparse')
    p.initialize(init=mx.init.Uniform(1.0), ctx=mx.cpu())
    tr = gluon.Trainer([p], 'sgd', {'learning_rate': 0.1}, kvstore='local')
    before = p._reduce().asnumpy().copy()
    sub = p.row_sparse_data(nd.array([1, 3], dtype='int64'))
    got = sub.asnumpy()
    np.testing.assert_allclose(got[[1, 3]], before[[1, 3]])
    assert np.all(got[[0, 2, 4, 5, 6, 7, 8, 9]] == 0)
    after = p._reduce().asnumpy()
    np.testing.assert_allclose(after, before)
    # save / load round trip through a ParameterDict keeps every row
    pd = gluon.ParameterDict()
    pd._params['emb_weight'] = p
    f = str(tmp_path / 'w.params')
    pd.save(f)
    loaded = nd.load(f)
    np.testing.assert_allclose(list(loaded.values())[0].asnumpy(), before)


def test_sparse_weight_rejects_kvstore_none():
    p = gluon.Parameter('w', shape=(6, 2), stype='row_sparse', grad_stype='row_sparse')
    p.initialize(ctx=mx.cpu())
    tr = gluon.Trainer([p], 'sgd', {'learning_rate': 0.1}, kvstore=None)
    with pytest.raises(TypeError):
        tr._init_kvstore()


def test_wait_for_var_inside_bulk_flushes_gathered_ops():
    """A wait inside bulk() must see the gathered writer executed (reference BulkFlush in WaitForVar)."""
    from mxnet_maintenance_amd import engine
    v = engine.new_var('bulkvar')
    hits = []
    with engine.bulk(16):
        engine.push(lambda: hits.append(1), (), (v,))
        engine.wait_for_var(v)
        assert hits == [1]
        engine.push(lambda: hits.append(2), (), (v,))
        engine.wait_all()
        assert hits == [1, 2]


@pytest.mark.gpu
def test_pinned_source_overwrite_after_async_copy():
    """as_in_context from a cpu_pinned array, then overwrite the host array: the GPU copy keeps the
    old values (the copy reads a private snapshot, not the user's buffer)."""
    import torch
    src = nd.array(np.arange(1 << 16, dtype=np.float32), ctx=mx.cpu_pinned())
    g = src.as_in_context(mx.gpu(0))
    src[:] = -1.0
    torch.cuda.synchronize()
    np.testing.assert_array_equal(g.asnumpy(), np.arange(1 << 16, dtype=np.float32))
