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
        engine.wait_for_var(v)      # (wait_all could surface other tests' pending engine failures)
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


def test_registry_register_alias_create():
    from mxnet_maintenance_amd import registry

    class Base:
        def __init__(self, v=0):
            self.v = v

    register = registry.get_register_func(Base, 'thing')
    alias = registry.get_alias_func(Base, 'thing')
    create = registry.get_create_func(Base, 'thing')

    @alias('bee', 'b2')
    class B(Base):
        pass
    register(B)
    assert set(registry.get_registry(Base)) == {'b', 'bee', 'b2'}
    assert create('BEE', v=3).v == 3
    assert create({'thing': 'b', 'v': 4}).v == 4
    assert create('["b2", {"v": 5}]').v == 5
    inst = B(7)
    assert create(inst) is inst
    with pytest.raises(AssertionError):
        create('nothere')


def test_error_registry_maps_prefixed_messages():
    from mxnet_maintenance_amd import error
    e = error.make_error('ValueError: bad shape')
    assert isinstance(e, ValueError) and isinstance(e, mx.MXNetError)
    assert isinstance(error.make_error('TypeError: x'), TypeError)
    assert type(error.make_error('plain failure')) is mx.MXNetError
    ie = error.InternalError('boom')
    assert 'MXNet hint' in str(ie)


def test_tensorboard_event_file_roundtrip(tmp_path):
    from mxnet_maintenance_amd.contrib import tensorboard as tb
    assert tb.crc32c(b'123456789') == 0xE3069283      # CRC-32C check value
    cb = tb.LogMetricsCallback(str(tmp_path), prefix='train')

    class P:
        epoch = 3
        eval_metric = mx.metric.Accuracy()
    P.eval_metric.update([nd.array([1, 0])], [nd.array([[0.1, 0.9], [0.8, 0.2]])])
    cb(P)
    rows = tb.read_scalars(cb.summary_writer.path)
    assert rows == [(3, 'train-accuracy', 1.0)]


def test_pandas_logger_and_args_wrapper():
    from mxnet_maintenance_amd.notebook import callback as nbcb
    log = nbcb.PandasLogger(batch_size=8, frequent=1)

    class P:
        nbatch = 1
        epoch = 0
        eval_metric = mx.metric.Accuracy()
    log.train_cb(P)
    log.epoch_cb()
    assert len(log.train_df) == 1 and 'records_per_sec' in log.train_df.columns
    assert len(log.epoch_df) == 1
    args = nbcb.args_wrapper(log)
    assert set(args) == {'batch_end_callback', 'eval_end_callback', 'epoch_end_callback'}


def test_data_parallel_executor_manager_two_cpu_contexts():
    from mxnet_maintenance_amd import executor_manager as em
    assert em._split_input_slice(10, [1, 1, 2]) == [slice(0, 2), slice(2, 5), slice(5, 10)] or \
        em._split_input_slice(10, [1, 1, 2])[-1].stop == 10
    data = mx.sym.Variable('data')
    net = mx.sym.FullyConnected(data, num_hidden=3, name='fc')
    net = mx.sym.SoftmaxOutput(net, name='softmax')
    it = mx.io.NDArrayIter(np.random.rand(8, 5).astype('float32'), np.arange(8) % 3, batch_size=8)
    args = net.list_arguments()
    params = [a for a in args if a not in ('data', 'softmax_label')]
    mgr = em.DataParallelExecutorManager(net, [mx.cpu(0), mx.cpu(1)], it, args, params,
                                         net.list_auxiliary_states())
    arg_params = {'fc_weight': nd.array(np.random.rand(3, 5)), 'fc_bias': nd.zeros((3,))}
    mgr.set_params(arg_params, {})
    batch = next(iter(it))
    mgr.load_data_batch(batch)
    mgr.forward(is_train=True)
    mgr.backward()
    assert len(mgr.grad_arrays) == 2 and all(len(g) == 2 for g in mgr.grad_arrays)
    out = {k: nd.zeros(v.shape) for k, v in arg_params.items()}
    mgr.copy_to(out, {})
    np.testing.assert_allclose(out['fc_weight'].asnumpy(), arg_params['fc_weight'].asnumpy(), rtol=1e-6)
    m = mx.metric.Accuracy()
    mgr.update_metric(m, batch.label)
    assert m.get()[1] >= 0
