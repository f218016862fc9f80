"""In-process multi-device reduce/broadcast (kvstore/comm.py; reference src/kvstore/comm.h)."""
import numpy as np
import pytest
import torch

import mxnet_maintenance_amd as mx
from mxnet_maintenance_amd.kvstore.comm import DeviceComm


def test_root_placement_balances_bytes():
    c = DeviceComm()
    # two devices (host + meta stand in for two GPUs): roots alternate so merge bytes stay balanced
    big = [torch.ones(1000), torch.ones(1000, device='meta')]
    small = [torch.ones(10), torch.ones(10, device='meta')]
    assert c.root_for('a', big) == 0
    assert c.root_for('b', big) == 1
    assert c.root_for('c', small) == 0
    assert c.root_for('a', big) == 0          # sticky per key


def test_reduce_and_broadcast_host_copies():
    c = DeviceComm()
    vals = [[torch.full((3,), float(i + j)) for j in range(3)] for i in range(4)]
    sums = c.reduce(list(range(4)), vals)
    for i, s in enumerate(sums):
        np.testing.assert_allclose(s.numpy(), np.full(3, 3.0 * i + 3.0))
        assert all(s.data_ptr() != v.data_ptr() for v in vals[i])    # fresh merge buffer
    outs = [[torch.zeros(3), torch.zeros(3, dtype=torch.float64)] for _ in range(4)]
    c.broadcast(sums, outs)
    for s, os_ in zip(sums, outs):
        for o in os_:
            np.testing.assert_allclose(o.numpy(), s.numpy())


def test_kvstore_multi_context_pushpull_cpu():
    kv = mx.kv.create('device')
    shape = (4, 5)
    kv.init('w', mx.nd.zeros(shape))
    vals = [mx.nd.ones(shape, ctx=mx.cpu(i)) * (i + 1) for i in range(3)]
    outs = [mx.nd.zeros(shape, ctx=mx.cpu(i)) for i in range(3)]
    kv.pushpull('w', vals, out=outs)
    for o in outs:
        np.testing.assert_allclose(o.asnumpy(), np.full(shape, 6.0))
    kv.push('w', vals)
    kv.pull('w', out=outs)
    for o in outs:
        np.testing.assert_allclose(o.asnumpy(), np.full(shape, 6.0))


@pytest.mark.gpu
def test_kvstore_multi_context_pushpull_gpu():
    n = max(1, torch.cuda.device_count())
    ctxs = [mx.gpu(i % n) for i in range(2)]
    kv = mx.kv.create('device')
    shape = (64, 33)
    kv.init(3, mx.nd.zeros(shape, ctx=ctxs[0]))
    vals = [mx.nd.ones(shape, ctx=c) * (i + 1) for i, c in enumerate(ctxs)]
    outs = [mx.nd.zeros(shape, ctx=c) for c in ctxs]
    kv.pushpull(3, vals, out=outs)
    for o in outs:
        np.testing.assert_allclose(o.asnumpy(), np.full(shape, 3.0))


def test_device_comm_rccl_path_with_fake_collectives(monkeypatch):
    """The in-process RCCL path of DeviceComm (distinct GPUs) driven on the host: the collectives are
    replaced by CPU stand-ins with the same contracts, so key grouping, root placement, coalescing
    and the broadcast fan-out are exercised without several GPUs."""
    from mxnet_maintenance_amd.kvstore import comm as C
    calls = {'reduce': [], 'bcast': []}

    def fake_reduce(inputs, destination, buffer_size):
        calls['reduce'].append((len(inputs), len(inputs[0]), destination))
        return [sum(per_dev[k] for per_dev in inputs) for k in range(len(inputs[0]))]

    def fake_bcast(tensors, devices, buffer_size):
        calls['bcast'].append((len(tensors), list(devices)))
        return [[t.clone() for t in tensors] for _ in devices]

    monkeypatch.setattr(C, '_distinct_gpus', lambda ts: len(ts) > 1)
    monkeypatch.setattr(C, '_rccl_ok', lambda ts: True)
    monkeypatch.setattr(C, '_rccl_broadcast_ok', lambda s, ds: len(ds) > 1)
    monkeypatch.setattr(C, '_reduce_coalesced', fake_reduce)
    monkeypatch.setattr(C, '_broadcast_coalesced', fake_bcast)
    c = C.DeviceComm()
    ndev, keys = 4, ['a', 'b', 'c']
    vals = [[torch.full((5,), float(10 * k + d)) for d in range(ndev)] for k in range(len(keys))]
    sums = c.reduce(keys, vals)
    for k, s in enumerate(sums):
        np.testing.assert_allclose(s.numpy(), np.full(5, sum(10.0 * k + d for d in range(ndev))))
    # keys with the same (devices, root, dtype) share one coalesced collective
    assert sum(n for _, n, _ in calls['reduce']) == len(keys)
    assert all(n_dev == ndev for n_dev, _, _ in calls['reduce'])
    outs = [[torch.zeros(5) for _ in range(ndev)] for _ in keys]
    c.broadcast(sums, outs)
    assert sum(n for n, _ in calls['bcast']) == len(keys)
    for s, row in zip(sums, outs):
        for o in row:
            np.testing.assert_allclose(o.numpy(), s.numpy())


def test_bucket_size_model(monkeypatch):
    from mxnet_maintenance_amd.parallel import buckets as B
    monkeypatch.delenv('MXAMD_BUCKET_MB', raising=False)
    mb = 1 << 20
    assert B.bucket_bytes_for(51 * mb) == 16 * mb                   # ResNet-50 fp16 grads
    assert B.bucket_bytes_for(220 * mb) == 55 * mb                  # BERT-base bf16 grads
    assert B.bucket_bytes_for(4000 * mb) == 64 * mb
    assert 0.75 < B.link_efficiency(16 * mb) < B.link_efficiency(64 * mb) < 0.95
    monkeypatch.setenv('MXAMD_BUCKET_MB', '8')
    assert B.bucket_bytes_for(51 * mb) == 8 * mb
