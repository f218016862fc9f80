"""Native runtime (engine, storage, recordio) and KVStore incl. multi-process (parity:
test_engine.py, test_exc_handling.py, test_recordio.py, test_kvstore.py, test_kvstore_custom.py,
tests/nightly/dist_sync_kvstore.py)."""
import os
import tempfile
import threading
import time

import numpy as np
import pytest
import torch
import torch.multiprocessing as tmp

import mxnet_maintenance_amd as mx
from mxnet_maintenance_amd import nd, engine, recordio


def test_native_available():
    assert engine.native_available()
    from mxnet_maintenance_amd._lib import _native  # noqa: F401


def test_engine_write_read_ordering():
    from mxnet_maintenance_amd._lib import _native
    eng = _native.Engine(4, False)
    v = eng.new_var('v')
    log = []
    lock = threading.Lock()

    def writer(i):
        def f():
            time.sleep(0.002)
            with lock:
                log.append(('w', i))
        return f

    def reader(i):
        def f():
            with lock:
                log.append(('r', i))
        return f
    eng.push(writer(0), [], [v])
    for i in range(4):
        eng.push(reader(i), [v], [])
    eng.push(writer(1), [], [v])
    eng.wait_for_all()
    assert log[0] == ('w', 0) and log[-1] == ('w', 1)
    assert sorted(log[1:5]) == [('r', i) for i in range(4)]
    assert v.version == 2


def test_engine_parallel_independent_vars():
    from mxnet_maintenance_amd._lib import _native
    eng = _native.Engine(4, False)
    vs = [eng.new_var() for _ in range(4)]
    t0 = time.time()
    for v in vs:
        eng.push(lambda: time.sleep(0.1), [], [v])
    eng.wait_for_all()
    assert time.time() - t0 < 0.35   # ran concurrently


def test_engine_exception_propagation():
    from mxnet_maintenance_amd._lib import _native
    eng = _native.Engine(2, False)
    v = eng.new_var()

    def bad():
        raise ValueError('boom')
    eng.push(bad, [], [v])
    with pytest.raises(ValueError):
        eng.wait_for_var(v)
    eng.push(lambda: None, [], [v])
    eng.wait_for_all()


def test_naive_engine():
    from mxnet_maintenance_amd._lib import _native
    eng = _native.Engine(0, True)
    out = []
    v = eng.new_var()
    eng.push(lambda: out.append(1), [], [v])
    assert out == [1]


def test_engine_async_file_write():
    with tempfile.TemporaryDirectory() as d:
        f = os.path.join(d, 'x.bin')
        v = engine.new_var()
        engine.push_write_file(f, b'hello', mutable_vars=[v])
        engine.wait_for_var(v)
        assert open(f, 'rb').read() == b'hello'


def test_host_storage_pool():
    from mxnet_maintenance_amd._lib import _native
    s = _native.HostStorage(False)
    p = s.alloc(1000)
    s.free(p)
    q = s.alloc(900)
    assert q == p and s.hits == 1
    s.free(q)
    s.release_all()
    assert s.pooled_bytes == 0


def test_recordio_roundtrip_and_magic_split():
    with tempfile.TemporaryDirectory() as d:
        f = os.path.join(d, 'a.rec')
        magic = (0xced7230a).to_bytes(4, 'little')
        payloads = [b'abc', b'', b'x' * 1001, b'1234' + magic + b'5678' + magic, os.urandom(333)]
        w = recordio.MXRecordIO(f, 'w')
        for p in payloads:
            w.write(p)
        w.close()
        r = recordio.MXRecordIO(f, 'r')
        got = []
        while True:
            b = r.read()
            if b is None:
                break
            got.append(b)
        assert got == payloads
        # the python codec reads what the native writer wrote
        pr = recordio._PyReader(f)
        assert [pr.read() for _ in payloads] == payloads


def test_indexed_recordio_and_pack():
    with tempfile.TemporaryDirectory() as d:
        f, idx = os.path.join(d, 'b.rec'), os.path.join(d, 'b.idx')
        w = recordio.MXIndexedRecordIO(idx, f, 'w')
        for i in range(5):
            w.write_idx(i, recordio.pack(recordio.IRHeader(0, float(i), i, 0), b'data%d' % i))
        w.close()
        r = recordio.MXIndexedRecordIO(idx, f, 'r')
        assert r.keys == list(range(5))
        h, s = recordio.unpack(r.read_idx(3))
        assert h.label == 3.0 and s == b'data3'
        h2, _ = recordio.unpack(recordio.pack(recordio.IRHeader(0, [1., 2.], 7, 0), b''))
        assert list(h2.label) == [1., 2.]


def test_kvstore_local_single_process():
    kv = mx.kv.create('local')
    assert kv.rank == 0 and kv.num_workers == 1
    kv.init(3, nd.ones((2, 3)))
    kv.push(3, [nd.ones((2, 3)) * 2, nd.ones((2, 3)) * 3])
    out = nd.zeros((2, 3))
    kv.pull(3, out=out)
    np.testing.assert_allclose(out.asnumpy(), 5)
    out = nd.zeros((2, 3)).tostype("row_sparse")
    kv.row_sparse_pull(3, out=out, row_ids=nd.array([1]))
    np.testing.assert_allclose(out.asnumpy()[0], 0)
    # a store takes one kind of key (the reference's restriction): string keys go to another store
    with pytest.raises(mx.base.MXNetError):
        kv.init('g', nd.ones((4,)))
    skv = mx.kv.create('local')
    vals = [nd.ones((4,)), nd.ones((4,)) * 2]
    skv.pushpull('g', vals, vals)
    np.testing.assert_allclose(vals[0].asnumpy(), 3)
    skv.set_optimizer(mx.optimizer.SGD(learning_rate=0.1))
    skv.init('w', nd.ones((2,)))
    skv.push('w', nd.ones((2,)))
    o = nd.zeros((2,))
    skv.pull('w', out=o)
    np.testing.assert_allclose(o.asnumpy(), 0.9, rtol=1e-6)


def test_custom_kvstore_registry():
    kv = mx.kv.create('teststore')
    assert kv.type == 'teststore' and not kv.is_capable('optimizer')
    a, b = nd.ones((2,)), nd.ones((2,)) * 2
    out = nd.zeros((2,))
    kv.pushpull('k', [a, b], out=out)
    np.testing.assert_allclose(out.asnumpy(), 3)


def test_gradient_compression_codec():
    from mxnet_maintenance_amd.kvstore.compression import quantize_2bit, dequantize_2bit
    g = torch.tensor([0.6, -0.7, 0.1, 0.0, 2.0])
    res = torch.zeros(5)
    p = quantize_2bit(g, res, 0.5)
    d = dequantize_2bit(p, 5, 0.5)
    assert d.tolist() == [0.5, -0.5, 0.0, 0.0, 0.5]
    np.testing.assert_allclose(res.numpy(), [0.1, -0.2, 0.1, 0.0, 1.5], atol=1e-6)


def _dist_worker(rank, world, port, q):
    os.environ.update({'RANK': str(rank), 'WORLD_SIZE': str(world), 'LOCAL_RANK': str(rank),
                       'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port), 'MXAMD_DIST_BACKEND': 'gloo'})
    import mxnet_maintenance_amd as mx
    from mxnet_maintenance_amd import nd, gluon, autograd
    try:
        kv = mx.kv.create('dist_sync')
        assert kv.num_workers == world and kv.rank == rank
        kv.init('a', nd.ones((3,)) * (rank + 1))          # rank 0 value is broadcast
        out = nd.zeros((3,))
        kv.pull('a', out=out)
        r1 = out.asnumpy().tolist()
        v = [nd.ones((3,)) * (rank + 1), nd.ones((5,)) * 10]
        kv.pushpull(['x', 'y'], v, v)
        r2 = v[0].asnumpy().tolist() + v[1].asnumpy().tolist()
        # Gluon data-parallel step: weights stay identical across ranks, grads are summed
        mx.random.seed(0)
        net = gluon.nn.Dense(2, in_units=3)
        net.initialize(mx.init.One())
        tr = gluon.Trainer(net.collect_params(), 'sgd', {'learning_rate': 0.1}, kvstore='device')
        x = nd.ones((4, 3)) * (rank + 1)
        with autograd.record():
            l = net(x).sum()
        l.backward()
        tr.step(4 * world)
        r3 = net.weight.data().asnumpy().reshape(-1).tolist()
        q.put((rank, r1, r2, r3))
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, 'ERR', traceback.format_exc(), None))
    finally:
        import torch.distributed as d
        if d.is_initialized():
            d.destroy_process_group()


def test_kvstore_dist_sync_two_processes_gloo():
    ctx = tmp.get_context('spawn')
    q = ctx.Queue()
    port = 29000 + os.getpid() % 1000
    procs = [ctx.Process(target=_dist_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        item = q.get(timeout=240)
        res[item[0]] = item
    for p in procs:
        p.join(timeout=60)
    for r in range(2):
        assert res[r][1] != 'ERR', res[r][2]
        assert res[r][1] == [1, 1, 1]
        assert res[r][2] == [3, 3, 3] + [20] * 5
    # grads: d(sum(xW^T))/dW = sum over batch of x -> rank0: 4*1, rank1: 4*2 -> sum 12 per element
    expect = 1 - 0.1 * 12 / 8
    np.testing.assert_allclose(res[0][3], expect, rtol=1e-5)
    assert res[0][3] == res[1][3]


def test_arena_bucket_layout_small_tail():
    """Trainer gradient buckets: contiguous arena slices, big buckets first, small tail buckets for the
    first layers (reduced after backward ends)."""
    import torch
    from mxnet_maintenance_amd.gluon.trainer import _ArenaBuckets

    class _P:
        def __init__(self, t):
            self._t = t

        def list_data(self):
            return [self._t]

        _all_data = list_data

    sizes = [3000, 500, 800, 12000, 9000, 7000, 100]
    offs = np.cumsum([0] + sizes[:-1]).tolist()

    class _A:
        g = torch.zeros(sum(sizes), dtype=torch.float16)
        params = [_P(mx.nd.zeros((n,))) for n in sizes]
        views = [(o, n, (n,)) for o, n in zip(offs, sizes)]

    kb = 1024
    b = _ArenaBuckets([_A()], bucket_bytes=24 * kb, tail_bytes=4 * kb)
    spans = [(x.flat.data_ptr() - _A.g.data_ptr()) // 2 for x in b.buckets]
    lens = [x.flat.numel() for x in b.buckets]
    # buckets tile the arena back to front without gaps
    assert sum(lens) == sum(sizes)
    assert all(s + n == prev for s, n, prev in zip(spans[1:], lens[1:], spans[:-1]))
    # the last bucket (first layers) is under the tail cap unless a single tensor is larger
    assert lens[-1] * 2 <= 4 * kb or b.buckets[-1].count == 1
    assert max(lens[:2]) * 2 > 4 * kb


def _dp_mlp_train(rank, world, xs, ys, steps):
    import mxnet_maintenance_amd as mx
    from mxnet_maintenance_amd import nd, gluon, autograd
    mx.random.seed(3)
    net = gluon.nn.HybridSequential()
    net.add(gluon.nn.Dense(16, activation='relu', in_units=6), gluon.nn.Dense(16, activation='tanh', in_units=16),
            gluon.nn.Dense(3, in_units=16))
    net.initialize(mx.init.Xavier())
    net.hybridize()
    tr = gluon.Trainer(net.collect_params(), 'sgd', {'learning_rate': 0.2, 'momentum': 0.9, 'wd': 1e-3},
                       kvstore='device')
    loss_fn = gluon.loss.SoftmaxCrossEntropyLoss()
    for s in range(steps):
        x, y = nd.array(xs[s]), nd.array(ys[s])
        with autograd.record():
            l = loss_fn(net(x), y)
        l.backward()
        tr.step(x.shape[0] * world)
    return [p.data().asnumpy() for p in net.collect_params().values()], len(getattr(tr, '_buckets', None).buckets
                                                                             if getattr(tr, '_buckets', None) else [])


def _dp_worker(rank, world, port, q, xs, ys, steps):
    os.environ.update({'RANK': str(rank), 'WORLD_SIZE': str(world), 'LOCAL_RANK': str(rank),
                       'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port), 'MXAMD_DIST_BACKEND': 'gloo',
                       'MXAMD_BUCKET_MB': '0.0005', 'MXAMD_TAIL_BUCKET_MB': '0.0002'})
    try:
        import mxnet_maintenance_amd as mx  # noqa: F401
        from mxnet_maintenance_amd.parallel import dist
        dist.init()
        w, nb = _dp_mlp_train(rank, world, [x[rank] for x in xs], [y[rank] for y in ys], steps)
        q.put((rank, w, nb))
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, 'ERR', traceback.format_exc()))
    finally:
        import torch.distributed as d
        if d.is_initialized():
            d.destroy_process_group()


def test_data_parallel_bucketed_overlap_matches_single_process():
    """2-rank DP (gloo) with several overlapped gradient buckets == one process on the concatenated
    batch (SGD momentum + wd, global-batch normalisation)."""
    rs = np.random.RandomState(1)
    steps, world = 3, 2
    xs = [rs.randn(world, 5, 6).astype('float32') for _ in range(steps)]
    ys = [rs.randint(0, 3, size=(world, 5)).astype('float32') for _ in range(steps)]
    ctx = tmp.get_context('spawn')
    q = ctx.Queue()
    port = 30000 + os.getpid() % 1000
    procs = [ctx.Process(target=_dp_worker, args=(r, world, port, q, xs, ys, steps)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        item = q.get(timeout=240)
        res[item[0]] = item
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert res[r][1] != 'ERR', res[r][2]
    assert res[0][2] >= 3, 'expected several gradient buckets, got %d' % res[0][2]
    ref, _ = _dp_mlp_train(0, 1, [x.reshape(-1, 6) for x in xs], [y.reshape(-1) for y in ys], steps)
    for a, b, c in zip(res[0][1], res[1][1], ref):
        np.testing.assert_array_equal(a, b)
        np.testing.assert_allclose(a, c, rtol=1e-4, atol=1e-5)


def _compression_worker(rank, world, port, q, pushes):
    os.environ.update({'RANK': str(rank), 'WORLD_SIZE': str(world), 'LOCAL_RANK': str(rank),
                       'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port), 'MXAMD_DIST_BACKEND': 'gloo'})
    try:
        import mxnet_maintenance_amd as mx
        from mxnet_maintenance_amd import nd
        kv = mx.kv.create('dist_sync')
        kv.set_gradient_compression({'type': '2bit', 'threshold': 0.5})
        keys = ['a', 'b', 'c']
        grads = {'a': 0.25, 'b': 0.75, 'c': -0.125}
        for k in keys:
            kv.init(k, nd.zeros((4,)))
        outs = []
        for _ in range(pushes):
            vals = [nd.ones((4,)) * grads[k] for k in keys]
            res = [nd.zeros((4,)) for _ in keys]
            kv.pushpull(keys, vals, out=res)
            outs.append([float(r.asnumpy()[0]) for r in res])
        q.put((rank, outs, len(kv._compression._residuals)))
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, 'ERR', traceback.format_exc()))
    finally:
        import torch.distributed as d
        if d.is_initialized():
            d.destroy_process_group()


def test_gradient_compression_residual_per_key_two_processes():
    """2-bit compression keeps ONE error-feedback residual per kvstore key, even for same-size keys
    pushed through fresh buffers (reference comm.h buf.residual), and sums the quantised codes."""
    world, pushes, thr = 2, 5, 0.5
    ctx = tmp.get_context('spawn')
    q = ctx.Queue()
    port = 31000 + os.getpid() % 1000
    procs = [ctx.Process(target=_compression_worker, args=(r, world, port, q, pushes)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        item = q.get(timeout=240)
        res[item[0]] = item
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert res[r][1] != 'ERR', res[r][2]
        assert res[r][2] == 3
    # host model of error feedback, per key; both ranks push the same gradient so the sum is 2x
    expect = []
    resid = {'a': 0.0, 'b': 0.0, 'c': 0.0}
    for _ in range(pushes):
        row = []
        for k, g in (('a', 0.25), ('b', 0.75), ('c', -0.125)):  # exact in fp32
            resid[k] += g
            q_ = thr if resid[k] >= thr else (-thr if resid[k] <= -thr else 0.0)
            resid[k] -= q_
            row.append(world * q_)
        expect.append(row)
    np.testing.assert_allclose(res[0][1], expect, atol=1e-6)
    assert res[0][1] == res[1][1]


def test_bench_gpus_flag_launches_ranks():
    """`bench.py --gpus 2` without a launcher starts 2 worker processes (gloo on CPU) and reports n_gpus=2."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK')}
    out = subprocess.run([sys.executable, os.path.join(root, 'bench.py'), '--gpus', '2', '--steps', '1',
                          '--warmup', '1', '--batch', '2', '--image-size', '32', '--dtype', 'float32',
                          '--model', 'resnet18_v1b'], capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec['n_gpus'] == 2 and rec['config']['parallelism'] == 'dp2' and rec['config']['global_batch'] == 4


def test_bench_eight_ranks_through_torchrun():
    """The driver's N=8 launch (`torch.distributed.run --nproc-per-node 8 bench.py --gpus 8`) rehearsed
    on gloo: every rank joins, gradients are reduced in buckets, and rank 0 prints one dp8 line."""
    import json
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    env = {k: v for k, v in os.environ.items() if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK')}
    env['OMP_NUM_THREADS'] = '1'
    out = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '8',
                          '--master-addr', '127.0.0.1', '--master-port', str(port), 'bench.py', '--gpus', '8',
                          '--steps', '1', '--warmup', '1', '--batch', '2', '--image-size', '32',
                          '--dtype', 'float32', '--model', 'resnet18_v1b'],
                         capture_output=True, text=True, timeout=600, env=env, cwd=root)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec['n_gpus'] == 8 and rec['config']['parallelism'] == 'dp8' and rec['config']['global_batch'] == 16
    assert rec['value'] > 0
