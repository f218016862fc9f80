"""Worker-stream dispatch (engine.op_stream) leaves CPU operators alone and keeps results identical."""
import numpy as onp

import mxnet_maintenance_amd as mx
from mxnet_maintenance_amd import engine


def test_cpu_ops_ignore_worker_streams():
    prev = engine.set_gpu_workers(3)
    try:
        a = mx.nd.array(onp.arange(12.0).reshape(3, 4))
        b = mx.nd.tanh(a) + a
        assert engine.slot_of(b) is None
        assert engine.op_stream([a._data]) == (None, None)
        out = mx.nd.zeros((3, 4))
        mx.nd.elemwise_add(a, a, out=out)
        onp.testing.assert_allclose(out.asnumpy(), 2 * onp.arange(12.0).reshape(3, 4))
        onp.testing.assert_allclose(b.asnumpy(), onp.tanh(a.asnumpy()) + a.asnumpy(), rtol=1e-6)
    finally:
        engine.set_gpu_workers(prev)
    assert engine.GPU_WORKERS == prev


def _disp():
    from mxnet_maintenance_amd import engine as E
    nat = E._load_native()
    if nat is None:
        import pytest
        pytest.skip('native engine not built')
    d = nat.Dispatcher(True)              # trace mode: wait edges are logged, no HIP calls
    d.set_streams(0, [11, 12])            # slots 1, 2 (fake stream handles)
    return d, (lambda: E.get().new_var(''))


def test_native_dispatcher_chains_and_cross_slot_waits():
    """The native dispatcher's protocol (src/native/engine.cc Dispatcher), traced on the host:
    round-robin for new chains, chain affinity, GPU waits only across slots, in-place writes wait for
    the other slots' readers, joins wait for every dirty worker slot."""
    d, var = _disp()
    x, w = var(), var()                   # written outside dispatch (caller's stream)
    a0 = d.begin(0, 99, [x, w])           # new chain -> slot 0 (round robin)
    assert a0 == 0 and d.take_trace() == []
    a = var()
    d.end(0, a0, [x, w], [a])
    b0 = d.begin(0, 99, [x, w])           # second chain -> slot 1, orders after the caller's stream once
    assert b0 == 1 and sorted(d.take_trace()) == [(0, 1, 0)]
    b = var()
    d.end(0, b0, [x, w], [b])
    assert d.begin(0, 99, [b, w]) == 1 and d.take_trace() == []   # chain stays on slot 1; w seen this epoch
    b2 = var()
    d.end(0, 1, [b, w], [b2])
    c0 = d.begin(0, 99, [a, b2])          # joins the chains on a's slot: waits for slot 1
    assert c0 == 0 and d.take_trace() == [(0, 0, 1)]
    c = var()
    d.end(0, c0, [a, b2], [c])
    # in-place write of x on slot 2: x was read on slots 0 and 1 -> wait for both; outside writer -> slot 0
    d.write(0, 99, 2, x)
    assert sorted(set(d.take_trace())) == [(0, 2, 0), (0, 2, 1)]
    d.end(0, 2, [], [x])
    assert type(d).slot_of(x) == 2 and type(d).slot_of(c) == 0
    assert sorted(d.join(0, 99)) == [1, 2]
    assert sorted(d.take_trace()) == [(0, 0, 1), (0, 0, 2)]
    assert d.join(0, 99) == []            # nothing new since the last join
    # after the join (new epoch) a worker slot orders after the caller's stream again for w
    assert d.begin(0, 99, [w]) == 2 and d.take_trace() == [(0, 2, 0)]   # round robin continues at 2
    d.end(0, 2, [w], [var()])
    assert d.begin(0, 99, [w]) == 0 and d.take_trace() == []
    d.end(0, 0, [w], [var()])
    assert d.begin(0, 99, [w]) == 1 and d.take_trace() == [(0, 1, 0)]
