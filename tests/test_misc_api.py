"""Profiler, test_utils, custom operators, visualization, RTC (parity: test_profiler.py,
test_operator.py custom-op tests, test_viz.py, test_rtc.py)."""
import json
import os
import tempfile

import numpy as np
import pytest
import torch

import mxnet_maintenance_amd as mx
from mxnet_maintenance_amd import nd, autograd, profiler
from mxnet_maintenance_amd import test_utils as tu


def test_profiler_spans_trace_and_aggregate():
    with tempfile.TemporaryDirectory() as d:
        fn = os.path.join(d, 'p.json')
        profiler.set_config(profile_all=True, aggregate_stats=True, filename=fn)
        profiler.set_state('run')
        a = nd.ones((8, 8))
        nd.dot(a, a).wait_to_read()
        dom = profiler.Domain('custom')
        with dom.new_task('mytask'):
            c = dom.new_counter('ctr', 1)
            c += 4
            dom.new_marker('m').mark()
        ex = mx.sym.FullyConnected(mx.sym.var('x'), num_hidden=2).simple_bind(mx.cpu(), x=(3, 4))
        with profiler.scope('fc:'):
            ex.forward()
        profiler.pause()
        nd.dot(a, a)
        profiler.resume()
        profiler.set_state('stop')
        table = profiler.dumps()
        assert 'dot' in table and 'mytask' in table and 'fc:FullyConnected' in table
        stats = json.loads(profiler.dumps(format='json', reset=True))
        assert stats['Time']['operator']['dot']['Count'] == 1
        profiler.dump()
        ev = json.load(open(fn))['traceEvents']
        names = {e['name'] for e in ev}
        assert {'dot', 'mytask', 'ctr', 'm'} <= names
        assert any(e['ph'] == 'C' and e['args'].get('ctr') == 5 for e in ev)


def test_test_utils_checks():
    x = mx.sym.var('x')
    w = mx.sym.var('w')
    y = mx.sym.FullyConnected(x, weight=w, no_bias=True, num_hidden=3)
    tu.check_numeric_gradient(y, {'x': np.random.rand(2, 4), 'w': np.random.rand(3, 4)}, numeric_eps=1e-3,
                              rtol=1e-2, atol=1e-3, dtype=np.float64)
    xv = np.random.rand(3, 3)
    tu.check_symbolic_forward(mx.sym.tanh(x), {'x': xv}, [np.tanh(xv)])
    tu.check_symbolic_backward(mx.sym.tanh(x), {'x': xv}, [np.ones((3, 3))], {'x': 1 - np.tanh(xv) ** 2})
    tu.check_consistency(mx.sym.relu(x), [{'ctx': mx.cpu(), 'x': (4, 4), 'type_dict': {'x': np.float32}},
                                          {'ctx': mx.cpu(), 'x': (4, 4), 'type_dict': {'x': np.float64}}])
    tu.assert_almost_equal(np.ones(3), np.ones(3) + 1e-7)
    with pytest.raises(AssertionError):
        tu.assert_almost_equal(np.ones(3), np.ones(3) * 2)
    assert tu.rand_ndarray((4, 5), 'row_sparse', density=0.5).stype == 'row_sparse'
    assert len(tu.rand_shape_nd(3)) == 3
    with tu.environment({'MXAMD_TEST_ENV': '7'}):
        assert os.environ['MXAMD_TEST_ENV'] == '7'
    assert 'MXAMD_TEST_ENV' not in os.environ
    import scipy.stats as ss
    buckets, probs = tu.gen_buckets_probs_with_ppf(lambda p: ss.norm.ppf(p, 0, 1), 5)
    tu.verify_generator(lambda n: np.random.normal(0, 1, size=n), buckets, probs, nsamples=20000, nrepeat=3)


class _Sigmoid(mx.operator.CustomOp):
    def forward(self, is_train, req, in_data, out_data, aux):
        self.assign(out_data[0], req[0], 1 / (1 + nd.exp(-in_data[0])))

    def backward(self, req, out_grad, in_data, out_data, in_grad, aux):
        y = out_data[0]
        self.assign(in_grad[0], req[0], out_grad[0] * y * (1 - y))


@mx.operator.register('test_sigmoid')
class _SigmoidProp(mx.operator.CustomOpProp):
    def __init__(self, scale='1'):
        super().__init__(need_top_grad=True)
        self.scale = float(scale)

    def create_operator(self, ctx, shapes, dtypes):
        return _Sigmoid()


def test_custom_op_imperative_symbolic_hybrid():
    x = nd.array([[0., 1.], [2., -1.]])
    x.attach_grad()
    with autograd.record():
        y = nd.Custom(x, op_type='test_sigmoid', scale=2)
    y.backward()
    s = 1 / (1 + np.exp(-x.asnumpy()))
    np.testing.assert_allclose(y.asnumpy(), s, rtol=1e-6)
    np.testing.assert_allclose(x.grad.asnumpy(), s * (1 - s), rtol=1e-5)
    sym = mx.sym.Custom(mx.sym.var('x'), op_type='test_sigmoid', name='c')
    assert sym.infer_shape(x=(2, 5))[1] == [(2, 5)]
    tu.check_symbolic_forward(sym, {'x': x.asnumpy()}, [s])
    sym2 = mx.sym.load_json(sym.tojson())
    assert sym2.list_outputs() == ['c_output']

    class Net(mx.gluon.HybridBlock):
        def hybrid_forward(self, F, a):
            return F.Custom(a, op_type='test_sigmoid') * 2
    net = Net()
    net.hybridize()
    np.testing.assert_allclose(net(x).asnumpy(), 2 * s, rtol=1e-6)


def test_visualization():
    data = mx.sym.var('data')
    net = mx.sym.Convolution(data, kernel=(3, 3), num_filter=8, name='conv')
    net = mx.sym.BatchNorm(net, name='bn')
    net = mx.sym.Activation(net, act_type='relu')
    net = mx.sym.FullyConnected(mx.sym.flatten(net), num_hidden=10, name='fc')
    mx.viz.print_summary(net, shape={'data': (1, 3, 8, 8)})
    dot = mx.viz.plot_network(net, shape={'data': (1, 3, 8, 8)})
    assert 'Convolution' in dot.source and 'fc' in dot.source


def test_rtc_compiles_for_gfx950():
    src = 'extern "C" __global__ void axpy(const float* x, float* y, float a) {' \
          ' int i = blockIdx.x * blockDim.x + threadIdx.x; y[i] += a * x[i]; }'
    with tu.environment('MXAMD_RTC_CACHE', tempfile.mkdtemp()):
        mod = mx.rtc.CudaModule(src, exports=['axpy'])
        assert os.path.getsize(mod.path) > 0
        k = mod.get_kernel('axpy', 'const float* x, float* y, float a')
        assert [a[0] for a in k.args] == [True, True, False]


@pytest.mark.gpu
def test_rtc_launch_gpu():
    src = 'extern "C" __global__ void axpy(const float* x, float* y, float a) {' \
          ' int i = blockIdx.x * blockDim.x + threadIdx.x; y[i] += a * x[i]; }'
    mod = mx.rtc.CudaModule(src, exports=['axpy'])
    k = mod.get_kernel('axpy', 'const float* x, float* y, float a')
    x = nd.ones((64,), ctx=mx.gpu(0))
    y = nd.ones((64,), ctx=mx.gpu(0))
    k.launch([x, y, 3.0], mx.gpu(0), (1, 1, 1), (64, 1, 1))
    np.testing.assert_allclose(y.asnumpy(), 4.0)
