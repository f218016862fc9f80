"""Extension-library graph passes, partitioners and subgraph operators (library_graph.py), driven
with the reference's own example libraries (example/extensions/lib_pass, lib_subgraph) compiled
here from their sources against include/mxnet/lib_api.h -- the reference's
example/extensions/lib_subgraph/test_subgraph.py flow: partition with a supportedOps partitioner and
with a selector partitioner, run the subgraph through the library's stateful op, then a graph pass
that adds an input (allocated through nd_malloc) to the subgraph node."""
import os
import subprocess

import numpy as np
import pytest

import mxnet_maintenance_amd as mx

REF = '/root/reference'


def _build(tmp_path, example, name):
    src = os.path.join(REF, 'example', 'extensions', example, name + '.cc')
    if not (os.path.exists(src) and os.path.exists(os.path.join(REF, 'src', 'lib_api.cc'))):
        pytest.skip('reference example sources not available')
    so = str(tmp_path / ('lib%s.so' % name))
    subprocess.check_call(['g++', '-shared', '-fPIC', '-O1', '-std=c++17', '-I' + os.path.join(REF, 'include'), src,
                           os.path.join(REF, 'src', 'lib_api.cc'), '-o', so])
    return so


@pytest.fixture(scope='module')
def subgraph_lib(tmp_path_factory):
    so = _build(tmp_path_factory.mktemp('ext'), 'lib_subgraph', 'subgraph_lib')
    mx.library.load(so, verbose=False)
    return so


def _net():
    a, b = mx.sym.var('a'), mx.sym.var('b')
    return mx.sym.log(mx.sym.exp(a + b))


@pytest.mark.parametrize('backend', ['myProp', 'mySelect'])
def test_partitioner_builds_library_subgraph_op(subgraph_lib, backend):
    sym = _net()
    args = {'a': mx.nd.ones((3, 2)), 'b': mx.nd.ones((3, 2)) * 0.5}
    part = sym.optimize_for(backend, args, dedup_subgraph=True)
    import json
    ops = [n['op'] for n in json.loads(part.tojson())['nodes']]
    assert '_custom_subgraph_op' in ops and 'exp' not in ops and 'log' not in ops
    node = [n for n in json.loads(part.tojson())['nodes'] if n['op'] == '_custom_subgraph_op'][0]
    assert node['attrs'].get('myKey') == 'myVal'                 # reviewSubgraph's extra attribute
    assert json.loads(node['attrs']['subgraph_sym_json'])['nodes'][1]['op'] == 'exp'
    out = part.bind(mx.cpu(), args).forward()[0].asnumpy()
    ref = sym.bind(mx.cpu(), args).forward()[0].asnumpy()
    np.testing.assert_allclose(out, ref, rtol=1e-6)


def test_graph_pass_adds_subgraph_input(subgraph_lib):
    sym = _net()
    args = {'a': mx.nd.ones((3, 2)), 'b': mx.nd.ones((3, 2))}
    part = sym.optimize_for('myProp', args)
    part2 = part.optimize_for('addInputPass', args)
    assert len(part2.list_arguments()) == 3 and '_op0_input' in args       # allocated by the pass
    assert args['_op0_input'].shape == (1,)
    out = part2.bind(mx.cpu(), args).forward()[0].asnumpy()
    np.testing.assert_allclose(out, np.full((3, 2), 2.0), rtol=1e-6)


def test_unknown_backend_is_a_no_op():
    sym = _net()
    assert sym.optimize_for('no_such_backend') is not None


def test_hybridblock_backend_and_pass(subgraph_lib):
    """HybridBlock.hybridize(backend=...) / optimize_for: partitioned cached graph, then a pass whose
    new input the block feeds itself."""
    sym = _net()
    inputs = [mx.sym.var('a'), mx.sym.var('b')]
    blk = mx.gluon.SymbolBlock(sym, inputs)
    blk.initialize()
    a, b = mx.nd.ones((3, 2)), mx.nd.ones((3, 2)) * 2
    ref = np.log(np.exp(a.asnumpy() + b.asnumpy()))
    blk.hybridize(backend='myProp', backend_opts={'dedup_subgraph': True})
    np.testing.assert_allclose(blk(a, b).asnumpy(), ref, rtol=1e-6)
    import json
    ops = [n['op'] for n in json.loads(blk._cached_op.sym.tojson())['nodes']]
    assert '_custom_subgraph_op' in ops
    blk2 = mx.gluon.SymbolBlock(sym, inputs)
    blk2.initialize()
    blk2.optimize_for(a, b, backend='myProp')
    blk2.hybridize(backend='addInputPass', clear=False)
    np.testing.assert_allclose(blk2(a, b).asnumpy(), ref, rtol=1e-6)
