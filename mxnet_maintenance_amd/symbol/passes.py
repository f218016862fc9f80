"""Graph passes applied when a Symbol is bound (the nnvm passes of src/executor/graph_executor.cc).

* ``eliminate_common_expr`` -- common-subexpression elimination (reference
  src/nnvm/eliminate_common_expr.cc, on by default, ``MXNET_ELIMINATE_COMMON_EXPR``): two nodes with
  the same operator, attributes and input entries compute the same value, so the later one is
  dropped and its consumers read the earlier one.  Operators with side effects or random outputs
  (samplers, Dropout, ops that update auxiliary states, Custom) are never merged.  When merging makes
  two graph outputs the same entry, a ``_copy`` keeps them distinct arrays, as the reference does.
* ``fuse_pointwise`` -- pointwise fusion (reference src/executor/pointwise_fusion_pass.cc,
  ``MXNET_USE_FUSION``): maximal single-consumer chains of elementwise operators become one
  ``_FusedOp`` node whose body runs the chain in one go (one HIP kernel on a GPU, see
  ops/fused_ops.py), so the intermediates never reach memory.
* ``memory_plan`` -- bytes of intermediate storage a bound graph needs (forward entries, and the
  gradient buffers when any argument receives a gradient), reported by ``Executor.debug_str`` as the
  reference's "Total N MB allocated".
"""
import os

from ..ops import registry

__all__ = ['eliminate_common_expr', 'fuse_pointwise', 'memory_plan', 'optimize']

# never merged: outputs are random or the op mutates state
_NONDETERMINISTIC_PREFIX = ('_random', '_sample', 'random_', '_npi_random', '_npi_choice', '_npi_shuffle',
                            'sample_', 'Dropout', '_npx_dropout', 'Custom', '_contrib_quantize', '_shuffle', 'shuffle')
# outputs that alias their input (no storage of their own in the memory plan)
_ALIAS_OPS = ('BlockGrad', '_copy', 'Reshape', 'Flatten', 'expand_dims', 'squeeze', 'identity',
              '_npx_reshape', 'reshape_like')


def _cse_ok(node):
    """Whether ``node`` may be merged with an identical node.  As in the reference
    (eliminate_common_expr_pass.cc: nodes without inputs are never grouped, nor ops that request a
    random resource) -- source nodes (zeros, arange, every sampler called with a ``size``) and all
    samplers, including the NumPy ones taking array parameters, stay distinct."""
    if not node.inputs:
        return False
    op = node.opdef()
    if op.get_aux_names(node.parsed()):
        return False
    from ..ndarray.register import _is_sampler
    name = op.name
    if _is_sampler(name) or _is_sampler(node.op):
        return False
    return not any(name.startswith(p) for p in _NONDETERMINISTIC_PREFIX)


def _attr_key(attrs):
    return tuple(sorted((k, str(v)) for k, v in attrs.items() if not (k.startswith('__') and k.endswith('__'))))


def eliminate_common_expr(sym):
    """A new Symbol with duplicate subexpressions merged (the input Symbol is unchanged)."""
    from .symbol import Symbol, _Node
    order = sym._topo()
    remap = {}
    canon = {}
    for n in order:
        if n.op is None:
            remap[id(n)] = n
            continue
        ins = [(remap[id(a)], j) for a, j in n.inputs]
        key = None
        if _cse_ok(n):
            key = (n.op, _attr_key(n.attrs), tuple((id(a), j) for a, j in ins))
            hit = canon.get(key)
            if hit is not None:
                remap[id(n)] = hit
                continue
        nn = _Node(n.op, n.name, n.attrs, ins)
        remap[id(n)] = nn
        if key is not None:
            canon[key] = nn
    outs = []
    seen = set()
    for n, j in sym._outputs:
        e = (remap[id(n)], j)
        k = (id(e[0]), j)
        if k in seen and e[0].op is not None:
            # two outputs became one entry: a copy keeps the output arrays distinct
            cp = _Node('_copy', '%s_copy%d' % (e[0].name, len(outs)), {}, [e])
            e = (cp, 0)
        seen.add(k)
        outs.append(e)
    return Symbol(outs)


# elementwise operators the fusion pass may chain (same-shape in and out, no attributes beyond scalars)
FUSABLE_UNARY = {'relu', 'sigmoid', 'tanh', 'exp', 'log', 'sqrt', 'rsqrt', 'square', 'abs', 'negative',
                 'reciprocal', 'sin', 'cos', 'erf', 'softsign', 'log1p', 'expm1', 'floor', 'ceil', 'round',
                 'trunc', 'sign', 'cbrt', 'rcbrt', 'log2', 'log10', 'gelu'}
FUSABLE_SCALAR = {'_plus_scalar', '_minus_scalar', '_rminus_scalar', '_mul_scalar', '_div_scalar',
                  '_rdiv_scalar', '_power_scalar', '_rpower_scalar', '_maximum_scalar', '_minimum_scalar'}
FUSABLE_BINARY = {'elemwise_add', 'elemwise_sub', 'elemwise_mul', 'elemwise_div', '_plus', '_minus', '_mul',
                  '_div', '_add', '_sub', '_maximum', '_minimum'}


def _fusable(node):
    if node.op is None:
        return False
    name = node.opdef().name
    if name in FUSABLE_UNARY or name in FUSABLE_SCALAR or name in FUSABLE_BINARY:
        return True
    if name == 'Activation':
        return node.parsed().get('act_type') in ('relu', 'sigmoid', 'tanh', 'softrelu', 'softsign')
    return False


def fuse_pointwise(sym, min_ops=2):
    """Group single-consumer chains of elementwise nodes into ``_FusedOp`` nodes.  Each fused node
    carries the chain as a JSON subgraph attribute (``subgraph``) with its external inputs as
    ``data0..dataN`` variables; ops/fused_ops.py compiles it."""
    import json
    from .symbol import Symbol, _Node
    order = sym._topo()
    consumers = {}
    for n in order:
        for a, j in n.inputs:
            consumers.setdefault((id(a), j), []).append(n)
    for n, j in sym._outputs:
        consumers.setdefault((id(n), j), []).append(None)   # graph outputs count as consumers
    group_of = {}
    groups = []
    for n in order:
        if not _fusable(n) or n.num_outputs() != 1:
            continue
        # join the group of a fusable producer whose only consumer is this node
        joined = None
        for a, j in n.inputs:
            g = group_of.get(id(a))
            if g is not None and len(consumers.get((id(a), j), [])) == 1:
                joined = g
                break
        if joined is None:
            joined = []
            groups.append(joined)
        joined.append(n)
        group_of[id(n)] = joined
    fused = [g for g in groups if len(g) >= min_ops]
    if not fused:
        return sym
    in_fused = {id(n): g for g in fused for n in g}
    remap = {}
    built = {}

    def entry(a, j):
        return (remap[id(a)], j) if id(a) in remap else (a, j)

    new_nodes = {}
    for n in order:
        g = in_fused.get(id(n))
        if g is None:
            if n.op is None:
                remap[id(n)] = n
                continue
            nn = _Node(n.op, n.name, n.attrs, [entry(a, j) for a, j in n.inputs])
            remap[id(n)] = nn
            continue
        if id(g[-1]) != id(n):
            continue      # built when the chain's last node is reached (all its inputs exist then)
        members = {id(m) for m in g}
        ext, ext_index = [], {}
        sub_nodes = []
        local = {}
        for m in g:
            ins = []
            for a, j in m.inputs:
                if id(a) in members:
                    ins.append([local[id(a)], j, 0])
                else:
                    k = (id(a), j)
                    if k not in ext_index:
                        ext_index[k] = len(ext)
                        ext.append((a, j))
                        sub_nodes.append({'op': 'null', 'name': 'data%d' % ext_index[k], 'inputs': []})
                        local[('ext',) + k] = len(sub_nodes) - 1
                    ins.append([local[('ext',) + k], 0, 0])
            sub_nodes.append({'op': m.op, 'name': m.name, 'attrs': {k: str(v) for k, v in m.attrs.items()},
                              'inputs': ins})
            local[id(m)] = len(sub_nodes) - 1
        sub = {'nodes': sub_nodes, 'arg_nodes': [i for i, d in enumerate(sub_nodes) if d['op'] == 'null'],
               'heads': [[len(sub_nodes) - 1, 0, 0]], 'attrs': {}}
        fn = _Node('_FusedOp', '%s_fused' % n.name, {'num_inputs': str(len(ext)), 'subgraph': json.dumps(sub)},
                   [entry(a, j) for a, j in ext])
        for m in g:
            remap[id(m)] = fn
        built[id(n)] = fn
    return Symbol([(remap[id(n)], j) if id(n) in remap else (n, j) for n, j in sym._outputs])


def memory_plan(sym, arg_shapes, arg_dtypes, grad_needed):
    """Bytes of intermediate storage: every operator output that is not an alias of its input (views,
    BlockGrad, copies), counted once more for the gradient buffers when any argument gets a gradient."""
    import numpy as np
    internals = sym.get_internals()
    try:
        _, out_shapes, _ = internals.infer_shape_partial(**arg_shapes)
        _, out_types, _ = internals.infer_type_partial(**arg_dtypes)
    except Exception:   # pylint: disable=broad-except
        return 0
    total = 0
    for (n, _i), shp, dt in zip(internals._outputs, out_shapes or [], out_types or []):
        if n.op is None or n.opdef().name in _ALIAS_OPS or not shp:
            continue
        total += int(np.prod(shp)) * np.dtype(dt if dt is not None else np.float32).itemsize
    return total * (2 if grad_needed else 1)


def grad_reachable(sym, wrt):
    """Names in ``wrt`` whose gradient can be non-zero: a path to an output that does not cross a
    gradient-blocking operator (BlockGrad / stop_gradient)."""
    order = sym._topo()
    live = set()
    for n, _ in sym._outputs:
        live.add(id(n))
    for n in reversed(order):
        if id(n) not in live or n.op is None:
            continue
        if n.opdef().name == 'BlockGrad':
            continue
        for a, _ in n.inputs:
            live.add(id(a))
    return [n.name for n in order if n.op is None and id(n) in live and n.name in wrt]


def optimize(sym, ctx=None):
    """The passes a bound graph goes through (env switches as in the reference; pointwise fusion,
    like the reference's, only for GPU contexts)."""
    if os.environ.get('MXNET_ELIMINATE_COMMON_EXPR', '1') != '0':
        sym = eliminate_common_expr(sym)
    on_gpu = ctx is not None and getattr(ctx, 'device_type', 'cpu') == 'gpu'
    if on_gpu and os.environ.get('MXNET_USE_FUSION', '1') != '0' and registry.has('_FusedOp'):
        sym = fuse_pointwise(sym)
    return sym
