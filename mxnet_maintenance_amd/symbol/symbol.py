"""Symbolic graphs.

Parity: python/mxnet/symbol/symbol.py (Symbol, Variable/var, Group, load,
load_json, composition, attributes, list_arguments/outputs/auxiliary_states,
get_internals, get_children, infer_shape(_partial), infer_type, tojson, save,
bind, simple_bind, eval, arithmetic overloads) and the nnvm graph JSON format
(3rdparty/tvm/nnvm/src/pass/saveload_json.cc, including the legacy
``param``/``attr``/``backward_source_id`` layout read by LoadLegacyJSON).

A Symbol is a list of output entries ``(node, index)`` over a DAG of ``_Node``.
Shape/type inference executes the operator implementations on PyTorch ``meta``
tensors, so every registered operator is inferable without a separate
shape function; parameter shapes that cannot be derived forward (weights) come
from the operator's ``infer_params`` hook.
"""
import copy
import json
import math
import warnings

import numpy as np
import torch

from ..attribute import AttrScope
from ..base import NotImplementedForSymbol, MXNetError, numeric_types, torch_dtype, np_dtype, dtype_name
from ..name import NameManager
from ..ops import registry

__all__ = ['Symbol', 'var', 'Variable', 'Group', 'load', 'load_json', 'zeros', 'ones', 'full', 'arange',
           'pow', 'power', 'maximum', 'minimum', 'hypot', 'eye', 'linspace', 'histogram', 'split_v2']

_MXNET_VERSION = 10901


class _Node:
    __slots__ = ('op', 'name', 'attrs', 'inputs', '_parsed', '__weakref__')

    def __init__(self, op, name, attrs=None, inputs=None):
        self.op = op          # OpDef name or None for a variable
        self.name = name
        self.attrs = dict(attrs or {})   # string attributes (op params + user attrs)
        self.inputs = list(inputs or [])  # list of (node, out_index)
        self._parsed = None

    def is_var(self):
        return self.op is None

    def opdef(self):
        return registry.get(self.op)

    def parsed(self):
        if self._parsed is None:
            op = self.opdef()
            params = {k: v for k, v in self.attrs.items()
                      if k in op.params or (op.extra_params and not (k.startswith('__') and k.endswith('__')))}
            self._parsed = op.parse_attrs(params)
        return self._parsed

    def num_outputs(self):
        if self.op is None:
            return 1
        return self.opdef().get_num_outputs(self.parsed())

    def num_visible_outputs(self):
        if self.op is None:
            return 1
        return self.opdef().get_num_visible_outputs(self.parsed())


def _topo(entries):
    order, seen = [], set()
    stack = [(e[0], False) for e in reversed(entries)]
    while stack:
        node, done = stack.pop()
        if done:
            order.append(node)
            continue
        if id(node) in seen:
            continue
        seen.add(id(node))
        stack.append((node, True))
        for inp, _ in reversed(node.inputs):
            if id(inp) not in seen:
                stack.append((inp, False))
    return order


def _aux_var_ids(order):
    aux = set()
    for n in order:
        if n.op is None:
            continue
        if n.op == '_CachedOp':
            # a partitioned subgraph keeps its auxiliary inputs at their original positions
            for i in (int(x) for x in n.attrs.get('aux_indices', '').split(',') if x != ''):
                if i < len(n.inputs) and n.inputs[i][0].op is None:
                    aux.add(id(n.inputs[i][0]))
            continue
        op = n.opdef()
        nargs = len(op.get_arg_names(n.parsed()))
        for i, (inp, _) in enumerate(n.inputs):
            if i >= nargs and inp.op is None:
                aux.add(id(inp))
    return aux


def _attr_lookup(attrs, key):
    if key in attrs:
        return attrs[key]
    dk = '__%s__' % key
    if dk in attrs:
        return attrs[dk]
    if key.startswith('__') and key.endswith('__') and key[2:-2] in attrs:
        return attrs[key[2:-2]]
    return None


class Symbol:
    """Symbolic expression: an ordered list of output entries of a graph."""
    __array_priority__ = 1000.0

    def __init__(self, outputs):
        import ctypes
        if isinstance(outputs, ctypes.c_void_p):
            # a handle filled in by the C-API shim (base._LIB), e.g. MXBuildSubgraphByOpNames
            from ..base import _handle_object
            outputs = _handle_object(outputs)._outputs
        self._outputs = list(outputs)

    # ------------------------------------------------------------ structure
    @property
    def name(self):
        if len(self._outputs) != 1:
            return None
        node, idx = self._outputs[0]
        return node.name

    @property
    def handle(self):
        return self

    def __repr__(self):
        name = self.name
        if name is None:
            return '<Symbol group [%s]>' % ', '.join(s.name for s in self)
        return '<Symbol %s>' % name

    def __iter__(self):
        return (Symbol([o]) for o in self._outputs)

    def __len__(self):
        return len(self._outputs)

    def __copy__(self):
        return self.__deepcopy__(None)

    def __deepcopy__(self, memo):
        return load_json(self.tojson())

    def __getstate__(self):
        return {'json': self.tojson()}

    def __setstate__(self, state):
        self._outputs = load_json(state['json'])._outputs

    def _output(self, i):
        """Output ``i`` as its own Symbol (output selection whatever the indexing mode)."""
        return Symbol([self._outputs[i]])

    def __getitem__(self, index):
        if isinstance(index, str):
            names = self.list_outputs()
            idx = [i for i, n in enumerate(names) if n == index]
            if len(idx) != 1:
                raise ValueError('There are multiple outputs with name "%s"' % index if idx else
                                 'Cannot find output that matches name "%s"' % index)
            index = idx[0]
        from .. import util as _util
        if (_util.is_np_array() and not getattr(self, '_legacy', False)
                and (not isinstance(index, (int, np.integer)) or len(self._outputs) == 1)):
            # numpy semantics: basic indexing of the (single) output, not output selection
            from ..ops.tensor import encode_basic_index
            return _create('_npi_basic_index', [self], {'key': encode_basic_index(index)})
        if isinstance(index, slice):
            return Symbol(self._outputs[index])
        return Symbol([self._outputs[index]])

    def _topo(self):
        return _topo(self._outputs)

    def list_arguments(self):
        order = self._topo()
        aux = _aux_var_ids(order)
        return [n.name for n in order if n.op is None and id(n) not in aux]

    def list_auxiliary_states(self):
        order = self._topo()
        aux = _aux_var_ids(order)
        return [n.name for n in order if n.op is None and id(n) in aux]

    def list_inputs(self):
        return [n.name for n in self._topo() if n.op is None]

    def list_outputs(self):
        names = []
        for node, idx in self._outputs:
            if node.op is None:
                names.append(node.name)
                continue
            op = node.opdef()
            if op.output_names:
                names.append('%s_%s' % (node.name, op.output_names[idx]))
            elif node.num_outputs() == 1 or (idx == 0 and node.num_visible_outputs() == 1):
                # one (visible) output: BatchNorm's mean / var and Dropout's mask are hidden
                names.append(node.name + '_output')
            else:
                names.append('%s_output%d' % (node.name, idx))
        return names

    def as_np_ndarray(self):
        """The same graph viewed with NumPy semantics (``mx.sym.np``); graphs here are
        dtype/shape-polymorphic, so only the array-kind mark changes."""
        if not getattr(self, '_legacy', False):
            return self
        return Symbol(self._outputs)

    def as_nd_ndarray(self):
        """The same graph as a legacy (mx.sym) symbol: marked, so a NumPy-mode HybridBlock can refuse
        outputs that mix the two array kinds, as the reference does."""
        s = Symbol(self._outputs)
        s._legacy = True
        return s

    def get_internals(self):
        """Every visible output of every node (nnvm GetInternals honours FNumVisibleOutputs)."""
        outs = []
        for n in self._topo():
            k = n.num_visible_outputs() if n.op is not None else 1
            for i in range(k):
                outs.append((n, i))
        return Symbol(outs)

    def _gen_atomic_symbol(self):
        """A fresh single-node symbol with this (single-node) symbol's operator and attributes and new
        variables for its inputs (reference symbol.py _gen_atomic_symbol)."""
        node = self._outputs[0][0]
        if node.op is None:
            return Symbol([(_Node(None, node.name, dict(node.attrs)), 0)])
        attrs = {k: v for k, v in node.attrs.items()}
        fresh = _Node(node.op, node.name, attrs, [(_Node(None, '%s_in%d' % (node.name, i)), 0)
                                                  for i in range(len(node.inputs))])
        return Symbol([(fresh, i) for i in range(fresh.num_visible_outputs())])

    def get_children(self):
        """Inputs of every output node, in order (None when there are none: variables)."""
        kids, seen = [], set()
        for node, _ in self._outputs:
            if id(node) not in seen:
                seen.add(id(node))
                kids.extend(node.inputs)
        return Symbol(kids) if kids else None

    def __bool__(self):
        raise NotImplementedForSymbol(self.__bool__, 'bool')

    __nonzero__ = __bool__

    def _var_nodes(self):
        return {n.name: n for n in self._topo() if n.op is None}

    # ------------------------------------------------------------ attributes
    def attr(self, key):
        if len(self._outputs) != 1:
            return None
        return _attr_lookup(self._outputs[0][0].attrs, key)

    def list_attr(self, recursive=False):
        if recursive:
            raise DeprecationWarning('Symbol.list_attr with recursive=True has been deprecated. '
                                     'Please use attr_dict instead.')
        return dict(self._outputs[0][0].attrs)

    def attr_dict(self):
        ret = {}
        for n in self._topo():
            if n.attrs:
                ret[n.name] = dict(n.attrs)
        return ret

    def _set_attr(self, **kwargs):
        for k, v in kwargs.items():
            if not isinstance(v, str):
                raise ValueError('Set Attr only accepts string values')
            for node, _ in self._outputs:
                node.attrs[k] = v
                node._parsed = None

    # ----------------------------------------------------------- composition
    def __call__(self, *args, **kwargs):
        s = copy.deepcopy(self)
        s._compose(*args, **kwargs)
        return s

    def _compose(self, *args, **kwargs):
        name = kwargs.pop('name', None)
        vars_ = self._var_nodes()
        order = self._topo()
        repl = {}
        if args:
            argnames = self.list_arguments()
            for n, a in zip(argnames, args):
                repl[n] = a
        for k, v in kwargs.items():
            if k in vars_:
                repl[k] = v
        for n in order:
            n.inputs = [((repl[i.name]._outputs[0][0], repl[i.name]._outputs[0][1]) if i.op is None and i.name in repl
                         else (i, j)) for i, j in n.inputs]
        self._outputs = [((repl[o.name]._outputs[0]) if o.op is None and o.name in repl else (o, i))
                         for o, i in self._outputs]
        if name and len(self._outputs) == 1:
            self._outputs[0][0].name = name

    # ------------------------------------------------------------ arithmetic
    def _bin(self, other, bop, sop, reverse=False):
        if isinstance(other, Symbol):
            return _create(bop, [other, self] if reverse else [self, other], {})
        if isinstance(other, numeric_types):
            return _create(sop, [self], {'scalar': float(other)})
        raise TypeError('type %s not supported' % str(type(other)))

    def __add__(self, o):
        return self._bin(o, 'elemwise_add', '_plus_scalar')

    __radd__ = __add__

    def __sub__(self, o):
        return self._bin(o, 'elemwise_sub', '_minus_scalar')

    def __rsub__(self, o):
        return self._bin(o, 'elemwise_sub', '_rminus_scalar', reverse=True)

    def __mul__(self, o):
        return self._bin(o, 'elemwise_mul', '_mul_scalar')

    __rmul__ = __mul__

    def __truediv__(self, o):
        return self._bin(o, 'elemwise_div', '_div_scalar')

    def __rtruediv__(self, o):
        return self._bin(o, 'elemwise_div', '_rdiv_scalar', reverse=True)

    __div__ = __truediv__
    __rdiv__ = __rtruediv__

    def __mod__(self, o):
        return self._bin(o, '_mod', '_mod_scalar')

    def __rmod__(self, o):
        return self._bin(o, '_mod', '_rmod_scalar', reverse=True)

    def __pow__(self, o):
        return self._bin(o, '_power', '_power_scalar')

    def __rpow__(self, o):
        return self._bin(o, '_power', '_rpower_scalar', reverse=True)

    def __neg__(self):
        return self.__mul__(-1.0)

    def _cmp(self, o, bop, sop):
        out = self._bin(o, bop, sop)
        from .. import util as _util
        if _util.is_np_array() and not getattr(self, '_legacy', False):
            # numpy semantics: comparisons produce booleans (the legacy ops produce 0 / 1 floats)
            out = _create('Cast', [out], {'dtype': 'bool'})
        return out

    def __eq__(self, o):
        return self._cmp(o, '_equal', '_equal_scalar')

    def __ne__(self, o):
        return self._cmp(o, '_not_equal', '_not_equal_scalar')

    def __gt__(self, o):
        return self._cmp(o, '_greater', '_greater_scalar')

    def __ge__(self, o):
        return self._cmp(o, '_greater_equal', '_greater_equal_scalar')

    def __lt__(self, o):
        return self._cmp(o, '_lesser', '_lesser_scalar')

    def __le__(self, o):
        return self._cmp(o, '_lesser_equal', '_lesser_equal_scalar')

    def __hash__(self):
        return id(self)

    def __abs__(self):
        return _create('abs', [self], {})

    def __getattr__(self, name):
        if name.startswith('__'):
            raise AttributeError(name)
        from ..ndarray.ndarray import _FLUENT
        from .. import util as _util
        if (name in _NP_METHODS and _util.is_np_array() and not vars(self).get('_legacy', False)):
            # numpy-mode symbols: the method is the mx.np function (numpy axis / keepdims semantics,
            # e.g. axis=() reduces nothing), not the legacy operator of the same name
            from .. import numpy as _mnp
            fn = getattr(_mnp, name, None)
            if fn is not None:
                return lambda *a, **k: fn(self, *a, **k)
        if name in _FLUENT and registry.has(_FLUENT[name]):
            opname = _FLUENT[name]
            return lambda *a, **k: _op_func(opname)(self, *a, **k)
        if name in ('reshape', 'transpose', 'flatten', 'expand_dims', 'squeeze', 'astype', 'split',
                    'broadcast_to', 'broadcast_like', 'reshape_like', 'zeros_like', 'ones_like',
                    'slice', 'swapaxes', 'diag'):
            opname = {'reshape': 'Reshape', 'flatten': 'Flatten', 'astype': 'Cast', 'split': 'SliceChannel'}.get(name, name)
            if name != 'astype' and registry.has(name) and registry.get(name) is registry.get(opname):
                opname = name      # the alias the method is named after also names the node (split0)

            from .. import util as _util
            if name == 'flatten' and _util.is_np_array() and not getattr(self, '_legacy', False):
                return lambda *a, **k: _op_func('_npi_ravel')(self)     # ndarray.flatten: 1-D copy

            def f(*a, **k):
                if name == 'reshape' and a:
                    k['shape'] = a[0] if len(a) == 1 and isinstance(a[0], (tuple, list)) else a
                    a = ()
                if name == 'transpose' and a:
                    k['axes'] = a[0] if len(a) == 1 and isinstance(a[0], (tuple, list)) else a
                    a = ()
                if name == 'astype' and a:
                    k['dtype'] = a[0]
                    a = ()
                return _op_func(opname)(self, *a, **k)
            return f
        if name.startswith('_'):
            raise AttributeError(name)
        if not vars(self).get('_legacy', False):
            # np-style symbols take the mx.np functions as methods (x.cumsum(axis=...), x.clip(...))
            from .. import numpy as _mnp
            meth = _mnp.ndarray.__dict__.get(name)      # only ndarray *methods*, never properties
            fn = getattr(_mnp, name, None) if callable(meth) and not isinstance(meth, property) else None
            if callable(fn) and not isinstance(fn, type):
                return lambda *a, **k: fn(self, *a, **k)
        raise AttributeError("'Symbol' object has no attribute '%s'" % name)

    # ----------------------------------------------------------- inference
    def infer_shape(self, *args, **kwargs):
        res = self._infer(args, kwargs, partial=False, what='shape')
        return res

    def infer_shape_partial(self, *args, **kwargs):
        return self._infer(args, kwargs, partial=True, what='shape')

    def infer_type(self, *args, **kwargs):
        return self._infer(args, kwargs, partial=False, what='type')

    def infer_type_partial(self, *args, **kwargs):
        return self._infer(args, kwargs, partial=True, what='type')

    def _infer(self, args, kwargs, partial, what):
        arg_names = self.list_arguments()
        known = {}
        if args:
            for n, v in zip(arg_names, args):
                if v is not None:
                    known[n] = v
        names = set(arg_names) | set(self.list_auxiliary_states())
        for k, v in kwargs.items():
            # names that are not inputs (e.g. op attributes passed along to simple_bind) are ignored,
            # as by the reference's MXSymbolInferShape keyword matching
            if v is not None and k in names:
                known[k] = v
        if what == 'shape':
            shapes, dtypes = {k: tuple(v) for k, v in known.items()}, {}
        else:
            shapes, dtypes = {}, {k: torch_dtype(v) for k, v in known.items()}
        res = infer_graph(self, shapes, dtypes, what=what, partial=partial)
        arg_res, out_res, aux_res = res
        if what == 'shape':
            complete = all(s is not None for s in arg_res + out_res + aux_res)
            if not complete and not partial:
                warnings.warn('Cannot decide shape for some arguments', stacklevel=2)
                return None, None, None
            from ..util import is_np_shape
            empty = None if is_np_shape() else ()      # a completely unknown shape
            fix = lambda l: [s if s is not None else empty for s in l]     # noqa: E731
            return fix(arg_res), fix(out_res), fix(aux_res)
        complete = all(s is not None for s in arg_res + out_res + aux_res)
        if not complete and not partial:
            return None, None, None
        conv = lambda l: [np_dtype(d) if d is not None else None for d in l]
        return conv(arg_res), conv(out_res), conv(aux_res)

    # --------------------------------------------------------- serialization
    def tojson(self, remove_amp_cast=True):
        order = self._topo()
        index = {id(n): i for i, n in enumerate(order)}
        nodes, arg_nodes, row_ptr = [], [], [0]
        for i, n in enumerate(order):
            d = {'op': 'null' if n.op is None else n.op, 'name': n.name,
                 'inputs': [[index[id(a)], j, 0] for a, j in n.inputs]}
            if n.attrs:
                d['attrs'] = {k: str(v) for k, v in n.attrs.items()}
            nodes.append(d)
            if n.op is None:
                arg_nodes.append(i)
            row_ptr.append(row_ptr[-1] + (n.num_outputs() if n.op is not None else 1))
        heads = [[index[id(n)], j, 0] for n, j in self._outputs]
        from ..util import is_np_shape
        gattrs = {'mxnet_version': ['int', _MXNET_VERSION]}
        if is_np_shape():
            gattrs['is_np_shape'] = ['int', 1]
        return json.dumps({'nodes': nodes, 'arg_nodes': arg_nodes, 'node_row_ptr': row_ptr,
                           'heads': heads, 'attrs': gattrs}, indent=2)

    def save(self, fname, remove_amp_cast=True):
        with open(fname, 'w') as f:
            f.write(self.tojson())

    # --------------------------------------------------------------- binding
    def bind(self, ctx, args, args_grad=None, grad_req='write', aux_states=None, group2ctx=None,
             shared_exec=None):
        from ..executor import Executor
        from . import subgraph
        return Executor(subgraph.env_partition(self), ctx, args, args_grad, grad_req, aux_states)

    def _bind(self, *a, **k):
        return self.bind(*a, **k)

    def simple_bind(self, ctx, grad_req='write', type_dict=None, stype_dict=None, group2ctx=None,
                    shared_arg_names=None, shared_exec=None, shared_buffer=None, force_rebind=False, **kwargs):
        from ..executor import Executor
        from .. import ndarray as nd
        arg_shapes, _, aux_shapes = self.infer_shape(**kwargs)
        if arg_shapes is None:
            raise MXNetError('simple_bind: cannot infer shapes from %s' % kwargs)
        arg_names = self.list_arguments()
        type_dict = type_dict or {}
        arg_types, _, aux_types = self.infer_type(**{k: v for k, v in type_dict.items() if k in arg_names})
        if arg_types is None:
            arg_types = [np.float32] * len(arg_names)
            aux_types = [np.float32] * len(aux_shapes)
        args = []
        var_nodes = self._var_nodes()

        def place(name):
            # model parallelism: a variable created under AttrScope(ctx_group=g) lives on group2ctx[g]
            va = var_nodes[name].attrs if name in var_nodes else {}
            g = va.get('__ctx_group__', va.get('ctx_group'))
            return group2ctx[g] if (group2ctx and g in group2ctx) else ctx
        for n, s, t in zip(arg_names, arg_shapes, arg_types):
            if shared_buffer is not None and n in shared_buffer and shared_buffer[n].shape == tuple(s):
                args.append(shared_buffer[n])
            else:
                st = (stype_dict or {}).get(n, 'default')
                a = nd.zeros(s, ctx=place(n), dtype=t or np.float32, stype=st) if st != 'default' else \
                    nd.zeros(s, ctx=place(n), dtype=t or np.float32)
                if shared_buffer is not None:
                    shared_buffer[n] = a
                args.append(a)
        if isinstance(grad_req, str):
            reqs = {n: grad_req for n in arg_names}
        elif isinstance(grad_req, (list, tuple)):
            reqs = dict(zip(arg_names, grad_req))
        else:
            reqs = {n: grad_req.get(n, 'null') for n in arg_names}
        rsp_grads = self._row_sparse_grad_args()
        grads = {n: (nd.zeros(s, ctx=place(n), dtype=t or np.float32, stype='row_sparse') if n in rsp_grads else
                     nd.zeros(s, ctx=place(n), dtype=t or np.float32))
                 for n, s, t in zip(arg_names, arg_shapes, arg_types) if reqs.get(n, 'null') != 'null'}
        aux = [nd.zeros(s, ctx=ctx, dtype=t or np.float32) for s, t in zip(aux_shapes, aux_types)]
        from . import subgraph
        return Executor(subgraph.env_partition(self), ctx, args, grads, reqs, aux)

    def _row_sparse_grad_args(self):
        """Arguments whose gradient storage the backward storage-type inference makes row_sparse:
        the weight of an Embedding with ``sparse_grad`` (src/operator/tensor/indexing_op.cc
        EmbeddingOpBackwardStorageType) when no other consumer needs a dense gradient."""
        rsp, dense = set(), set()
        for n in self._topo():
            if n.op is None:
                continue
            sparse_w = n.op in ('Embedding', '_contrib_SparseEmbedding') and \
                (n.op == '_contrib_SparseEmbedding' or str(n.attrs.get('sparse_grad', 'False')) in ('True', 'true', '1'))
            for k, (src, _j) in enumerate(n.inputs):
                if src.op is not None:
                    continue
                (rsp if (sparse_w and k == 1) else dense).add(src.name)
        return rsp - dense

    def eval(self, ctx=None, **kwargs):
        from ..context import current_context
        ctx = ctx or current_context()
        ex = self.bind(ctx, kwargs)
        return ex.forward()

    def gradient(self, wrt):
        raise NotImplementedError('Symbol.gradient is not supported; use autograd or Executor.backward')

    def debug_str(self):
        lines = []
        for n in self._topo():
            if n.op is None:
                lines.append('Variable:%s' % n.name)
            else:
                lines.append('Op:%s, Name=%s\nInputs:\n%s' % (n.op, n.name, '\n'.join(
                    '\targ[%d]=%s(%d)' % (i, a.name, j) for i, (a, j) in enumerate(n.inputs))))
        return '\n'.join(lines)

    def optimize_for(self, backend, args=None, aux=None, ctx=None, **kwargs):
        """Apply the graph pass or partitioner ``backend`` registered by an extension library
        (library_graph.py: the library sees the graph, ``args`` / ``aux`` and the options in
        ``kwargs``; arrays a pass allocates are added to ``args`` / ``aux`` when they are dicts), or
        partition for a subgraph backend whose operator names were registered
        (MXSetSubgraphPropertyOpNames[V2]); the graph is returned unchanged for unknown backends."""
        from .. import library_graph
        opts = {k: v for k, v in kwargs.items() if k not in ('shape_dict', 'type_dict', 'stype_dict', 'skip_infer')}
        a = args if isinstance(args, dict) else (dict(zip(self.list_arguments(), args)) if args else None)
        x = aux if isinstance(aux, dict) else (dict(zip(self.list_auxiliary_states(), aux)) if aux else None)
        res = library_graph.optimize_for(self, backend, a, x, **opts)
        if res is not None:
            sym, new_args, new_aux = res
            if isinstance(args, dict):
                args.update({k: v for k, v in new_args.items() if k not in args})
            if isinstance(aux, dict):
                aux.update({k: v for k, v in new_aux.items() if k not in aux})
            return sym
        from . import subgraph
        return subgraph.partition_for_backend(self, backend)

    def get_backend_symbol(self, backend):
        return self


# ---------------------------------------------------------------------------
# graph construction
# ---------------------------------------------------------------------------

_NP_METHODS = frozenset(('max', 'min', 'sum', 'mean', 'prod', 'std', 'var', 'argmax', 'argmin', 'cumsum',
                         'clip', 'any', 'all', 'round', 'repeat', 'take', 'dot', 'squeeze', 'swapaxes',
                         'sort', 'argsort', 'nonzero', 'diagonal', 'tile'))


def _create(op_name, inputs, attrs, name=None, attr=None):
    """Create a Symbol applying ``op_name`` to input Symbols (missing args become variables)."""
    op = registry.get(op_name)
    if op.name == '_CachedOp' and attrs.get('subgraph') and 'num_inputs' not in attrs:
        from .subgraph import user_attrs
        attrs = user_attrs(attrs)
    # the default node name follows the name the operator was called by (an alias such as flip
    # names its node flip0, as the reference's generated functions do)
    hint = (op_name if op_name.lower().lstrip('_') else op.name).lower()
    name = NameManager.current.get(name, hint)
    scope_attr = AttrScope.current.get(attr)
    node_attrs = {}
    for k, v in attrs.items():
        if v is None:
            if k in op.params and str(op.params[k][0]).endswith('?') and op.params[k][1] is not None:
                node_attrs[k] = 'None'      # explicit None overriding a non-None default (sort axis)
            continue
        node_attrs[k] = registry.format_value(v) if not isinstance(v, str) else v
    for k, v in (scope_attr or {}).items():
        node_attrs[k] = v
        if not (k.startswith('__') and k.endswith('__')):
            node_attrs['__%s__' % k] = v
    node = _Node(op.name, name, node_attrs)
    parsed = node.parsed()
    arg_names = op.get_arg_names(parsed)
    aux_names = op.get_aux_names(parsed)
    entries = []
    if isinstance(inputs, dict):
        pos, named = inputs.get('_pos', []), {k: v for k, v in inputs.items() if k != '_pos'}
    else:
        pos, named = inputs, {}
    all_names = arg_names + aux_names
    # hidden attributes (lr_mult, wd_mult, ctx_group, ... from the call or the AttrScope) are inherited by the
    # variables created for missing inputs, like nnvm's Compose does for the op's auto-named arguments
    var_attrs = {(k if k.startswith('__') and k.endswith('__') else '__%s__' % k): v
                 for k, v in (scope_attr or {}).items()}
    default_init = _COMPOSE_VAR_INIT.get(op.name, {})
    for i, an in enumerate(all_names):
        s = None
        if i < len(pos):
            s = pos[i]
        elif an in named:
            s = named[an]
        if s is None:
            v = _Node(None, '%s_%s' % (name, an), dict(var_attrs))
            entries.append((v, 0))
        else:
            if len(s._outputs) != 1:
                raise MXNetError('Cannot compose a grouped symbol as input %s of %s' % (an, name))
            entries.append(s._outputs[0])
        src = entries[-1][0]
        if i in default_init and src.is_var() and '__init__' not in src.attrs:
            src.attrs['__init__'] = default_init[i]
    for s in pos[len(all_names):]:
        if s is not None:       # e.g. an explicit None bias of a no_bias Convolution
            entries.append(s._outputs[0])
    node.inputs = entries
    nvis = node.num_visible_outputs()
    out = Symbol([(node, i) for i in range(nvis)])
    if any(getattr(x, '_legacy', False) for x in list(pos) + list(named.values()) if isinstance(x, Symbol)):
        out._legacy = True
    return out


# Initializers that operators give their input variables at compose time when the variable has none
# (nnvm FSetInputVarAttrOnCompose; reference src/operator/leaky_relu.cc:203, nn/batch_norm.cc:668,
# nn/upsampling.cc:205): PReLU slope 0.25, BatchNorm moving mean 0 / moving var 1, bilinear upsampling kernel.
_COMPOSE_VAR_INIT = {
    'LeakyReLU': {1: '["Constant", {"value": 0.25}]'},
    'BatchNorm': {3: '["zero", {}]', 4: '["one", {}]'},
    'UpSampling': {1: '["bilinear", {}]'},
}


def _op_func(op_name):
    op = registry.get(op_name)

    def f(*args, **kwargs):
        name = kwargs.pop('name', None)
        attr = kwargs.pop('attr', None)
        kwargs.pop('out', None)
        pos = []
        extra_pos = []
        for a in args:
            if isinstance(a, Symbol) and not extra_pos:
                pos.append(a)
            elif isinstance(a, (list, tuple)) and a and all(isinstance(x, Symbol) for x in a) and not extra_pos:
                pos.extend(a)
            elif a is None and not extra_pos:
                pos.append(None)
            elif isinstance(a, Symbol):
                raise TypeError('%s: Symbol inputs must precede positional parameters' % op_name)
            else:
                extra_pos.append(a)
        named = {k: v for k, v in kwargs.items() if isinstance(v, Symbol)}
        # an explicit None for an optional parameter (e.g. sort axis=None: flatten) is kept
        attrs = {k: v for k, v in kwargs.items() if not isinstance(v, Symbol) and (
            v is not None or (k in op.params and isinstance(op.params[k][0], str) and op.params[k][0].endswith('?')
                              and op.params[k][1] is not None))}
        if extra_pos:
            # positional attribute values follow the declared param order (as in the nd frontend)
            for p, v in zip([p for p in op.params if p not in attrs], extra_pos):
                attrs[p] = v
        extra = {}
        for k in list(attrs):
            if k not in op.params and k != op.key_var_num_args:
                if k in ('lr_mult', 'wd_mult', 'ctx_group', 'force_mirroring', 'init', 'dtype_hint',
                         'mirror_stage', 'storage_type'):
                    extra[k] = str(attrs.pop(k))
        if op.key_var_num_args and op.key_var_num_args not in attrs:
            attrs[op.key_var_num_args] = len(pos) + len(named)
        if 'dtype' in attrs and attrs['dtype'] is not None and not isinstance(attrs['dtype'], str):
            attrs['dtype'] = dtype_name(attrs['dtype'])
        if extra:
            attr = dict(attr or {})
            for k, v in extra.items():
                attr[k] = v
        inputs = {'_pos': pos}
        inputs.update(named)
        return _create(op_name, inputs, attrs, name=name, attr=attr)
    f.__name__ = op_name
    return f


def var(name, attr=None, shape=None, lr_mult=None, wd_mult=None, dtype=None, init=None, stype=None,
        **kwargs):
    """Create a symbolic variable."""
    if not isinstance(name, str):
        raise TypeError('Expect a string for variable `name`')
    attr = AttrScope.current.get(attr)
    attrs = {}
    for k, v in (attr or {}).items():
        attrs[k] = v
    if shape is not None:
        attrs['__shape__'] = registry.format_value((shape,) if isinstance(shape, (int, np.integer))
                                                   else tuple(shape))
    if lr_mult is not None:
        attrs['__lr_mult__'] = str(lr_mult)
    if wd_mult is not None:
        attrs['__wd_mult__'] = str(wd_mult)
    if dtype is not None:
        # the reference stores the mshadow type flag (python/mxnet/symbol/symbol.py var())
        from ..base import dtype_to_flag
        attrs['__dtype__'] = str(dtype_to_flag(dtype))
    if init is not None:
        if not isinstance(init, str):
            init = init.dumps()
        attrs['__init__'] = init
    if stype is not None:
        from ..ndarray.ndarray import _STORAGE_TYPE_STR_TO_ID
        attrs['__storage_type__'] = str(_STORAGE_TYPE_STR_TO_ID.get(stype, stype))
    for k, v in kwargs.items():
        if k.startswith('__') and k.endswith('__'):
            attrs[k] = str(v)
        else:
            raise ValueError('Attribute name=%s is not supported. Additional attributes must start and '
                             'end with double underscores, e.g, __yourattr__' % k)
    return Symbol([(_Node(None, name, attrs), 0)])


Variable = var


def Group(symbols, create_fn=None):
    if not symbols or any(not isinstance(s, Symbol) for s in symbols):
        raise TypeError('Expected a list of symbols as input')
    outs = []
    for s in symbols:
        outs.extend(s._outputs)
    return Symbol(outs)


def load_json(json_str):
    """Load a Symbol from MXNet JSON (current nnvm layout and the legacy 0.8 layout)."""
    g = json.loads(json_str)
    nodes = []
    for nd_ in g['nodes']:
        op = nd_['op']
        attrs = {}
        for key in ('attrs', 'attr', 'param'):
            if key in nd_ and nd_[key]:
                attrs.update({k: str(v) for k, v in nd_[key].items()})
        if 'attr' in nd_ and nd_['attr']:
            for k, v in nd_['attr'].items():
                if not (k.startswith('__') and k.endswith('__')):
                    attrs['__%s__' % k] = str(v)
        node = _Node(None if op == 'null' else op, nd_['name'], attrs)
        if op != 'null' and not registry.has(op):
            raise MXNetError('Operator %s is not registered' % op)
        node.inputs = [(nodes[e[0]], e[1]) for e in nd_['inputs']]
        nodes.append(node)
    # legacy files: ops whose implicit aux inputs were not serialised
    heads = g.get('heads')
    if heads is None:
        heads = [[len(nodes) - 1, 0, 0]]
    return Symbol([(nodes[h[0]], h[1]) for h in heads])


def load(fname):
    with open(fname) as f:
        return load_json(f.read())


# ---------------------------------------------------------------------------
# shape/type inference
# ---------------------------------------------------------------------------

def _attr_shape(node):
    s = node.attrs.get('__shape__')
    if s is None:
        return None
    t = registry.parse_value('shape', s)
    if t is None or any(d == 0 for d in t) or len(t) == 0:
        return None
    return t


def _partial_attr_shape(node):
    """A variable's declared shape when it has some (not all) unknown dims."""
    v = node.attrs.get('__shape__')
    if v is None:
        return None
    t = registry.parse_value('shape', v)
    if not t or all(int(d) <= 0 for d in t) or all(int(d) > 0 for d in t):
        return None
    return t


def _attr_dtype(node):
    d = node.attrs.get('__dtype__')
    if d is None:
        return None
    try:
        if isinstance(d, str) and d.lstrip('-').isdigit():
            from ..base import flag_to_dtype
            return flag_to_dtype(int(d)) if int(d) >= 0 else None
        return torch_dtype(d)
    except Exception:
        return None


def _run_meta(op, parsed, shapes, dtypes):
    ins = []
    for s, d in zip(shapes, dtypes):
        if s is None:
            ins.append(None)
        else:
            ins.append(torch.empty(s, dtype=d or torch.float32, device='meta'))
    kw = dict(parsed)
    for k in ('ctx',):
        if k in kw:
            kw[k] = None
    try:
        with torch.no_grad():
            out = op.fn(*ins, **kw)
    except Exception:
        # ops with data-dependent host logic: run on small zero CPU tensors
        if any(s is not None and int(np.prod(s)) > (1 << 22) for s in shapes):
            raise
        ins = [None if s is None else torch.zeros(s, dtype=d or torch.float32) for s, d in zip(shapes, dtypes)]
        with torch.no_grad():
            out = op.fn(*ins, **kw)
    if not isinstance(out, (tuple, list)):
        out = [out]
    return [(tuple(o.shape), o.dtype) for o in out]


_SHAPE_PRESERVING = ('Cast', 'cast', 'amp_cast', 'amp_multicast', '_copy', 'identity', 'BlockGrad',
                     'stop_gradient')

_ELEMWISE_BINARY = frozenset(['elemwise_add', 'elemwise_sub', 'elemwise_mul', 'elemwise_div', '_grad_add', '_plus',
                              '_minus', '_mul', '_div', '_add', '_sub', 'add_n', 'ElementWiseSum', '_maximum',
                              '_minimum', '_power', '_hypot'])

_SAME_SHAPE = frozenset(['elemwise_add', 'elemwise_sub', 'elemwise_mul', 'elemwise_div', '_grad_add', '_plus',
                         '_minus', '_mul', '_div', '_add', '_sub', 'add_n', 'ElementWiseSum', '_maximum', '_minimum',
                         '_power', '_hypot', 'Activation', 'relu', 'sigmoid', 'tanh', 'softsign', 'Dropout',
                         'BlockGrad', 'stop_gradient', 'identity', '_copy', 'make_loss', 'MakeLoss', 'negative',
                         'abs', 'exp', 'log', 'sqrt', 'square', 'sin', 'cos', 'tan', 'arcsin', 'arccos',
                         'arctan', 'sinh', 'cosh', 'arcsinh', 'arccosh', 'arctanh', 'degrees', 'radians',
                         'expm1', 'log1p', 'log2', 'log10', 'rsqrt', 'cbrt', 'rcbrt', 'reciprocal', 'sign',
                         'round', 'rint', 'ceil', 'floor', 'trunc', 'fix', 'erf', 'erfinv', 'gamma', 'gammaln',
                         'LeakyReLU', 'softrelu', 'clip', 'zeros_like', 'ones_like', '_FusedOp',
                         '_identity_with_attr_like_rhs'])

_INIT_OPS = ('_zeros', '_ones', '_full', '_empty', 'zeros', 'ones', 'full')


def _unify_shapes(order, seeds):
    """Unify partial shapes across the graph (nnvm's bidirectional InferShape, unknown dims <= 0):
    elementwise ops share one shape, transposes permute it, shape-preserving ops pass it through,
    and a Reshape whose output is known sizes the one unknown dim of its input -- in both
    directions, until nothing changes.  ``seeds``: (id(node), 0) -> partial shape.  Returns the
    (id(node), out) -> partial shape map (unknown dims -1)."""
    part = {}
    memo = {}

    def merge(key, s):
        if s is None:
            return False
        s = tuple(int(d) if int(d) > 0 else -1 for d in s)
        cur = part.get(key)
        if cur is None:
            part[key] = s
            return True
        if len(cur) != len(s):
            return False
        new = tuple(c if c > 0 else d for c, d in zip(cur, s))
        if new != cur:
            part[key] = new
            return True
        return False

    full = lambda t: t is not None and all(d > 0 for d in t)     # noqa: E731
    for k, v in seeds.items():
        merge(k, v)
    for n in order:
        if n.op in _INIT_OPS and 'shape' in n.attrs and n.parsed().get('shape'):
            merge((id(n), 0), n.parsed()['shape'])
        elif n.op is None and n.attrs.get('__shape__'):
            merge((id(n), 0), registry.parse_value('shape', n.attrs['__shape__']))
    for _ in range(len(order) + 1):
        changed = False
        for n in order:
            if n.op is None or not n.inputs:
                continue
            keys = [(id(a), j) for a, j in n.inputs]
            out = (id(n), 0)
            if n.op in _SAME_SHAPE or n.op in _SHAPE_PRESERVING:
                group = (keys if n.op in _SAME_SHAPE else keys[:1]) + [out]
                for k in group:
                    for k2 in group:
                        if k2 != k and part.get(k2) is not None:
                            changed |= merge(k, part[k2])
            elif n.op == 'transpose' and len(keys) == 1:
                axes = tuple(n.parsed().get('axes') or ())
                src = part.get(keys[0])
                dst = part.get(out)
                nd = len(src) if src is not None else (len(dst) if dst is not None else 0)
                if not nd:
                    continue
                axes = axes or tuple(range(nd - 1, -1, -1))
                if src is not None:
                    changed |= merge(out, tuple(src[a] for a in axes))
                if dst is not None:
                    inv = [0] * nd
                    for i, a in enumerate(axes):
                        inv[a] = dst[i]
                    changed |= merge(keys[0], tuple(inv))
            elif n.op in ('Reshape', 'reshape') and len(keys) == 1:
                src, dst = part.get(keys[0]), part.get(out)
                if full(src) and not full(dst):
                    try:
                        o = _run_meta(n.opdef(), n.parsed(), [src], [torch.float32])
                        changed |= merge(out, o[0][0])
                    except Exception:   # pylint: disable=broad-except
                        pass
                elif full(dst) and src is not None and sum(1 for d in src if d <= 0) == 1:
                    known = math.prod(d for d in src if d > 0)
                    total = math.prod(dst)
                    if known and total % known == 0:
                        changed |= merge(keys[0], tuple(d if d > 0 else total // known for d in src))
                elif src is not None and dst is None:
                    # partial input: the output dims that do not move with the unknown ones are known
                    # (e.g. reshape(-1) of an RNN weight with unknown input size gives (-1,), so the
                    # parameter concatenation downstream can solve for it backwards)
                    try:
                        a_ = _run_meta(n.opdef(), n.parsed(), [_subst([src], _PROBES[0])[0]], [torch.float32])[0][0]
                        b_ = _run_meta(n.opdef(), n.parsed(), [_subst([src], _PROBES[1])[0]], [torch.float32])[0][0]
                        if len(a_) == len(b_):
                            changed |= merge(out, tuple(x if x == y else -1 for x, y in zip(a_, b_)))
                    except Exception:   # pylint: disable=broad-except
                        pass
            elif n.op not in _PROBE_SKIP:
                changed |= _probe_node(n, keys, part, merge, memo)
        if not changed:
            break
    return part


# ---- probing: partial shape inference through any operator's own shape function ----------------
# nnvm lets every operator infer shapes both ways with unknown dims.  Here each operator has one
# forward shape function (its meta-tensor execution), so unknown dims are *probed*: run the function
# with the unknown dims set to two different values; output dims that do not move are known.  The
# inverse direction solves for an input dim: an output dim that moves linearly with it and is known
# downstream determines it (checked by re-running the function with the solution).
_PROBES = (509, 521)
_PROBE_SKIP = frozenset(['where', '_npi_where'])      # the reference needs a fully known condition
_PROBE_MAX_ELEMS = 1 << 34


def _probe_eval(n, shapes):
    """Output shapes of node ``n`` for fully known input shapes, or None when the op rejects them."""
    if any(math.prod(s) > _PROBE_MAX_ELEMS for s in shapes):
        return None
    try:
        return [o[0] for o in _run_meta(n.opdef(), n.parsed(), shapes, [torch.float32] * len(shapes))]
    except Exception:   # pylint: disable=broad-except
        return None


def _probe_params(n, shapes):
    """Parameter shapes an operator derives from its (fully known) data shapes, or {}."""
    fn = n.opdef().infer_params
    if fn is None:
        return {}
    try:
        return {i: tuple(int(d) for d in v) for i, v in fn(shapes, n.parsed()).items()}
    except Exception:   # pylint: disable=broad-except
        return {}


def _subst(shapes, value, only=None):
    """Unknown dims (-1) replaced by ``value`` (``only``: just that (input, dim); others get probe 0)."""
    out = []
    for i, s in enumerate(shapes):
        row = []
        for d, v in enumerate(s):
            if v > 0:
                row.append(v)
            elif only is None or only == (i, d):
                row.append(value)
            else:
                row.append(_PROBES[0])
        out.append(tuple(row))
    return out


def _probe_node(n, keys, part, merge, memo):
    ins = [part.get(k) for k in keys]
    nout = n.num_outputs()
    outs = [part.get((id(n), i)) for i in range(nout)]
    sig = (tuple(ins), tuple(outs))
    if memo.get(id(n)) == sig:
        return False
    memo[id(n)] = sig
    changed = False
    # parameters (weights, biases) from partially known data: probe the data dims
    if ins and ins[0] is not None and any(s is None or any(v <= 0 for v in s) for s in ins[1:]):
        def filled(v):
            return [None if x is None else _subst([x], v)[0] for x in ins]
        a = _probe_params(n, filled(_PROBES[0]))
        b = _probe_params(n, filled(_PROBES[1]))
        for idx in a:
            if (idx < len(keys) and idx > 0 and (ins[idx] is None or any(v <= 0 for v in ins[idx])) and idx in b
                    and len(a[idx]) == len(b[idx])):
                changed |= merge(keys[idx], tuple(x if x == y else -1 for x, y in zip(a[idx], b[idx])))
        ins = [part.get(k) for k in keys]
    if not ins or any(s is None for s in ins):
        return changed
    unknown = [(i, d) for i, s in enumerate(ins) for d, v in enumerate(s) if v <= 0]
    if not unknown:
        res = _probe_eval(n, list(ins))
        if res is not None:
            for i, o in enumerate(res[:nout]):
                changed |= merge((id(n), i), o)
        return changed
    # forward: dims of the outputs that do not depend on the unknown input dims
    r1 = _probe_eval(n, _subst(ins, _PROBES[0]))
    r2 = _probe_eval(n, _subst(ins, _PROBES[1]))
    if r1 is not None and r2 is not None and len(r1) == len(r2):
        for i, (a, b) in enumerate(zip(r1[:nout], r2[:nout])):
            if len(a) == len(b):
                changed |= merge((id(n), i), tuple(x if x == y else -1 for x, y in zip(a, b)))
    # backward: solve unknown input dims from known output dims (all together first, then one by one)
    outs = [part.get((id(n), i)) for i in range(nout)]
    if not any(o is not None and any(v > 0 for v in o) for o in outs):
        return changed
    for only in [None] + unknown:
        sol = _solve_dim(n, ins, outs, only)
        if sol is None:
            continue
        for i, s in enumerate(ins):
            new = tuple(sol if (v <= 0 and (only is None or only == (i, d))) else v for d, v in enumerate(s))
            changed |= merge(keys[i], new)
        if only is None:
            break
        ins = [part.get(k) for k in keys]
    return changed


def _solve_dim(n, ins, outs, only):
    """The value of the probed unknown dim(s) that reproduces every known output dim, or None."""
    p0, p1 = _PROBES
    ra = _probe_eval(n, _subst(ins, p0, only))
    rb = _probe_eval(n, _subst(ins, p1, only))
    if ra is None or rb is None:
        return None
    cands = set()
    for o, a, b in zip(outs, ra, rb):
        if o is None or len(o) != len(a) or len(a) != len(b):
            continue
        for t, x, y in zip(o, a, b):
            if t > 0 and x != y:
                slope = (y - x) / float(p1 - p0)
                v = p0 + (t - x) / slope
                for c in (math.floor(v), math.ceil(v), math.floor(v) - 1):
                    if c >= 1:
                        cands.add(int(c))
    for c in sorted(cands):
        r = _probe_eval(n, _subst(ins, c, only))
        if r is None:
            continue
        # every known output dim that depends on the probed dim(s) must come out right
        if all(o is None or (len(o) == len(x) and all(t <= 0 or xa == xb or t == v
                                                        for t, v, xa, xb in zip(o, x, a, b)))
               for o, x, a, b in zip(outs, r, ra, rb)):
            return c
    return None


def _unify_init_shapes(order):
    """Size init ops declared with unknown dims (0, or -1) from their consumers (_unify_shapes);
    fully resolved ones get the shape written into their ``shape`` attribute."""
    inits = [n for n in order if n.op in _INIT_OPS and 'shape' in n.attrs and n.parsed().get('shape')
             and any(int(d) <= 0 for d in n.parsed()['shape'])]
    if not inits:
        return
    part = _unify_shapes(order, {})
    for n in inits:
        s = part.get((id(n), 0))
        if s is not None and all(d > 0 for d in s):
            n.attrs['shape'] = str(s)
            n._parsed = None


def _resolve_unknown_init_shapes(sym, order, known_shapes, known_dtypes, what, partial=False):
    """Init ops declared with 0 (unknown) dims, e.g. RNN ``begin_state`` via ``sym.zeros``.

    The reference fills those dims by backward shape inference; here the
    candidate sizes are the dims of the known argument shapes, and the first
    candidate under which the whole graph infers consistently is written
    back into the node's ``shape`` attribute (so executors allocate it).
    """
    _unify_init_shapes(order)
    loop_data = set()
    for n in order:
        if n.op == '_foreach':
            ndata = len(json.loads(n.parsed().get('data_names') or '[]'))
            loop_data.update(id(a) for a, _ in n.inputs[:ndata])
    zero_nodes = []
    zero_vars = []      # variables declared with unknown (0) dims, e.g. RNN begin_state(func=Variable)
    for n in order:
        if n.op in _INIT_OPS and 'shape' in n.attrs:
            shp = n.parsed().get('shape')
            if shp and any(int(d) <= 0 for d in shp):
                shp = tuple(max(int(d), 0) for d in shp)
                zero_nodes.append((n, tuple(int(d) for d in shp)))
        elif n.op is None and n.name not in known_shapes and n.attrs.get('__shape__') and not (
                partial and id(n) in loop_data):
            # (the unknown sequence length of a foreach's data stays unknown in partial inference)
            shp = registry.parse_value('shape', n.attrs['__shape__'])
            if shp and any(int(d) == 0 for d in shp) and not all(int(d) == 0 for d in shp):
                zero_vars.append((n, tuple(int(d) for d in shp)))
    if not zero_nodes and not zero_vars:
        return None
    cands = sorted({int(d) for s in known_shapes.values() if s for d in s if int(d) >= 1})
    aux = _aux_var_ids(order)
    arg_nodes = [n for n in order if n.op is None and id(n) not in aux]
    complete = lambda r: all(x is not None for part in r for x in part)     # noqa: E731
    for v in cands:
        for n, shp in zero_nodes:
            n.attrs['shape'] = str(tuple(d if d else v for d in shp))
            n._parsed = None
        try:
            res = infer_graph(sym, known_shapes, known_dtypes, what, _resolve=False)
        except MXNetError:
            continue
        if not zero_vars or complete(res):
            return res
        # only variables the graph could not size itself (e.g. RNN states) take the candidate
        unresolved = {n.name for n, r in zip(arg_nodes, res[0]) if r is None}
        ks = dict(known_shapes)
        for n, shp in zero_vars:
            if n.name in unresolved:
                ks[n.name] = tuple(d if d else v for d in shp)
        try:
            res = infer_graph(sym, ks, known_dtypes, what, _resolve=False)
        except MXNetError:
            continue
        if complete(res):
            return res
    for n, shp in zero_nodes:
        n.attrs['shape'] = str(shp)
        n._parsed = None
    return None


def _unknown_dims(s):
    """True when a shape has unknown dims (-1 under np-shape semantics, 0 in legacy mode)."""
    from .. import util
    unk = -1 if util.is_np_shape() else 0
    return s is not None and any(int(d) == unk or int(d) < 0 for d in s)


def _slice_dim(dim, b, e, st):
    from .. import util
    if int(dim) == (-1 if util.is_np_shape() else 0) or int(dim) < 0:
        return int(dim)
    return len(range(*slice(b, e, st).indices(int(dim))))


def _partial_slice(d, a):
    """slice on a partially known shape: sliced axes of unknown extent stay unknown
    (reference src/operator/tensor/matrix_op-inl.h SliceOpShape)."""
    begin, end, step = tuple(a.get('begin') or ()), tuple(a.get('end') or ()), tuple(a.get('step') or ())
    out = []
    for i, dim in enumerate(d):
        if i >= len(begin):
            out.append(int(dim))
            continue
        st = step[i] if i < len(step) and step[i] is not None else 1
        out.append(_slice_dim(dim, begin[i], end[i] if i < len(end) else None, st))
    return tuple(out)


def _partial_slice_axis(d, a):
    ax = int(a.get('axis', 0)) % len(d)
    out = [int(x) for x in d]
    out[ax] = _slice_dim(d[ax], a.get('begin', 0), a.get('end'), 1)
    return tuple(out)


_PARTIAL_OUT = {'slice': _partial_slice, 'crop': _partial_slice, '_slice': _partial_slice,
                'slice_axis': _partial_slice_axis}


def _subgraph_same_shape(node):
    from .subgraph import same_shape
    return same_shape(node)


def _partial_zero_dims(order, shape):
    """Partial inference with unknown (0) dims: a variable declared with some 0 dims keeps that
    partial shape, shape-preserving ops (casts, copies) pass it on, and operators with parameter
    inference size their parameters from it (unknown dims stay 0), as nnvm's partial InferShape does."""
    def back_fill(a, j, s):
        while True:
            if (id(a), j) not in shape:
                shape[(id(a), j)] = s
            if a.op in _SHAPE_PRESERVING and a.inputs:
                a, j = a.inputs[0]
                continue
            return
    for n in order:
        if n.op is None:
            if (id(n), 0) not in shape and n.attrs.get('__shape__'):
                t = registry.parse_value('shape', n.attrs['__shape__'])
                if t and any(int(d) == 0 for d in t):
                    shape[(id(n), 0)] = tuple(int(d) for d in t)
            continue
        if n.op in _SHAPE_PRESERVING and n.inputs and (id(n), 0) not in shape:
            src = shape.get((id(n.inputs[0][0]), n.inputs[0][1]))
            if src is not None:
                shape[(id(n), 0)] = src
            continue
        op = n.opdef()
        in_shapes = [shape.get((id(a), j)) for a, j in n.inputs]
        if n.op in _PARTIAL_OUT and in_shapes and in_shapes[0] is not None and (id(n), 0) not in shape:
            shape[(id(n), 0)] = _PARTIAL_OUT[n.op](in_shapes[0], n.parsed())
            continue
        if op.infer_params is None or not in_shapes or in_shapes[0] is None or all(in_shapes):
            continue
        try:
            fill = op.infer_params(in_shapes, n.parsed())
        except Exception:   # pylint: disable=broad-except
            continue
        for idx, s in fill.items():
            if idx < len(n.inputs) and in_shapes[idx] is None:
                a, j = n.inputs[idx]
                back_fill(a, j, tuple(int(d) for d in s))


def infer_graph(sym, known_shapes, known_dtypes, what='shape', _resolve=True, partial=False):
    """Propagate shapes and dtypes through the graph.

    Returns (arg_list, out_list, aux_list) of shapes (or dtypes), None for unknown.
    """
    order = sym._topo()
    part = None
    partial_attr = any(n.op is None and n.name not in known_shapes and _partial_attr_shape(n) for n in order)
    if what == 'shape' and (partial_attr or (known_shapes and any(any(int(d) <= 0 for d in v)
                                                                  for v in known_shapes.values() if v))):
        # arguments with unknown dims (given or declared): size what the graph determines by
        # bidirectional unification / probing; the rest stays partial
        byname = {n.name: n for n in order if n.op is None}
        seeds = {(id(byname[k]), 0): v for k, v in known_shapes.items() if k in byname and v}
        part = _unify_shapes(order, seeds)
        known_shapes = dict(known_shapes)
        for name, node in byname.items():
            r = part.get((id(node), 0))
            if r is not None and len(r) and all(d > 0 for d in r):
                known_shapes[name] = r
    if _resolve and what == 'shape' and known_shapes:
        res = _resolve_unknown_init_shapes(sym, order, known_shapes, known_dtypes, what, partial)
        if res is not None:
            return res
    shape = {}   # (id(node), idx) -> shape
    dtype = {}
    for n in order:
        if n.op is None:
            s = known_shapes.get(n.name, _attr_shape(n))
            if s is not None:
                shape[(id(n), 0)] = tuple(s)
            d = known_dtypes.get(n.name, _attr_dtype(n))
            if d is not None:
                dtype[(id(n), 0)] = d
    default_dt = torch.float32
    if known_dtypes:
        default_dt = next(iter(known_dtypes.values()))
    progress = True
    done = set()
    while progress:
        progress = False
        for n in order:
            if n.op is None or id(n) in done:
                continue
            op = n.opdef()
            parsed = n.parsed()
            in_shapes = [shape.get((id(a), j)) for a, j in n.inputs]
            if (any(s is None for s in in_shapes) and op.infer_params is not None and in_shapes
                    and (in_shapes[0] is not None or (n.op == '_CachedOp' and any(in_shapes)))):
                try:
                    fill = op.infer_params(in_shapes, parsed)
                except Exception:
                    fill = {}
                for idx, s in fill.items():
                    if (idx < len(n.inputs) and in_shapes[idx] is not None and len(s) and len(in_shapes[idx])
                            and all(int(d) > 0 for d in in_shapes[idx]) and all(int(d) > 0 for d in s)
                            and tuple(int(d) for d in in_shapes[idx]) != tuple(int(d) for d in s)):
                        raise MXNetError('Error in operator %s (%s): shape inconsistent for input %d: '
                                         'provided %s, inferred %s' % (n.name, n.op, idx, tuple(in_shapes[idx]),
                                                                       tuple(s)))
                    if idx < len(n.inputs) and in_shapes[idx] is None:
                        a, j = n.inputs[idx]
                        shape[(id(a), j)] = tuple(s)
                        in_shapes[idx] = tuple(s)
                        progress = True
                        # shape-preserving producers (casts inserted by AMP, copies): the
                        # parameter behind them has the same shape
                        while a.op in _SHAPE_PRESERVING and a.inputs:
                            a, j = a.inputs[j if a.op == 'amp_multicast' else 0]
                            if (id(a), j) in shape:
                                break
                            shape[(id(a), j)] = tuple(s)
            if any(s is None for s in in_shapes) and (n.op in _SAME_SHAPE or (
                    n.op == '_CachedOp' and _subgraph_same_shape(n))):
                # elementwise ops (nnvm ElemwiseShape): every input and output has one shape, so a
                # known one fills the others (backward inference into unknown producers)
                ref = next((s for s in in_shapes + [shape.get((id(n), 0))] if s is not None), None)
                if ref is not None:
                    for idx, (a, j) in enumerate(n.inputs):
                        if in_shapes[idx] is None:
                            shape[(id(a), j)] = ref
                            in_shapes[idx] = ref
                            progress = True
            if any(s is None for s in in_shapes):
                if what == 'type':
                    # dtype-only propagation: parameters follow the data dtype, outputs
                    # follow the first input unless the op declares an output dtype.
                    in_dt = [dtype.get((id(a), j)) for a, j in n.inputs]
                    base_dt = next((d for d in in_dt if d is not None), None)
                    if base_dt is None and n.op in ('Cast', 'cast', 'amp_cast') and parsed.get('dtype'):
                        # a cast fixes its output type whatever the input is
                        if (id(n), 0) not in dtype:
                            dtype[(id(n), 0)] = torch_dtype(parsed['dtype'])
                            progress = True
                        continue
                    if base_dt is None:
                        continue
                    for (a, j) in n.inputs:
                        if (id(a), j) not in dtype and a.op is None:
                            dtype[(id(a), j)] = base_dt
                    odt = parsed.get('dtype') if n.op in ('Cast', 'cast', 'amp_cast') else None
                    odt = torch_dtype(odt) if odt else base_dt
                    for i in range(n.num_outputs()):
                        if (id(n), i) not in dtype:
                            dtype[(id(n), i)] = odt
                            progress = True
                continue
            in_dt = [dtype.get((id(a), j)) for a, j in n.inputs]
            base_dt = next((d for d in in_dt if d is not None), default_dt)
            in_dt = [d if d is not None else base_dt for d in in_dt]
            # parameters follow the data dtype unless declared
            for (a, j), d in zip(n.inputs, in_dt):
                if (id(a), j) not in dtype and a.op is None:
                    dtype[(id(a), j)] = d
            if (n.op in _ELEMWISE_BINARY and len({tuple(x) for x in in_shapes}) > 1
                    and not any(int(d) == 0 for x in in_shapes for d in x)):
                # nnvm ElemwiseShape: no broadcasting
                raise MXNetError('Error in operator %s (%s): incompatible input shapes %s'
                                 % (n.name, n.op, [tuple(x) for x in in_shapes]))
            pfn = _PARTIAL_OUT.get(n.op) if partial else None
            if partial and n.op in _PROBE_SKIP and any(_unknown_dims(s) for s in in_shapes):
                done.add(id(n))         # e.g. where: the output is unknown until the condition is known
                continue
            if pfn is not None and any(_unknown_dims(s) for s in in_shapes):
                outs = [(pfn(in_shapes[0], parsed), base_dt)]
            else:
                try:
                    outs = _run_meta(op, parsed, in_shapes, in_dt)
                except Exception as e:
                    if partial and any(_unknown_dims(s) for s in in_shapes):
                        done.add(id(n))     # output stays unknown
                        continue
                    raise MXNetError('Error in operator %s (%s): %s' % (n.name, n.op, e))
            for i, (s, d) in enumerate(outs):
                prev = shape.get((id(n), i))
                if prev is not None and tuple(prev) != tuple(s):
                    raise MXNetError('Error in operator %s (%s): inferred output shape %s conflicts with %s '
                                     'required by its consumers' % (n.name, n.op, tuple(s), tuple(prev)))
                shape[(id(n), i)] = s
                dtype[(id(n), i)] = d
            done.add(id(n))
            progress = True
    if what == 'type' and not partial:
        # variables only consumed through explicit casts (AMP graphs) default to fp32 storage
        consumers = {}
        for n in order:
            for a, _ in n.inputs:
                consumers.setdefault(id(a), []).append(n.op)
        for n in order:
            if n.op is None and (id(n), 0) not in dtype:
                ops = consumers.get(id(n), [])
                if ops and all(o in ('Cast', 'cast', 'amp_cast', 'amp_multicast') for o in ops):
                    dtype[(id(n), 0)] = torch.float32
    if what == 'shape' and partial:
        _partial_zero_dims(order, shape)
        if part is not None:
            from .. import util
            unk = -1 if util.is_np_shape() else 0
            for key, v in part.items():
                if shape.get(key) is None and v:
                    shape[key] = tuple(d if d > 0 else unk for d in v)
    aux = _aux_var_ids(order)
    table = shape if what == 'shape' else dtype
    args = [table.get((id(n), 0)) for n in order if n.op is None and id(n) not in aux]
    auxl = [table.get((id(n), 0)) for n in order if n.op is None and id(n) in aux]
    outs = [table.get((id(n), j)) for n, j in sym._outputs]
    return args, outs, auxl


# ---------------------------------------------------------------------------
# helper constructors (mirror python/mxnet/symbol/symbol.py module functions)
# ---------------------------------------------------------------------------

def zeros(shape, dtype=None, **kwargs):
    return _op_func('_zeros')(shape=shape, dtype=dtype_name(dtype or np.float32), **kwargs)


def ones(shape, dtype=None, **kwargs):
    return _op_func('_ones')(shape=shape, dtype=dtype_name(dtype or np.float32), **kwargs)


def full(shape, val, dtype=None, **kwargs):
    return _op_func('_full')(shape=shape, value=val, dtype=dtype_name(dtype or np.float32), **kwargs)


def arange(start, stop=None, step=1.0, repeat=1, infer_range=False, name=None, dtype=None):
    return _op_func('_arange')(start=start, stop=stop, step=step, repeat=repeat, name=name,
                               dtype=dtype_name(dtype or np.float32))


def linspace(start, stop, num, endpoint=True, name=None, dtype=None):
    return _op_func('_linspace')(start=start, stop=stop, num=num, endpoint=endpoint, name=name,
                                 dtype=dtype_name(dtype or np.float32))


def eye(N, M=0, k=0, dtype=None, **kwargs):
    return _op_func('_eye')(N=N, M=M, k=k, dtype=dtype_name(dtype or np.float32), **kwargs)


def _sym_or_scalar(bop, sop, rsop=None):
    def f(left, right):
        if isinstance(left, Symbol) and isinstance(right, Symbol):
            return _op_func(bop)(left, right)
        if isinstance(left, Symbol):
            return _op_func(sop)(left, scalar=float(right))
        if isinstance(right, Symbol):
            return _op_func(rsop or sop)(right, scalar=float(left))
        raise TypeError('at least one argument must be a Symbol')
    return f


pow = _sym_or_scalar('_power', '_power_scalar', '_rpower_scalar')  # pylint: disable=redefined-builtin
power = pow
maximum = _sym_or_scalar('_maximum', '_maximum_scalar')
minimum = _sym_or_scalar('_minimum', '_minimum_scalar')
hypot = _sym_or_scalar('_hypot', '_hypot_scalar')


def histogram(a, bins=10, range=None, **kwargs):  # pylint: disable=redefined-builtin
    if isinstance(bins, Symbol):
        return _op_func('_histogram')(a, bins, **kwargs)
    return _op_func('_histogram')(a, bin_cnt=bins, range=range, **kwargs)


def split_v2(ary, indices_or_sections, axis=0, squeeze_axis=False):
    if isinstance(indices_or_sections, int):
        return _op_func('_split_v2')(ary, axis=axis, squeeze_axis=squeeze_axis, sections=indices_or_sections)
    return _op_func('_split_v2')(ary, axis=axis, squeeze_axis=squeeze_axis,
                                 indices=(0,) + tuple(indices_or_sections))
