"""Graph passes, partitioners and subgraph operators of extension libraries (lib_api.h ABI v11).

Parity: the framework side of ``REGISTER_PASS`` / ``REGISTER_PARTITIONER`` / ``setIsSubgraphOp`` in
include/mxnet/lib_api.h (C entry points ``_passRegSize`` / ``_passRegGet`` / ``_passCallGraphPass``,
``_partRegSize`` / ``_partRegGetCount`` / ``_partRegGet`` / ``_partCallSupportedOps`` /
``_partCallCreateSelector`` / ``_partCallSelect*`` / ``_partCallFilter`` / ``_partCallReset`` /
``_partCallReviewSubgraph``) and of src/operator/subgraph/partitioner/custom_subgraph_property.h.

* ``Symbol.optimize_for(name, args, aux, **options)`` with a library pass name hands the graph
  JSON, the options and the bound arguments to the library and loads the graph it returns; arrays
  the pass allocates (``PassResource::alloc_arg/aux``) come back through ``nd_malloc`` and are
  added to ``args`` / ``aux``.
* with a library partitioner name, every strategy of the partitioner runs in turn: the library marks
  supported nodes (``supportedOps``, with subgraph ids: equal ids group, -1 joins any) or drives a
  selector (``createSelector`` + select / selectInput / selectOutput / filter / reset); convex groups
  are reviewed by ``reviewSubgraph`` (accept + extra attributes) and replaced by one node of the
  strategy's subgraph operator, carrying the subgraph JSON in ``subgraph_sym_json`` and the
  ``__ext_shape__`` / ``__ext_dtype__`` annotations the reference adds.
* a library subgraph operator runs through the library's stateful op (``createOpState`` receives the
  node attributes, subgraph JSON included) or its compute function; shapes and dtypes come from the
  subgraph itself.
"""
import ctypes
import json

import numpy as np
import torch

from .base import MXNetError

_PASSES = {}          # pass name -> _LibPass
_PARTITIONERS = {}    # partitioner name -> _LibPartitioner

_FLAG_OF = {torch.float32: 0, torch.float64: 1, torch.float16: 2, torch.uint8: 3, torch.int32: 4, torch.int8: 5,
            torch.int64: 6, torch.bfloat16: 12}
_TORCH_OF = {v: k for k, v in _FLAG_OF.items()}
_NP_FLAG = {'float32': 0, 'float64': 1, 'float16': 2, 'uint8': 3, 'int32': 4, 'int8': 5, 'int64': 6, 'bool': 7,
            'bfloat16': 12}

_ND_MALLOC = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64), ctypes.c_int, ctypes.c_char_p,
                              ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                              ctypes.POINTER(ctypes.c_void_p))


def _strs(values):
    arr = (ctypes.c_char_p * max(1, len(values)))()
    for i, v in enumerate(values):
        arr[i] = v.encode() if isinstance(v, str) else v
    return arr


def _options(opts):
    items = [(str(k), str(v)) for k, v in (opts or {}).items()]
    return _strs([k for k, _ in items]), _strs([v for _, v in items]), len(items)


def _as_tensor(a):
    from .ndarray.ndarray import NDArray
    return a._data if isinstance(a, NDArray) else a


class _ArrayTable:
    """The ``arg_*`` / ``aux_*`` parameter block of the pass / review calls for a {name: array} dict."""

    def __init__(self, arrays):
        arrays = {k: _as_tensor(v) for k, v in (arrays or {}).items() if v is not None}
        self.names = list(arrays)
        ts = [arrays[k].detach().contiguous() for k in self.names]
        self.keep = ts
        n = len(ts)
        self.shape_bufs = [(ctypes.c_int64 * max(1, t.dim()))(*t.shape) for t in ts]
        self.c_names = _strs(self.names)
        self.data = (ctypes.c_void_p * max(1, n))(*[t.data_ptr() for t in ts])
        self.shapes = (ctypes.POINTER(ctypes.c_int64) * max(1, n))(
            *[ctypes.cast(b, ctypes.POINTER(ctypes.c_int64)) for b in self.shape_bufs])
        self.dims = (ctypes.c_int * max(1, n))(*[t.dim() for t in ts])
        self.types = (ctypes.c_int * max(1, n))(*[_FLAG_OF.get(t.dtype, 0) for t in ts])
        self.ids = (ctypes.c_size_t * max(1, n))(*([0] * n))
        self.devt = _strs(['gpu' if t.is_cuda else 'cpu' for t in ts])
        self.devi = (ctypes.c_int * max(1, n))(*[t.device.index or 0 for t in ts])
        self.n = n

    def params(self):
        return [self.c_names, ctypes.c_int(self.n), self.data, self.shapes, self.dims, self.types, self.ids,
                self.devt, self.devi]


def graph_json(sym, args=None, aux=None):
    """(JSON string, nodes in JSON order) for ``sym``, with per-node ``__ext_shape__`` /
    ``__ext_dtype__`` annotations when the bound arrays determine them."""
    order = sym._topo()
    index = {id(n): i for i, n in enumerate(order)}
    shapes, dtypes = _entry_annotations(sym, args, aux)
    nodes = []
    for n in order:
        d = {'op': 'null' if n.op is None else n.op, 'name': n.name,
             'inputs': [[index[id(a)], j, 0] for a, j in n.inputs]}
        attrs = {k: str(v) for k, v in n.attrs.items()}
        k = n.num_outputs() if n.op is not None else 1
        sh = [shapes.get((id(n), i)) for i in range(k)]
        dt = [dtypes.get((id(n), i)) for i in range(k)]
        if any(s is not None for s in sh):
            attrs['__ext_shape__'] = '[' + ','.join('[None]' if s is None else '[' + ','.join(str(x) for x in s) + ']'
                                                    for s in sh) + ']'
        if any(t is not None for t in dt):
            attrs['__ext_dtype__'] = '[' + ','.join(str(-1 if t is None else t) for t in dt) + ']'
        d['attrs'] = attrs
        nodes.append(d)
    heads = [[index[id(n)], j, 0] for n, j in sym._outputs]
    g = {'nodes': nodes, 'arg_nodes': [i for i, n in enumerate(order) if n.op is None],
         'node_row_ptr': list(range(len(order) + 1)), 'heads': heads, 'attrs': {}}
    return json.dumps(g), order


def _entry_annotations(sym, args, aux):
    known = {}
    for src in (args or {}), (aux or {}):
        for k, v in src.items():
            if v is not None:
                known[k] = v
    if not known:
        return {}, {}
    internals = sym.get_internals()
    shapes, dtypes = {}, {}
    try:
        _, outs, _ = internals.infer_shape_partial(**{k: tuple(_as_tensor(v).shape) for k, v in known.items()})
        for (n, j), s in zip(internals._outputs, outs or []):
            if s is not None and all(int(x) > 0 for x in s):
                shapes[(id(n), j)] = tuple(int(x) for x in s)
    except Exception:   # noqa: BLE001 -- annotations are best effort, as in the reference
        pass
    try:
        _, touts, _ = internals.infer_type_partial(**{k: np.dtype(str(_as_tensor(v).dtype).replace('torch.', ''))
                                                       for k, v in known.items()
                                                       if str(_as_tensor(v).dtype) != 'torch.bfloat16'})
        for (n, j), t in zip(internals._outputs, touts or []):
            if t is not None:
                dtypes[(id(n), j)] = _NP_FLAG.get(np.dtype(t).name, -1)
    except Exception:   # noqa: BLE001
        pass
    return shapes, dtypes


# ------------------------------------------------------------------------------------- passes
class _LibPass:
    def __init__(self, lib, idx):
        fn, name = ctypes.c_void_p(), ctypes.c_char_p()
        lib.dll._passRegGet(ctypes.c_int(idx), ctypes.byref(fn), ctypes.byref(name))
        self.lib, self.fn, self.name = lib, fn, name.value.decode()

    def apply(self, sym, args=None, aux=None, **options):
        """Run the pass; returns (new Symbol, args, aux) -- arrays the pass allocated added."""
        from .symbol.symbol import load_json
        from . import ndarray as nd
        js, _ = graph_json(sym, args, aux)
        keys, vals, n = _options(options)
        at, xt = _ArrayTable(args), _ArrayTable(aux)
        new_args, new_aux = dict(args or {}), dict(aux or {})
        dev = next((t.device for t in at.keep + xt.keep), torch.device('cpu'))
        holder = []

        def nd_malloc(_alloc, shapes, num_shapes, dev_str, dev_id, dtype, name, is_arg, data):
            shp = tuple(shapes[i] for i in range(num_shapes))
            d = torch.device('cuda', dev_id) if dev_str and dev_str.decode() == 'gpu' else torch.device('cpu')
            t = torch.zeros(shp, dtype=_TORCH_OF.get(dtype, torch.float32), device=d)
            holder.append(t)
            (new_args if is_arg else new_aux)[name.decode()] = nd.NDArray(t)
            data[0] = t.data_ptr()
        cb = _ND_MALLOC(nd_malloc)
        out = ctypes.c_char_p()
        d = self.lib.dll
        d._passCallGraphPass.restype = ctypes.c_int
        rc = d._passCallGraphPass(self.fn, js.encode(), ctypes.byref(out), keys, vals, ctypes.c_int(n),
                                  self.name.encode(), *at.params(), *xt.params(), ctypes.cast(cb, ctypes.c_void_p),
                                  None)
        self.lib.check(rc, 'graph pass', self.name)
        text = ctypes.cast(out, ctypes.c_char_p).value.decode()
        d._opCallFree(ctypes.cast(out, ctypes.c_void_p))
        del dev
        return load_json(text), new_args, new_aux


# -------------------------------------------------------------------------------- partitioners
class _LibPartitioner:
    def __init__(self, lib, idx):
        d = lib.dll
        d._partRegGetCount.restype = ctypes.c_int
        name = ctypes.c_char_p()
        count = d._partRegGetCount(ctypes.c_int(idx), ctypes.byref(name))
        self.lib, self.name = lib, name.value.decode()
        self.strategies = []
        for s in range(count):
            strategy, op_name = ctypes.c_char_p(), ctypes.c_char_p()
            sup, csel, review = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
            d._partRegGet(ctypes.c_int(idx), ctypes.c_int(s), ctypes.byref(strategy), ctypes.byref(sup),
                          ctypes.byref(csel), ctypes.byref(review), ctypes.byref(op_name))
            self.strategies.append((strategy.value.decode(), sup, csel, review, op_name.value.decode()))

    def partition(self, sym, args=None, aux=None, **options):
        for strategy in self.strategies:
            sym = self._strategy(sym, strategy, args, aux, options)
        return sym

    def _strategy(self, sym, strategy, args, aux, options):
        from .symbol import subgraph
        from .symbol.symbol import _Node
        _name, sup, csel, review, op_name = strategy
        d = self.lib.dll
        js, order = graph_json(sym, args, aux)
        index = {id(n): i for i, n in enumerate(order)}
        keys, vals, n = _options(options)
        sel = None
        if sup.value:
            ids = (ctypes.c_int * max(1, len(order)))(*([-2] * len(order)))
            d._partCallSupportedOps.restype = ctypes.c_int
            rc = d._partCallSupportedOps(sup, js.encode(), ctypes.c_int(len(order)), ids, keys, vals, ctypes.c_int(n))
            self.lib.check(rc, 'supportedOps', self.name)
            supported = {i: ids[i] for i in range(len(order)) if ids[i] != -2}

            def selectable(node):
                return index[id(node)] in supported

            def joinable(a, node, _members):
                ia, inode = supported.get(index[id(a)], -2), supported.get(index[id(node)], -2)
                return inode != -2 and (ia == inode or inode == -1 or ia == -1)
        elif csel.value:
            handle = ctypes.c_void_p()
            d._partCallCreateSelector.restype = ctypes.c_int
            rc = d._partCallCreateSelector(csel, js.encode(), ctypes.byref(handle), keys, vals, ctypes.c_int(n))
            self.lib.check(rc, 'createSelector', self.name)
            sel = handle

            def ask(fn, *ids_):
                out = ctypes.c_int(0)
                fn(sel, *[ctypes.c_int(i) for i in ids_], ctypes.byref(out))
                return bool(out.value)

            def selectable(node):
                return ask(d._partCallSelect, index[id(node)])

            def joinable(a, node, _members):
                # growing a's group to its consumer: the selector must accept the edge both ways
                return ask(d._partCallSelectOutput, index[id(a)], index[id(node)]) or \
                    ask(d._partCallSelectInput, index[id(node)], index[id(a)])
        else:
            raise MXNetError('partitioner %s strategy %s registers neither supportedOps nor createSelector'
                             % (self.name, _name))
        groups = subgraph._group_convex(order, selectable, joinable)
        if sel is not None and groups:
            groups = self._filter(groups, index, order, sel)
            d._partCallReset(sel)
        if not groups:
            return sym
        descs = subgraph.describe_groups(sym, order, groups)
        accepted, extra = [], []
        for gi, (g, desc) in enumerate(zip(groups, descs)):
            ok, attrs = self._review(review, desc, gi, options, args, aux, order, index)
            if ok:
                accepted.append(g)
                extra.append((desc, attrs))
        if not accepted:
            return sym
        descs = [e[0] for e in extra]
        shapes, dtypes = _entry_annotations(sym, args, aux)

        def make(gi, desc, inputs):
            graph = dict(desc['graph'])
            nodes = [dict(x) for x in graph['nodes']]
            for k, (a, j) in enumerate(desc['ext']):
                at = dict(nodes[k].get('attrs', {}))
                at['isArg'] = 'True' if a.op is None else 'False'
                if a.op is None:
                    at['argName'] = a.name
                    nodes[k]['name'] = a.name
                nodes[k]['attrs'] = at
            graph['nodes'] = nodes
            attrs = {'subgraph_sym_json': json.dumps(graph)}
            sh = [shapes.get((id(m), j)) for m, j in desc['outs']]
            dt = [dtypes.get((id(m), j)) for m, j in desc['outs']]
            if all(s is not None for s in sh):
                attrs['__ext_shape__'] = '[' + ','.join('[' + ','.join(str(x) for x in s) + ']' for s in sh) + ']'
            if all(t is not None for t in dt):
                attrs['__ext_dtype__'] = '[' + ','.join(str(t) for t in dt) + ']'
            attrs.update(extra[gi][1])
            return _Node(op_name, '_op%d' % gi, attrs, inputs)
        return subgraph.rebuild(sym, order, accepted, descs, make)

    def _filter(self, groups, index, order, sel):
        d = self.lib.dll
        kept = []
        for g in groups:
            cand = (ctypes.c_int * len(g))(*[index[id(m)] for m in g])
            keep, nkeep = ctypes.POINTER(ctypes.c_int)(), ctypes.c_int()
            d._partCallFilter(sel, cand, ctypes.c_int(len(g)), ctypes.byref(keep), ctypes.byref(nkeep))
            ids = {keep[i] for i in range(nkeep.value)}
            if nkeep.value:
                d._opCallFree(ctypes.cast(keep, ctypes.c_void_p))
            g2 = [m for m in g if index[id(m)] in ids]
            if g2:
                kept.append(g2)
        return kept

    def _review(self, review, desc, gi, options, args, aux, order, index):
        if not review.value:
            return True, {}
        d = self.lib.dll
        graph = dict(desc['graph'])
        nodes = [dict(x) for x in graph['nodes']]
        aux_set = set(desc['aux'])
        for k in range(len(desc['ext'])):
            at = dict(nodes[k].get('attrs', {}))
            at['isAux'] = 'True' if k in aux_set else 'False'
            nodes[k]['attrs'] = at
        graph['nodes'] = nodes
        keys, vals, n = _options(options)
        accept = ctypes.c_int(1)
        akeys, avals, nattr = ctypes.POINTER(ctypes.c_void_p)(), ctypes.POINTER(ctypes.c_void_p)(), ctypes.c_int(0)
        at, xt = _ArrayTable(args), _ArrayTable(aux)
        d._partCallReviewSubgraph.restype = ctypes.c_int
        rc = d._partCallReviewSubgraph(review, json.dumps(graph).encode(), ctypes.c_int(gi), ctypes.byref(accept),
                                       keys, vals, ctypes.c_int(n), ctypes.byref(akeys), ctypes.byref(avals),
                                       ctypes.byref(nattr), *at.params(), *xt.params())
        self.lib.check(rc, 'reviewSubgraph', self.name)
        attrs = {}
        for i in range(nattr.value):
            attrs[ctypes.string_at(akeys[i]).decode()] = ctypes.string_at(avals[i]).decode()
        if nattr.value:
            for i in range(nattr.value):
                d._opCallFree(ctypes.c_void_p(akeys[i]))
                d._opCallFree(ctypes.c_void_p(avals[i]))
            d._opCallFree(ctypes.cast(akeys, ctypes.c_void_p))
            d._opCallFree(ctypes.cast(avals, ctypes.c_void_p))
        return bool(accept.value), attrs


# ------------------------------------------------------------------------- subgraph operators
_SUBGRAPH_SYMS = {}


def _subgraph_sym(text):
    s = _SUBGRAPH_SYMS.get(text)
    if s is None:
        from .symbol.symbol import load_json
        s = _SUBGRAPH_SYMS[text] = load_json(text)
    return s


def _sg_json(a, default):
    v = a.get('subgraph_sym_json', default)
    return json.loads(v) if isinstance(v, str) else v


def _sg_inputs(a):
    """The subgraph's inputs, then the extra inputs a graph pass attached (``__ext_extra_inputs__``)."""
    g = _sg_json(a, '{"nodes": []}')
    n = sum(1 for x in g['nodes'] if x['op'] == 'null') + int(a.get('__ext_extra_inputs__', 0) or 0)
    return ['data%d' % i for i in range(n)]


def _sg_num_outputs(a):
    g = _sg_json(a, '{"heads": [[0, 0, 0]]}')
    return len(g['heads'])


def _sg_out_meta(attrs, inputs):
    """Output shapes/dtypes of a subgraph node from its subgraph (inputs in data<i> order)."""
    text = attrs['subgraph_sym_json']
    text = text if isinstance(text, str) else json.dumps(text)
    sym = _subgraph_sym(text)
    names = sym.list_arguments() + sym.list_auxiliary_states()
    g = json.loads(text)
    in_names = [n['name'] for n in g['nodes'] if n['op'] == 'null']
    by_name = dict(zip(in_names, inputs))
    shapes = {k: tuple(by_name[k].shape) for k in names if k in by_name}
    _, outs, _ = sym.infer_shape(**shapes)
    dt = inputs[0].dtype if inputs else torch.float32
    return [tuple(s) for s in outs], dt


def register_subgraph_op(lib_op):
    """Register a library subgraph operator (``setIsSubgraphOp``) with this framework."""
    from .ops import registry
    from .library import _State

    class _SgFunction(torch.autograd.Function):
        @staticmethod
        def forward(ctx, attrs, *inputs):
            inputs = [t.contiguous() for t in inputs]
            shapes, dt = _sg_out_meta(attrs, inputs)
            outs = [torch.empty(s, dtype=dt, device=inputs[0].device) for s in shapes]
            if lib_op.create_state:
                state = lib_op.make_state(attrs, inputs)
                lib_op.stateful(True, state, inputs, outs)
                ctx.state = state
            else:
                lib_op.fcompute(lib_op.forward, attrs, inputs, outs)
                ctx.state = None
            ctx.attrs = attrs
            ctx.save_for_backward(*inputs, *outs)
            ctx.nin = len(inputs)
            return tuple(outs)

        @staticmethod
        def backward(ctx, *grads):
            saved = ctx.saved_tensors
            inputs, outs = list(saved[:ctx.nin]), list(saved[ctx.nin:])
            og = [(g if g is not None else torch.zeros_like(o)).contiguous() for g, o in zip(grads, outs)]
            ig = [torch.zeros_like(t) for t in inputs]
            if ctx.state is not None:
                lib_op.stateful(False, ctx.state, og + inputs + outs, ig)
            elif lib_op.backward:
                lib_op.fcompute(lib_op.backward, ctx.attrs, og + inputs + outs, ig)
            else:
                raise MXNetError('extension subgraph op %s has no backward' % lib_op.name)
            return (None,) + tuple(ig)

    def fn(*inputs, **attrs):
        attrs = {k: v for k, v in attrs.items()}
        if inputs and inputs[0].device.type == 'meta':
            shapes, dt = _sg_out_meta(attrs, list(inputs))
            outs = [torch.empty(s, dtype=dt, device='meta') for s in shapes]
            return outs[0] if len(outs) == 1 else tuple(outs)
        outs = _SgFunction.apply(attrs, *inputs)
        return outs[0] if len(outs) == 1 else tuple(outs)
    fn.__name__ = lib_op.name
    _ = _State
    registry.register(lib_op.name, fn, arg_names=_sg_inputs, num_outputs=_sg_num_outputs, extra_params=True,
                      params={'subgraph_sym_json': ('str', ''), '__ext_extra_inputs__': ('int', 0)})


def register_library(lib):
    """Passes and partitioners of a loaded lib_api library; returns (pass names, partitioner names)."""
    d = lib.dll
    passes, parts = [], []
    if hasattr(d, '_passRegSize'):
        d._passRegSize.restype = ctypes.c_int
        for i in range(d._passRegSize()):
            p = _LibPass(lib, i)
            _PASSES[p.name] = p
            passes.append(p.name)
    if hasattr(d, '_partRegSize'):
        d._partRegSize.restype = ctypes.c_int
        for i in range(d._partRegSize()):
            p = _LibPartitioner(lib, i)
            _PARTITIONERS[p.name] = p
            parts.append(p.name)
    return passes, parts


def optimize_for(sym, backend, args=None, aux=None, **options):
    """Apply a library pass or partitioner named ``backend``; None when no library registered it.
    Returns (Symbol, args, aux)."""
    if backend in _PASSES:
        return _PASSES[backend].apply(sym, args, aux, **options)
    if backend in _PARTITIONERS:
        return _PARTITIONERS[backend].partition(sym, args, aux, **options), args, aux
    return None
