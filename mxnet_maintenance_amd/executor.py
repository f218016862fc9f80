"""Graph executor for bound Symbols.

Parity: python/mxnet/executor.py (Executor.forward/backward/outputs/arg_dict/
grad_dict/aux_dict/output_dict/reshape/copy_params_from) and
src/executor/graph_executor.cc.

A Symbol is lowered once into a ``GraphProgram``: a flat list of steps
``(op fn, input slots, parsed attrs, output slots)`` in topological order.  The
same program drives ``Executor`` and Gluon's hybridized ``CachedOp``; with
static shapes the program can be captured into a HIP graph (see
gluon/block.py).  Gradients come from the autograd tape of the forward run.
"""
import os

import numpy as np
import torch

from . import _state
from . import profiler as _profiler
from .ops import amp_dispatch as _amp
from .base import MXNetError, AsyncOpError
from .ops import registry


def _call_monitor(cb, name, arr):
    """Executor monitor callbacks receive (name, NDArrayHandle) as from the reference's C API:
    ``NDArray(ctypes.cast(handle, NDArrayHandle))`` recovers the array.  The handle is live for the
    duration of the call."""
    from .base import _HANDLES, NDArrayHandle
    key = id(arr)
    _HANDLES[key] = arr
    try:
        cb(name, NDArrayHandle(key))
    finally:
        _HANDLES.pop(key, None)


class GraphProgram:
    """Topologically ordered, slot-addressed form of a Symbol."""

    def __init__(self, sym):
        from .symbol.symbol import _aux_var_ids
        order = sym._topo()
        self.symbol = sym
        slot = {}
        nslots = 0
        self.var_names = []
        self.var_slots = []
        aux = _aux_var_ids(order)
        self.arg_names = []
        self.aux_names = []
        for n in order:
            if n.op is None:
                slot[(id(n), 0)] = nslots
                self.var_names.append(n.name)
                self.var_slots.append(nslots)
                (self.aux_names if id(n) in aux else self.arg_names).append(n.name)
                nslots += 1
        self.steps = []
        for n in order:
            if n.op is None:
                continue
            op = n.opdef()
            parsed = dict(n.parsed())
            k = op.get_num_outputs(parsed)
            outs = []
            for i in range(k):
                slot[(id(n), i)] = nslots
                outs.append(nslots)
                nslots += 1
            ins = [slot[(id(a), j)] for a, j in n.inputs]
            self.steps.append((op.fn, ins, parsed, outs, n.name, op.name))
        self.out_slots = [slot[(id(n), j)] for n, j in sym._outputs]
        self.nslots = nslots
        self._var_of_slot = {s: n for n, s in zip(self.var_names, self.var_slots)}
        self.name_to_slot = dict(zip(self.var_names, self.var_slots))

    # operators whose monitor input names are positional in the reference (no FListInputNames)
    _POSITIONAL_INPUTS = ('SoftmaxActivation', 'Activation')

    @staticmethod
    def _input_names(opname, attrs, n):
        op = registry.get(opname)
        if op.name in GraphProgram._POSITIONAL_INPUTS:
            return ['input%d' % j for j in range(n)]
        names = op.get_arg_names(attrs) + op.get_aux_names(attrs)
        return [names[j] if j < len(names) else 'input%d' % j for j in range(n)]

    def run(self, feed, monitor=None, monitor_all=False, record=None, int_dtypes=None):
        """``feed``: dict var name -> torch tensor.  Returns output tensors.

        ``int_dtypes`` (var name -> integer torch dtype) marks inputs that are integer variables
        carried in float64 for autograd (NDArray.attach_grad); operators on them, and operators
        casting a differentiable input to an integer dtype, run the shadow path of the imperative
        invoke, and ``self.out_idts`` reports the outputs' integer dtypes.

        ``monitor(name, tensor)`` is called for every operator output (and,
        with ``monitor_all``, every operator input) — the engine-level monitor
        callback of src/executor/graph_executor.cc (ExecuteMonCallback).
        """
        vals = [None] * self.nslots
        for name, s in self.name_to_slot.items():
            vals[s] = feed.get(name)
        islot = {}
        if int_dtypes:
            islot = {self.name_to_slot[n]: d for n, d in int_dtypes.items() if n in self.name_to_slot}
        self.failure = None       # first operator execution failure of this run (deferred to sync)
        sched = self._stream_sched(vals) if _GRAPH_STREAMS > 1 else None
        try:
            for si, (fn, ins, attrs, outs, name, opname) in enumerate(self.steps):
                args = [vals[i] for i in ins]
                if sched is not None:
                    sched.before(si, args)
                if _amp.active:
                    args = _amp.cast_inputs(opname, args, attrs)
                if record is not None:
                    record.append((name, args))
                if monitor is not None and monitor_all:
                    # reference order: a variable input under its own name, then every input as
                    # <node>_<argument name>
                    argn = self._input_names(opname, attrs, len(args))
                    for j, a in enumerate(args):
                        if a is None:
                            continue
                        var = self._var_of_slot.get(ins[j])
                        if var is not None:
                            monitor(var, a)
                        monitor('%s_%s' % (name, argn[j]), a)
                try:
                    if (islot and any(i in islot for i in ins)) or (attrs.get('dtype') is not None and
                                                                     _int_dtype_attr(attrs) and torch.is_grad_enabled()):
                        r = self._run_shadow(fn, args, attrs, ins, outs, islot, opname)
                    elif _profiler.active_symbolic:
                        with _profiler.op_span(_profiler.current_scope() + opname, symbolic=True):
                            r = fn(*args, **attrs)
                    else:
                        r = fn(*args, **attrs)
                except AsyncOpError as e:
                    # the graph keeps running on a zero stand-in; the outputs carry the failure
                    from .ndarray.register import _placeholder
                    if self.failure is None:
                        self.failure = AsyncOpError('Error in operator %s (%s): %s' % (name, opname, e))
                    r = _placeholder(attrs, [])
                except MXNetError:
                    if self.failure is None:
                        raise
                    from .ndarray.register import _placeholder
                    r = _placeholder(attrs, [])
                except (RuntimeError, IndexError) as e:
                    if self.failure is not None:
                        from .ndarray.register import _placeholder
                        r = _placeholder(attrs, [])
                    else:
                        raise MXNetError('Error in operator %s (%s): %s' % (name, opname, e)) from e
                if sched is not None:
                    sched.after(si)
                if len(outs) == 1:
                    vals[outs[0]] = r[0] if isinstance(r, (tuple, list)) else r
                else:
                    for o, t in zip(outs, r):
                        vals[o] = t
                if monitor is not None:
                    op = registry.get(opname)
                    onames = op.output_names or (['output'] if len(outs) == 1 else
                                                 ['output%d' % k for k in range(len(outs))])
                    for o, on in zip(outs, onames):
                        if vals[o] is not None:
                            monitor('%s_%s' % (name, on), vals[o])
        finally:
            if sched is not None:
                torch.cuda.set_stream(sched.main)
        self.out_idts = [islot.get(s) for s in self.out_slots] if islot else None
        if sched is not None:
            sched.finish([vals[s] for s in self.out_slots])
        return [vals[s] for s in self.out_slots]

    # ------------------------------------------------------------------ multi-stream schedule
    def _stream_plan(self, nstreams):
        """Static assignment of the graph's operators to ``nstreams`` HIP streams (the dependency
        engine's job for a bound graph, src/executor/graph_executor.cc + threaded_engine): an operator
        continues the stream of its latest producer while that stream's last operator is that
        producer; a heavy operator (conv, FC, ...) whose producers' streams have moved on starts a
        branch on a side stream.  Cross-stream edges become event waits.  Returns (stream index per
        step, producer steps to wait for per step, steps whose completion is recorded)."""
        producer = {}
        for i, st in enumerate(self.steps):
            for o in st[3]:
                producer[o] = i
        n = len(self.steps)
        stream_of = [0] * n
        tail = [-1] * nstreams
        waits = [()] * n
        need_ev = set()
        rr = 1
        for i, (_fn, ins, _attrs, _outs, _name, opname) in enumerate(self.steps):
            prods = sorted({producer[x] for x in ins if x in producer})
            # an operator fed only by graph inputs hangs off a virtual producer (-1) on the caller's
            # stream: the first such operator continues it, later ones can branch
            cands = prods or [-1]
            # streams on which a producer is still the last operator; joins prefer the lowest
            # (the caller's stream keeps the trunk)
            live = [stream_of[p] if p >= 0 else 0 for p in cands if tail[stream_of[p] if p >= 0 else 0] == p]
            choice = min(live) if live else None
            if choice is None:
                if opname in _BRANCH_OPS and nstreams > 1:
                    choice = rr
                    rr = 1 + rr % (nstreams - 1)
                else:
                    choice = stream_of[prods[-1]] if prods else 0
            stream_of[i] = choice
            tail[choice] = i
            w = tuple(p for p in prods if stream_of[p] != choice)
            waits[i] = w
            need_ev.update(w)
        return stream_of, waits, need_ev

    def _stream_sched(self, vals):
        dev = next((v.device for v in vals if isinstance(v, torch.Tensor) and v.is_cuda), None)
        if dev is None or torch.cuda.is_current_stream_capturing() and not _GRAPH_STREAMS_CAPTURE:
            return None
        plan = getattr(self, '_splan', None)
        if plan is None:
            plan = self._splan = self._stream_plan(_GRAPH_STREAMS)
        if max(plan[0], default=0) == 0:
            return None
        return _StreamSched(plan, dev)
    @staticmethod
    def _run_shadow(fn, args, attrs, ins, outs, islot, opname=None):
        """One operator over integer values carried in float64 (see ``run``): the integer result's
        values and dtype, the float copy's gradient path."""
        from .ndarray.register import _merge_shadow, INT_ZERO_GRAD
        true_args = [a.detach().to(islot[i]) if (i in islot and a is not None) else a for a, i in zip(args, ins)]
        with torch.no_grad():
            res_t = fn(*true_args, **attrs)
        multi = isinstance(res_t, (tuple, list))
        if not torch.is_grad_enabled() or not any(a is not None and a.requires_grad for a in args) or \
                opname in INT_ZERO_GRAD:
            for o in outs:
                islot.pop(o, None)
            return res_t
        kw_f = dict(attrs, dtype='float64') if _int_dtype_attr(attrs) else attrs
        res_f = fn(*args, **kw_f)
        pairs = [_merge_shadow(f, t) for f, t in zip(res_f, res_t)] if multi else [_merge_shadow(res_f, res_t)]
        for o, (_, d) in zip(outs, pairs):
            if d is not None:
                islot[o] = d
            else:
                islot.pop(o, None)
        return [p[0] for p in pairs] if multi else pairs[0][0]


_GRAPH_STREAMS = int(os.environ.get('MXNET_GRAPH_STREAMS', '1') or 1)
_GRAPH_STREAMS_CAPTURE = os.environ.get('MXNET_GRAPH_STREAMS_CAPTURE', '0') == '1'
# operators worth a branch of their own on a side stream
_BRANCH_OPS = frozenset(('Convolution', 'Deconvolution', 'FullyConnected', '_contrib_DeformableConvolution',
                         '_contrib_ModulatedDeformableConvolution', 'Pooling', 'dot', 'batch_dot', '_npi_matmul',
                         'RNN', '_FusedOp'))
_SIDE_STREAMS = {}


def _side_streams(dev, n):
    lst = _SIDE_STREAMS.get(dev)
    if lst is None or len(lst) < n:
        lst = _SIDE_STREAMS[dev] = [torch.cuda.Stream(device=dev) for _ in range(n)]
    return lst


class _StreamSched:
    """Runs one GraphProgram pass on the streams of a static plan (see GraphProgram._stream_plan):
    side streams fork from the caller's stream at their first operator and join it at the end, so
    the pass is also capturable into one HIP graph with parallel branches.  Tensors that cross
    streams are recorded on the consuming stream for the caching allocator."""

    def __init__(self, plan, dev):
        self.stream_of, self.waits, self.need_ev = plan
        self.main = torch.cuda.current_stream(dev)
        self.streams = [self.main] + _side_streams(dev, _GRAPH_STREAMS - 1)
        self.events = {}
        self.started = set()
        self.start_ev = None
        self.side_steps = set()

    def before(self, i, args):
        k = self.stream_of[i]
        s = self.streams[k]
        if k and k not in self.started:
            if self.start_ev is None:
                self.start_ev = torch.cuda.Event()
                self.start_ev.record(self.main)
            s.wait_event(self.start_ev)
            self.started.add(k)
        for p in self.waits[i]:
            s.wait_event(self.events[p])
        if k or self.waits[i]:
            for a in args:
                if isinstance(a, torch.Tensor) and a.is_cuda:
                    a.record_stream(s)
        if k:
            self.side_steps.add(i)
            torch.cuda.set_stream(s)

    def after(self, i):
        k = self.stream_of[i]
        if k:
            torch.cuda.set_stream(self.main)
        if i in self.need_ev:
            ev = torch.cuda.Event()
            ev.record(self.streams[k])
            self.events[i] = ev

    def finish(self, outs):
        for k in sorted(self.started):
            ev = torch.cuda.Event()
            ev.record(self.streams[k])
            self.main.wait_event(ev)
        if self.side_steps:
            for o in outs:
                if isinstance(o, torch.Tensor) and o.is_cuda:
                    o.record_stream(self.main)


def _int_dtype_attr(attrs):
    dt = attrs.get('dtype')
    return dt is not None and str(dt).replace('torch.', '').startswith(('int', 'uint', 'bool'))


# binary / scatter operators whose row_sparse lhs keeps its storage (reference scatter_* and
# elemwise FInferStorageType: rows come from the lhs, or the union of both row_sparse operands)
_SPARSE_LHS = frozenset(('_scatter_elemwise_div', '_scatter_plus_scalar', '_scatter_minus_scalar',
                         '_mul_scalar', '_div_scalar'))
_SPARSE_ADD = frozenset(('elemwise_add', 'elemwise_sub', '_grad_add', '_plus', '_minus', '_add', '_sub'))
_SPARSE_MUL = frozenset(('elemwise_mul', '_mul'))
_SPARSE_SAME = frozenset(('_maximum', '_minimum', '_hypot', 'maximum', 'minimum', 'hypot'))


def _binary_stype(op, ins):
    """Output storage of the sparse-aware binary operators (FInferStorageType of
    src/operator/tensor/elemwise_binary_op_basic.cc and elemwise_scatter_op.cc); None when the
    operator has no rule here."""
    if not ins or all(t == 'default' for t in ins):
        return None
    if op in _SPARSE_LHS:
        return ins[0] if ins[0] != 'default' else None
    if len(ins) != 2:
        return None
    lt, rt = ins
    if op in _SPARSE_ADD or op in _SPARSE_SAME:
        return lt if lt == rt else 'default'
    if op in _SPARSE_MUL:
        if lt == rt:
            return lt
        if 'default' in (lt, rt):
            return rt if lt == 'default' else lt          # dense * sparse keeps the sparse pattern
        return 'default'
    if op in ('elemwise_div', '_div'):
        return 'default'
    return None


def registry_parse(node):
    from .ops import registry
    try:
        return registry.get(node.op).parse_attrs(node.attrs)
    except Exception:  # pragma: no cover - unknown attribute formats: infer as dense
        return {}


class Executor:
    """Executor bound to arrays for arguments, gradients and auxiliary states."""

    def __init__(self, sym, ctx, args, args_grad=None, grad_req='write', aux_states=None):
        from .ndarray.ndarray import NDArray
        from .symbol import passes as _passes
        self._symbol = sym
        self._ctx = ctx
        # bind-time graph passes (common-subexpression elimination, pointwise fusion); argument /
        # output names and order are those of ``sym``
        from .symbol.symbol import _unify_init_shapes
        _unify_init_shapes(sym._topo())      # init ops with unknown dims sized from their consumers
        self._opt_symbol = _passes.optimize(sym, ctx)
        self._prog = GraphProgram(self._opt_symbol)
        arg_names = sym.list_arguments()
        aux_names = sym.list_auxiliary_states()
        if isinstance(args, dict):
            missing = [n for n in arg_names if n not in args]
            if missing:
                raise MXNetError('bind: missing arguments %s' % missing)
            self.arg_arrays = [args[n] for n in arg_names]
        else:
            if len(args) != len(arg_names):
                raise MXNetError('bind: expected %d arguments, got %d' % (len(arg_names), len(args)))
            self.arg_arrays = list(args)
        if isinstance(grad_req, str):
            self._grad_req = {n: grad_req for n in arg_names}
        elif isinstance(grad_req, (list, tuple)):
            self._grad_req = dict(zip(arg_names, grad_req))
        else:
            self._grad_req = {n: grad_req.get(n, 'null') for n in arg_names}
        if args_grad is None:
            self.grad_arrays = [None] * len(arg_names)
            self._grad_req = {n: 'null' for n in arg_names}
        elif isinstance(args_grad, dict):
            self.grad_arrays = [args_grad.get(n) for n in arg_names]
        else:
            self.grad_arrays = list(args_grad) + [None] * (len(arg_names) - len(args_grad))
        for n, g in zip(arg_names, self.grad_arrays):
            if g is None:
                self._grad_req[n] = 'null'
        if aux_states is None:
            aux_states = []
        if isinstance(aux_states, dict):
            self.aux_arrays = [aux_states[n] for n in aux_names]
        else:
            self.aux_arrays = list(aux_states)
        if len(self.aux_arrays) != len(aux_names):
            raise MXNetError('bind: expected %d aux states, got %d' % (len(aux_names), len(self.aux_arrays)))
        self._check_differentiable()
        self.outputs = self._preallocate_outputs()
        self._leaves = None
        self._out_tensors = None
        self._monitor_cb = None
        self._monitor_all = False

    # operators the reference registers without FGradient: binding for a gradient through them fails
    _NO_GRADIENT = ('batch_take',)

    def _check_differentiable(self):
        from .symbol import passes as _passes
        wanting = {n for n, r in self._grad_req.items() if r != 'null'}
        if not wanting:
            return
        order = self._symbol._topo()
        live = {id(n) for n, _ in self._symbol._outputs}
        for n in reversed(order):
            if id(n) not in live or n.op is None:
                continue
            name = n.opdef().name
            if name == 'BlockGrad':
                continue
            if name in self._NO_GRADIENT:
                from .symbol.symbol import Symbol
                if _passes.grad_reachable(Symbol([(n, 0)]), wanting):
                    raise MXNetError('Operator %s is non-differentiable because it didn\'t register '
                                     'FGradient attribute.' % name)
            for a, _ in n.inputs:
                live.add(id(a))

    def _preallocate_outputs(self):
        """Output arrays allocated at bind time (as the reference's graph executor does), so
        ``outputs`` exist before the first forward and a reshaped executor can alias them."""
        from . import ndarray as nd
        try:
            shapes = {n: a.shape for n, a in zip(self._symbol.list_arguments(), self.arg_arrays)}
            _, out_shapes, _ = self._symbol.infer_shape(**shapes)
            _, out_types, _ = self._symbol.infer_type(**{n: a.dtype for n, a in
                                                          zip(self._symbol.list_arguments(), self.arg_arrays)})
        except Exception:   # pylint: disable=broad-except
            return []
        if not out_shapes or any(s is None for s in out_shapes):
            return []
        return [nd.zeros(tuple(s), ctx=self._ctx, dtype=t if t is not None else 'float32')
                for s, t in zip(out_shapes, out_types or [None] * len(out_shapes))]

    @property
    def arg_dict(self):
        return dict(zip(self._symbol.list_arguments(), self.arg_arrays))

    @property
    def grad_dict(self):
        return dict(zip(self._symbol.list_arguments(), self.grad_arrays))

    @property
    def aux_dict(self):
        return dict(zip(self._symbol.list_auxiliary_states(), self.aux_arrays))

    @property
    def output_dict(self):
        return dict(zip(self._symbol.list_outputs(), self.outputs))

    def forward(self, is_train=False, **kwargs):
        from .ndarray.ndarray import NDArray
        for k, v in kwargs.items():
            ad = self.arg_dict
            if k not in ad:
                raise MXNetError('forward: unknown argument %s' % k)
            src = v._data if isinstance(v, NDArray) else torch.as_tensor(np.asarray(v))
            with torch.no_grad():
                ad[k]._data.copy_(src.reshape(ad[k].shape))
        need_grad = is_train and any(r != 'null' for r in self._grad_req.values())
        self._last_is_train = bool(is_train)
        return self._run(is_train, need_grad)

    def _run(self, is_train, need_grad):
        from . import engine as _eng
        _eng.join_workers()   # graph programs run on the caller's stream
        from .ndarray.ndarray import NDArray
        arg_names = self._symbol.list_arguments()
        feed = {}
        leaves = []
        int_dtypes = None
        for n, a in zip(arg_names, self.arg_arrays):
            t = a._data.detach()
            if need_grad and self._grad_req[n] != 'null':
                if not (t.is_floating_point() or t.is_complex()):
                    # an integer argument with a gradient: carried in float64 through the graph's
                    # integer shadow path (GraphProgram.run), so casts out of it back-propagate
                    int_dtypes = int_dtypes or {}
                    int_dtypes[n] = t.dtype
                    t = t.to(torch.float64)
                t = t.requires_grad_(True)
                leaves.append((n, t))
            feed[n] = t
        for n, a in zip(self._symbol.list_auxiliary_states(), self.aux_arrays):
            feed[n] = a._data
        prev_train = _state.STATE.training
        _state.STATE.training = bool(is_train)
        try:
            mon = None
            if self._monitor_cb is not None:
                cb = self._monitor_cb

                def mon(name, t):
                    _call_monitor(cb, name, NDArray(t.detach()))
            record = [] if (mon is not None and need_grad) else None
            with torch.set_grad_enabled(need_grad):
                outs = self._prog.run(feed, mon, self._monitor_all, record, int_dtypes=int_dtypes)
            self._mon_record = record
            self._mon_grads = {}
            if record:
                # gradients flowing into every operator input, reported by backward() like the
                # reference's monitor over the backward graph's nodes
                for _name, args in record:
                    for t in args:
                        if isinstance(t, torch.Tensor) and t.requires_grad and id(t) not in self._mon_grads:
                            self._mon_grads[id(t)] = None

                            def hook(g, key=id(t)):
                                self._mon_grads[key] = g.detach()
                            t.register_hook(hook)
        finally:
            _state.STATE.training = prev_train
        self._leaves = leaves
        self._out_tensors = outs
        idts = getattr(self._prog, 'out_idts', None) or [None] * len(outs)
        vals = [o.detach().to(d) if d is not None else o.detach() for o, d in zip(outs, idts)]
        if len(self.outputs) == len(vals) and all(
                b.shape == tuple(o.shape) and b._data.dtype == o.dtype for b, o in zip(self.outputs, vals)):
            # write into the bind-time output arrays (they may be views shared with a reshaped executor)
            with torch.no_grad():
                for b, o in zip(self.outputs, vals):
                    b._data.copy_(o)
        else:
            self.outputs = [NDArray(o) for o in vals]
        st = self._output_stypes()
        if st is not None:
            from .ndarray import sparse
            self.outputs = [sparse.cast_storage(o, t) if t != 'default' else o for o, t in zip(self.outputs, st)]
        self._failure = getattr(self._prog, 'failure', None)
        self._failure_box = None
        if self._failure is not None:
            from . import engine
            box = self._failure_box = engine.record_failure(self._failure)
            for o in self.outputs:
                o._exc = box
        return self.outputs

    def _output_stypes(self):
        """Storage types of the outputs when sparse arguments are bound (reference: FInferStorageType
        over the graph); None when every argument is dense.  Operators keep a sparse first input's
        storage where register._kept_stype says so; everything else falls back to dense."""
        cached = getattr(self, '_stype_cache', False)
        if cached is not False:
            return cached
        from .ndarray.register import _kept_stype, _check_storage
        args = dict(zip(self._symbol.list_arguments(), self.arg_arrays))
        if all(getattr(a, 'stype', 'default') == 'default' for a in args.values()):
            self._stype_cache = None
            return None

        class _S:
            __slots__ = ('stype',)

            def __init__(self, st):
                self.stype = st
        memo = {}
        for n in self._symbol._topo():
            if n.op is None:
                memo[(id(n), 0)] = getattr(args.get(n.name), 'stype', 'default')
                continue
            ins = [memo.get((id(i), j), 'default') for i, j in n.inputs]
            attrs = registry_parse(n)
            _check_storage(n.op, ins, attrs)
            st = _binary_stype(n.op, ins)
            if st is None:
                st = _kept_stype(n.op, [_S(t) for t in ins], attrs) if ins else None

            memo[(id(n), 0)] = st or 'default'
        self._stype_cache = [memo.get((id(n), i), 'default') for n, i in self._symbol._outputs]
        return self._stype_cache

    def backward(self, out_grads=None, is_train=True):
        from .ndarray.ndarray import NDArray
        if not self._leaves:
            if not any(r != 'null' for r in self._grad_req.values()) or not self.grad_arrays:
                return
            # forward() ran without recording (is_train=False, the default): the reference still
            # computes gradients here (python/mxnet/executor.py:156), so replay the program with the
            # tape on, in the same train/predict mode as that forward
            self._run(getattr(self, '_last_is_train', False), True)
        if out_grads is None:
            out_grads = [None] * len(self._out_tensors)
        elif isinstance(out_grads, NDArray):
            out_grads = [out_grads]
        heads, hgs = [], []
        for o, g in zip(self._out_tensors, out_grads):
            if not o.requires_grad:
                continue
            heads.append(o)
            hgs.append(torch.ones_like(o) if g is None else g._data.to(o.dtype).reshape(o.shape))
        names = [n for n, _ in self._leaves]
        ts = [t for _, t in self._leaves]
        # no differentiable path (e.g. a cast to an integer type): every gradient is zero
        grads = (torch.autograd.grad(heads, ts, hgs, allow_unused=True, retain_graph=False)
                 if heads and ts else [None] * len(ts))
        gd = self.grad_dict
        with torch.no_grad():
            for n, g in zip(names, grads):
                buf = gd[n]
                if g is None:
                    if self._grad_req[n] == 'write':
                        buf._data.zero_()
                    continue
                if self._grad_req[n] == 'add':
                    buf._data.add_(g.to(buf._data.dtype))
                else:
                    buf._data.copy_(g)
            # inputs that cannot carry a gradient (integer arrays) get the zero gradient the
            # reference's backward writes for them
            got = set(names)
            for n, buf in gd.items():
                if n not in got and buf is not None and self._grad_req.get(n) == 'write':
                    buf._data.zero_()
        record = getattr(self, '_mon_record', None)
        if record and self._monitor_cb is not None:
            for name, args in reversed(record):
                for i, t in enumerate(args):
                    if not isinstance(t, torch.Tensor):
                        continue
                    g = self._mon_grads.get(id(t))
                    _call_monitor(self._monitor_cb, '%s_backward_in%d' % (name, i),
                                  NDArray(g if g is not None else torch.zeros_like(t)))
            self._mon_record = None
        box = getattr(self, '_failure_box', None)
        if box is not None and box[0] is not None:
            # gradients of a failed forward carry its (shared) failure
            for n in names:
                gd[n]._exc = box
        self._leaves = None

    def set_monitor_callback(self, callback, monitor_all=False):
        """``callback(name, NDArray)`` for every operator output (inputs too with ``monitor_all``)."""
        self._monitor_cb = callback
        self._monitor_all = monitor_all

    def copy_params_from(self, arg_params, aux_params=None, allow_extra_params=False):
        for name, array in arg_params.items():
            if name in self.arg_dict:
                self.arg_dict[name][:] = array.as_in_context(self.arg_dict[name].context)
            elif not allow_extra_params:
                raise ValueError('Find name "%s" that is not in the arguments' % name)
        if aux_params is not None:
            for name, array in aux_params.items():
                if name in self.aux_dict:
                    self.aux_dict[name][:] = array.as_in_context(self.aux_dict[name].context)
                elif not allow_extra_params:
                    raise ValueError('Find name %s that is not in the auxiliary states' % name)

    def reshape(self, partial_shaping=False, allow_up_sizing=False, **kwargs):
        """A new executor for new input shapes that shares memory with this one.

        Arrays whose shape is unchanged (typically the weights) are the same
        NDArrays; arrays that shrink become views of this executor's storage;
        arrays that grow are freshly allocated, which needs ``allow_up_sizing``.
        Output arrays are aliased the same way.
        """
        from .ndarray.ndarray import NDArray
        from . import ndarray as nd
        sym = self._symbol
        known = {n: a.shape for n, a in zip(sym.list_arguments(), self.arg_arrays)}
        for k in kwargs:
            if k not in known:
                raise MXNetError('reshape: %s is not an argument of the symbol' % k)
        if not partial_shaping:
            known = {k: v for k, v in known.items() if k not in kwargs}
            known.update(kwargs)
        else:
            known.update(kwargs)
        arg_shapes, out_shapes, aux_shapes = sym.infer_shape(**known)

        def fit(old, shape, what):
            if old is None:
                return None
            shape = tuple(shape)
            if shape == tuple(old.shape):
                return old
            n = 1
            for d in shape:
                n *= d
            if n <= old.size:
                return NDArray(old._data.reshape(-1)[:n].view(shape))
            if not allow_up_sizing:
                raise MXNetError('reshape: %s grows from %s to %s; pass allow_up_sizing=True'
                                 % (what, old.shape, shape))
            return nd.zeros(shape, ctx=old.context, dtype=old.dtype)

        names = sym.list_arguments()
        args = [fit(a, s, n) for a, s, n in zip(self.arg_arrays, arg_shapes, names)]
        grads = [fit(g, s, n + '_grad') for g, s, n in zip(self.grad_arrays, arg_shapes, names)]
        auxs = [fit(a, s, n) for a, s, n in zip(self.aux_arrays, aux_shapes, sym.list_auxiliary_states())]
        exe = Executor(sym, self._ctx, args, grads if any(g is not None for g in grads) else None,
                       dict(self._grad_req), auxs)
        if len(self.outputs) == len(out_shapes):
            try:
                exe.outputs = [fit(o, s, 'output') for o, s in zip(self.outputs, out_shapes)]
            except MXNetError:
                pass
        exe._monitor_cb, exe._monitor_all = self._monitor_cb, self._monitor_all
        return exe

    def get_optimized_symbol(self):
        """The graph this executor runs, after its bind-time passes."""
        return self._opt_symbol

    def debug_str(self):
        """The optimized graph plus the intermediate-storage plan ('Total N MB allocated')."""
        from .symbol import passes as _passes
        names = self._symbol.list_arguments()
        wanting = [n for n in names if self._grad_req.get(n, 'null') != 'null']
        grad = bool(_passes.grad_reachable(self._opt_symbol, set(wanting)))
        shapes = {n: a.shape for n, a in zip(names, self.arg_arrays)}
        dtypes = {n: a.dtype for n, a in zip(names, self.arg_arrays)}
        nbytes = _passes.memory_plan(self._opt_symbol, shapes, dtypes, grad)
        return '%s\nTotal %d MB allocated\n' % (self._opt_symbol.debug_str(), nbytes // (1 << 20))
