"""Imperative operator invocation and ``mx.nd.*`` function generation.

Parity: python/mxnet/ndarray/register.py (_make_ndarray_function) and
src/imperative/imperative.cc (Imperative::Invoke / RecordOp).  Instead of
generating ctypes stubs we bind each registered OpDef to a Python function that
runs the op's torch-level implementation under the right autograd mode.
"""
import contextlib

import sys

import torch

from .. import _state
from .. import engine as _engine
from .. import profiler as _profiler
from ..ops import amp_dispatch as _amp
from ..base import MXNetError, AsyncOpError
from ..ops import registry
from .ndarray import NDArray

_SKIP_KW = ('name', 'attr', 'out')
_NULL_CTX = contextlib.nullcontext()
_NP_CLS = [None]     # mx.np.ndarray, set when mx.numpy is imported


def _np_wrap(inputs, outs):
    """Outputs become mx.np.ndarray when any input is one (a legacy mx.nd operator on legacy arrays
    returns legacy arrays even under npx.set_np(), as in the reference; input-less creation ops follow
    the active mode)."""
    cls = _NP_CLS[0]
    if cls is None:
        return outs
    has_inputs = any(x is not None for x in inputs)
    if (_state.STATE.np_array and not has_inputs) or any(x is not None and x.__class__ is cls for x in inputs):
        for o in outs:
            if o.__class__ is NDArray:
                o.__class__ = cls
    return outs


def _split_args(op, args, kwargs):
    """Split python call arguments into (inputs, attrs, out)."""
    out = kwargs.pop('out', None)
    kwargs.pop('name', None)
    kwargs.pop('attr', None)
    attrs = {}
    inputs_pos = []
    extra_pos = []
    for a in args:
        if isinstance(a, NDArray) or (a is None and not extra_pos):
            inputs_pos.append(a)
        elif isinstance(a, (list, tuple)) and a and all(isinstance(x, NDArray) for x in a) and not extra_pos:
            inputs_pos.extend(a)
        else:
            extra_pos.append(a)
    named_inputs = {}
    for k, v in list(kwargs.items()):
        if isinstance(v, NDArray):
            named_inputs[k] = v
        elif v is None:
            spec = op.params.get(k)
            if spec is not None and isinstance(spec[0], str) and spec[0].endswith('?'):
                attrs[k] = None         # explicit None for an optional parameter (e.g. topk axis=None)
            continue
        else:
            attrs[k] = v
    if op.key_var_num_args and op.key_var_num_args not in attrs:
        attrs[op.key_var_num_args] = len(inputs_pos) + len(named_inputs)
    pattrs = op.parse_attrs(attrs)
    if extra_pos:
        # positional attribute values follow the declared param order
        pnames = [p for p in op.params if p not in attrs]
        for p, v in zip(pnames, extra_pos):
            pattrs[p] = registry.parse_value(op.params[p][0], v) if isinstance(v, str) else v
    arg_names = op.get_arg_names(pattrs) + op.get_aux_names(pattrs)
    if named_inputs:
        inputs = list(inputs_pos) + [None] * max(0, len(arg_names) - len(inputs_pos))
        for k, v in named_inputs.items():
            if k in arg_names:
                inputs[arg_names.index(k)] = v
            else:
                inputs.append(v)
        while inputs and inputs[-1] is None:
            inputs.pop()
    else:
        inputs = inputs_pos
    return inputs, pattrs, out


def _run(fn, tinputs, kw):
    rec = _state.STATE.recording
    if torch.is_grad_enabled() != rec:
        prev = not rec
        torch._C._set_grad_enabled(rec)
        try:
            return fn(*tinputs, **kw)
        finally:
            torch._C._set_grad_enabled(prev)
    return fn(*tinputs, **kw)


def _note_leaves(inputs):
    if _state.STATE.recording:
        tl = _state.STATE.tape_leaves
        for x in inputs:
            if x is not None and x._grad_req is not None:
                tl[id(x)] = x


def _failed_input(inputs):
    """The pending failure box of the first input produced by a failed operator, if any (the
    reference shares one exception slot along a chain of dependent operators)."""
    for x in inputs:
        box = getattr(x, '_exc', None) if x is not None else None
        if box is not None and box[0] is not None:
            return box
    return None


_SAMPLER_NAMES = frozenset(('_npi_normal', '_npi_uniform', '_npi_gamma', '_npi_exponential', '_npi_multinomial',
                            '_shuffle', '_npi_bernoulli', '_npi_sampler', '_npi_uniform_like', '_npi_normal_like',
                            '_npi_choice', '_npi_shuffle', '_npi_laplace', '_npi_logistic', '_npi_gumbel',
                            '_npi_pareto', '_npi_power', '_npi_rayleigh', '_npi_weibull', '_npi_chisquare',
                            '_npi_f', '_npi_beta', '_npi_lognormal', '_npi_poisson'))


def _is_sampler(name):
    """Operators whose output is a random draw (one predicate for the RNG failure box and for the
    graph passes, which must never merge two of them)."""
    return name.startswith(('_random_', '_sample_', '_npi_random', 'random_', 'sample_')) or name in _SAMPLER_NAMES


def _placeholder(attrs, inputs):
    """Output stand-in of an operator whose execution failed: zeros of the declared shape, so that
    dependent Python code (unpacking, shape arithmetic) keeps working until the error surfaces."""
    from ..base import torch_dtype
    shape = attrs.get('shape') or attrs.get('size') or (1,)
    shape = (shape,) if isinstance(shape, int) else tuple(shape)
    dt = attrs.get('dtype')
    try:
        td = torch_dtype(dt if dt not in (None, 'None') else 'float32')
    except Exception:   # pylint: disable=broad-except
        td = torch.float32
    ctx = attrs.get('ctx')
    dev = getattr(ctx, 'torch_device', None)
    if dev is None:
        dev = next((x._data.device for x in inputs if x is not None), torch.device('cpu'))
    return torch.zeros(shape, dtype=td, device=dev)


def _int_dtype_attr(attrs):
    dt = attrs.get('dtype')
    return dt is not None and str(dt).replace('torch.', '').startswith(('int', 'uint', 'bool'))


def _shadowed(arrays, attrs=None):
    """Integer variables among the inputs, or (while recording) a differentiable input cast to an
    integer result dtype: both run the float shadow path so the gradient survives the integer
    values (the reference's reductions with an integer dtype still back-propagate)."""
    if any(x is not None and getattr(x, '_idt', None) is not None for x in arrays):
        return True
    return attrs is not None and _state.STATE.recording and _int_dtype_attr(attrs) and \
        any(x is not None and x._data.requires_grad for x in arrays)


def _true_inputs(arrays):
    return [None if x is None else (x._data.detach().to(x._idt) if getattr(x, '_idt', None) is not None
                                    else x._data) for x in arrays]


def _merge_shadow(res_f, res_t):
    """Outputs of an operator on integer variables (see NDArray.attach_grad): the integer-input
    result's values and dtype, the float copy's gradient path.  Returns (tensor, int dtype or None)."""
    if not isinstance(res_f, torch.Tensor) or not res_f.requires_grad or not res_f.is_floating_point():
        return res_t, None
    if res_t.is_floating_point() or res_t.is_complex():
        return res_f.to(res_t.dtype) + (res_t - res_f.to(res_t.dtype)).detach(), None
    return res_f + (res_t.to(res_f.dtype) - res_f).detach(), res_t.dtype


# operators whose integer instantiation has a zero gradient in the reference (mshadow_op's
# mod_grad / mod_rgrad are 0 except for floating types)
INT_ZERO_GRAD = frozenset(('_npi_mod', '_npi_mod_scalar', '_npi_fmod', '_npi_fmod_scalar', '_mod', 'broadcast_mod',
                           '_mod_scalar', '_rmod_scalar'))


def _run_shadow(fn, inputs, kw, opname=None):
    """Run ``fn`` on arrays some of which are integer variables carried in float64."""
    with torch.no_grad():
        res_t = fn(*_true_inputs(inputs), **kw)
    if not _state.STATE.recording or opname in INT_ZERO_GRAD:
        return res_t, None
    kw_f = kw
    if _int_dtype_attr(kw):
        kw_f = dict(kw, dtype='float64')     # an integer result dtype keeps the float path differentiable
    res_f = _run(fn, [None if x is None else x._data for x in inputs], kw_f)
    if isinstance(res_t, (tuple, list)):
        pairs = [_merge_shadow(f, t) for f, t in zip(res_f, res_t)]
        return type(res_t)(p[0] for p in pairs), [p[1] for p in pairs]
    r, idt = _merge_shadow(res_f, res_t)
    return r, idt


def invoke(op, inputs, attrs, out=None):
    """Run ``op`` on NDArray ``inputs`` with parsed ``attrs``.

    Failures of the operator's execution (AsyncOpError) and failed inputs do not raise here: the
    outputs carry the failure to the next synchronisation point (engine.rethrow / rethrow_all)."""
    tin = [None if x is None else x._data for x in inputs]
    if _engine._JOIN_HOOKS and not _engine._workers.depth:
        _engine.run_join_hooks()      # e.g. weight gradients still running on a side stream
    _note_leaves(inputs)
    if _amp.active:
        tin = _amp.cast_inputs(op.name, tin, attrs)
    if op.name in _BN_OPS:
        _check_storage(op.name, [getattr(x, 'stype', 'default') for x in inputs], attrs)
    box = _failed_input(inputs)
    sampler = _is_sampler(op.name)
    if sampler and box is None:
        from .. import engine
        box = engine.rng_failure()
    idts = None
    ws_sid = ws_stream = None
    sctx = _NULL_CTX
    if _engine.GPU_WORKERS > 1 and not _engine._workers.depth:
        # MXNET_GPU_WORKER_NTHREADS > 1: the operator's worker stream (engine.op_stream); operators
        # nested in its body (Custom ops) run on that stream without bookkeeping
        ws_sid, ws_stream = _engine.op_stream(tin)
        if ws_stream is not None:
            sctx = torch.cuda.stream(ws_stream)
            _engine._workers.depth += 1
    try:
        with sctx:
            if _shadowed(inputs, attrs) and not _amp.active:
                res, idts = _run_shadow(op.fn, inputs, attrs, op.name)
            elif _profiler.active_imperative:
                with _profiler.op_span(_profiler.current_scope() + op.name):
                    res = _run(op.fn, tin, attrs)
            else:
                res = _run(op.fn, tin, attrs)
    except AsyncOpError as e:
        from .. import engine
        if box is None:
            box = engine.record_failure(e)
        if sampler:
            engine.set_rng_failure(box)
        res = _placeholder(attrs, inputs)
    except MXNetError:
        if box is None:
            raise
        res = _placeholder(attrs, inputs)    # an op fed garbage by a failed input: the input's error wins
    except (RuntimeError, IndexError) as e:
        # operator failures surface as MXNetError (a RuntimeError), as from the reference's C API
        if isinstance(e, IndexError):
            from ..base import MXNetIndexError
            raise MXNetIndexError('Error in operator %s: %s' % (op.name, e)) from e
        raise MXNetError('Error in operator %s: %s' % (op.name, e)) from e
    finally:
        if ws_stream is not None:
            _engine._workers.depth -= 1
            if sys.exc_info()[0] is not None:
                _engine._workers.pending.pop()      # the operator raised: no op_done will close it
    nvis = op.get_num_visible_outputs(attrs)
    if isinstance(res, (tuple, list)):
        outs = [NDArray(r) for r in res[:nvis]]
    else:
        outs = [NDArray(res)]
    if ws_sid is not None:
        _engine.op_done([o._data for o in outs], ws_sid)
    st = _kept_stype(op.name, inputs, attrs) if out is None else None
    if st is not None and not _state.STATE.recording:
        from . import sparse
        outs = [sparse.cast_storage(o, st) for o in outs]
    _np_wrap(inputs, outs)
    if idts is not None:
        for o, d in zip(outs, idts if isinstance(idts, list) else [idts]):
            if d is not None:
                o._idt = d
    if _state.STATE.recording:
        hist = (op.name, attrs, list(inputs))       # for autograd.get_symbol
        for i, o in enumerate(outs):
            o._recorded = True
            o._hist = (hist, i)
    if _profiler.active_memory and out is None:
        for o in outs:
            _profiler.memory_alloc(o)
    if box is not None:
        for o in outs:
            o._exc = box
    hctx = attrs.get('ctx') if 'ctx' in attrs else next(
        (x._host_ctx for x in inputs if x is not None and getattr(x, '_host_ctx', None) is not None), None)
    if hctx is not None:
        from .ndarray import _tag_host_ctx
        for o in outs:
            _tag_host_ctx(o, hctx)
    if out is not None:
        targets = out if isinstance(out, (list, tuple)) else [out]
        for t, o in zip(targets, outs):
            if _state.STATE.recording and o._data.requires_grad:
                t._data = o._data
            else:
                with torch.no_grad(), (torch.cuda.stream(ws_stream) if ws_stream is not None else _NULL_CTX):
                    if ws_sid is not None:
                        _engine.op_written(t._data, ws_sid, ws_stream)
                    t._data.copy_(o._data.reshape(t.shape) if o.shape != t.shape and o.size == t.size else o._data)
        return out
    if len(outs) == 1:
        return outs[0]
    return outs


# operators whose output keeps a sparse input's storage type (reference: their FInferStorageType --
# zero-preserving unary math, row selection of a csr matrix); everything else falls back to dense
_ZERO_PRESERVING = frozenset((
    'abs', 'sign', 'round', 'rint', 'ceil', 'floor', 'trunc', 'fix', 'square', 'sqrt', 'sin', 'tan',
    'arcsin', 'arctan', 'sinh', 'tanh', 'arcsinh', 'arctanh', 'expm1', 'log1p', 'relu', 'negative',
    'degrees', 'radians', '_copy', 'identity', 'cbrt', 'Cast', 'cast', 'stop_gradient', 'BlockGrad'))


_BN_OPS = ('BatchNorm', 'BatchNorm_v1', 'CuDNNBatchNorm', '_contrib_BatchNormWithReLU', 'BatchNormWithReLU')


def _check_storage(name, stypes, attrs):
    """Storage combinations an operator rejects at storage inference (reference:
    src/operator/nn/batch_norm.cc:528, BatchNormStorageType: ``fix_gamma`` with sparse inputs)."""
    if name in _BN_OPS and any(s != 'default' for s in stypes):
        fg = attrs.get('fix_gamma', True)
        if fg if isinstance(fg, bool) else str(fg) in ('True', 'true', '1'):
            raise MXNetError('fix_gamma=True is not supported for sparse ndarrays. Tracked at #11647')


def _kept_stype(name, inputs, attrs):
    x = inputs[0] if inputs else None
    st = getattr(x, 'stype', 'default') if x is not None else 'default'
    if st == 'default':
        return None
    if name in _ZERO_PRESERVING:
        return st
    if name == 'clip' and st != 'default':
        lo, hi = attrs.get('a_min', 0), attrs.get('a_max', 0)
        return st if (lo is None or float(lo) <= 0) and (hi is None or float(hi) >= 0) else None
    if name in ('_contrib_quadratic', 'quadratic') and float(attrs.get('c', 0.0) or 0.0) == 0.0:
        return st                           # a*x^2 + b*x keeps zeros
    if st == 'row_sparse' and name == '_square_sum':
        ax = attrs.get('axis')
        ax = ax[0] if isinstance(ax, (tuple, list)) and len(ax) == 1 else ax
        if ax == 1 and bool(attrs.get('keepdims', False)):
            return 'row_sparse'             # per-row sums of a row_sparse matrix stay row_sparse
    if st == 'csr' and name == 'take' and int(attrs.get('axis', 0)) == 0:
        return 'csr'
    if st == 'csr' and name in ('slice', 'crop', '_slice'):
        return 'csr'
    return None


def invoke_by_name(name, args, kwargs):
    op = registry.get(name)
    inputs, attrs, out = _split_args(op, args, dict(kwargs))
    return invoke(op, inputs, attrs, out)


def invoke_fn(fn, arrays):
    """Run an ad-hoc torch function (reshape, astype, ...) with autograd semantics."""
    _note_leaves(arrays)
    idt = None
    if _shadowed(arrays):
        res, idt = _run_shadow(fn, arrays, {})
    else:
        res = _run(fn, [a._data for a in arrays], {})
    out = _np_wrap(arrays, [NDArray(res)])[0]
    if idt is not None:
        out._idt = idt
    if _state.STATE.recording:
        out._recorded = True
    box = _failed_input(arrays)
    if box is not None:
        out._exc = box
    return out


def make_op_function(name):
    op = registry.get(name)

    def f(*args, **kwargs):
        inputs, attrs, out = _split_args(op, args, dict(kwargs))
        return invoke(op, inputs, attrs, out)
    f.__name__ = name
    f.__qualname__ = name
    params = ', '.join('%s=%r' % (k, v[1]) for k, v in op.params.items())
    args = op.arg_names if not callable(op.arg_names) else ['*data']
    f.__doc__ = '%s(%s%s%s)\n\nMXNet operator `%s` (see src/operator for reference semantics).' % (
        name, ', '.join(args), ', ' if params else '', params, name)
    return f


def populate(namespace, prefix_map=None):
    """Fill ``namespace`` (a dict) with functions for every registered op."""
    for name in registry.list_ops():
        if name not in namespace:
            namespace[name] = make_op_function(name)
    return namespace
