"""Gluon parameters.

Parity: python/mxnet/gluon/parameter.py (Parameter, Constant, ParameterDict,
DeferredInitializationError, deferred init, multi-context replicas, grad_req,
lr_mult/wd_mult, save/load, cast, var, zero_grad, reset_ctx).

Design here: a Parameter is a list of per-context replicas (NDArrays over torch
tensors; ``_data`` / ``_grad``) plus a lookup table keyed by ``(device type,
device id)``.  Until its shape is known a parameter holds a ``_PendingInit``
record (initializer, contexts, fallback initializer, optional data to load) and
materialises when the first forward pass has inferred the shape.  CPU contexts
``cpu(k)`` all live in host memory; replicas on them are labelled with their
context so ``data(cpu(k))`` / ``list_ctx()`` behave as in the reference.
"""
import warnings
from collections import OrderedDict

import numpy as np
import torch

from .. import _state, autograd, initializer
from ..base import MXNetError, torch_dtype, dtype_name
from ..context import Context, cpu, current_context
from ..ndarray.ndarray import NDArray, _tag_host_ctx
from .. import ndarray as nd

__all__ = ['DeferredInitializationError', 'Parameter', 'Constant', 'ParameterDict', 'tensor_types']

tensor_types = (NDArray,)

_STYPES = ('default', 'row_sparse', 'csr')


class DeferredInitializationError(MXNetError):
    """Raised when a parameter is used before its deferred initialisation ran."""


def _shape_known(shape):
    return bool(shape) and all(d > 0 for d in shape)


def _as_ctx_list(ctx):
    if ctx is None:
        return [current_context()]
    return [ctx] if isinstance(ctx, Context) else list(ctx)


def _ctx_key(ctx):
    return (ctx.device_typeid, ctx.device_id)


def _to_np_class(arrs):
    """Under ``npx.set_np()`` parameters hand out ``mx.np.ndarray`` (same object, NumPy semantics)."""
    from ..numpy import ndarray as _npnd
    for a in arrs:
        if a is not None and a.__class__ is NDArray:
            a.__class__ = _npnd


class _PendingInit:
    """What ``initialize`` was asked for while the shape was still unknown."""
    __slots__ = ('init', 'ctx', 'default_init', 'data')

    def __init__(self, init, ctx, default_init, data=None):
        self.init, self.ctx, self.default_init, self.data = init, list(ctx), default_init, data


class Parameter:
    """A Block's parameter: replicated data (+grad) on one or more contexts."""

    def __init__(self, name, grad_req='write', shape=None, dtype=np.float32, lr_mult=1.0, wd_mult=1.0,
                 init=None, allow_deferred_init=False, differentiable=True, stype='default',
                 grad_stype='default'):
        if stype not in _STYPES:
            raise AssertionError("Invalid stype '%s' for Parameter '%s', expected one of %s" % (stype, name, _STYPES))
        if grad_stype not in _STYPES:
            raise AssertionError("Invalid grad_stype '%s' for Parameter '%s', expected one of %s"
                                 % (grad_stype, name, _STYPES))
        self.name = name
        self._shape = (shape,) if isinstance(shape, int) else shape
        self._dtype = dtype
        self._stype, self._grad_stype = stype, grad_stype
        self._differentiable = differentiable
        self._allow_deferred_init = allow_deferred_init
        self.lr_mult, self.wd_mult, self.init = lr_mult, wd_mult, init
        # replicas
        self._data = None          # [NDArray] per context, or None before initialisation
        self._grad = None          # [NDArray] gradient buffers (grad_req != 'null')
        self._ctx_list = None      # contexts, in replica order
        self._slot = {}            # (device type, device id) -> replica index
        self._deferred_init = None  # _PendingInit while waiting for the shape
        self._var = None
        self._trainer = None
        self._grad_req = None
        self.grad_req = grad_req

    def __repr__(self):
        return 'Parameter {} (shape={}, dtype={})'.format(self.name, self.shape, self.dtype)

    # ------------------------------------------------------------------ attributes
    @property
    def grad_req(self):
        return self._grad_req

    @grad_req.setter
    def grad_req(self, req):
        if req not in ('write', 'add', 'null'):
            raise AssertionError("grad_req must be one of 'write', 'add', or 'null', but got '%s'" % req)
        req = req if self._differentiable else 'null'
        if req == self._grad_req:
            return
        self._grad_req = req
        if self._data is None:
            return
        if req == 'null':
            if self._grad is not None:
                self._grad = None
                for arr in self._data:
                    arr.attach_grad('null')
        else:
            self._init_grad()

    @property
    def dtype(self):
        return self._dtype

    @dtype.setter
    def dtype(self, dtype):
        self.cast(dtype)

    @property
    def shape(self):
        return self._shape

    @shape.setter
    def shape(self, new_shape):
        new_shape = tuple(new_shape)
        if self._shape is not None:
            ok = len(self._shape) == len(new_shape) and all(
                old in (0, -1, new) for old, new in zip(self._shape, new_shape))
            if not ok:
                raise AssertionError("Expected shape %s is incompatible with given shape %s."
                                     % (str(new_shape), str(self._shape)))
        self._shape = new_shape

    @property
    def stype(self):
        return self._stype

    @property
    def grad_stype(self):
        return self._grad_stype

    def _set_trainer(self, trainer):
        """Attach the Trainer that updates this parameter (a sparse parameter allows only one)."""
        if (self._stype != 'default' and trainer is not None and self._trainer is not None
                and self._trainer is not trainer):
            raise RuntimeError("Failed to set the trainer for Parameter '%s' because it was already set. More "
                               "than one trainers for a %s Parameter is not supported." % (self.name, self._stype))
        self._trainer = trainer

    # ------------------------------------------------------------------ replica lookup
    def _not_ready_error(self):
        if self._deferred_init is not None:
            return DeferredInitializationError(
                "Parameter '%s' has not been initialized yet because initialization was deferred. Actual "
                "initialization happens during the first forward pass. Please pass one batch of data through "
                "the network before accessing Parameters." % self.name)
        return RuntimeError("Parameter '%s' has not been initialized. Note that you should initialize "
                            "parameters and create Trainer with Block.collect_params() instead of Block.params "
                            "because the later does not include Parameters of nested child Blocks" % self.name)

    def _check_and_get(self, arrays, ctx):
        """``arrays`` (this parameter's ``_data`` or ``_grad``) on ``ctx``; ``ctx=list`` -> all of them,
        ``ctx=None`` -> the only replica (or the one on the current context)."""
        if arrays is None:
            raise self._not_ready_error()
        if _state.STATE.np_array:
            _to_np_class(arrays)
        if ctx is list:
            return arrays
        if ctx is None:
            if len(arrays) == 1:
                return arrays[0]
            ctx = current_context()
        idx = self._slot.get(_ctx_key(ctx))
        if idx is None and ctx.device_typeid in (1, 3, 5):
            # every CPU context is host memory: any host replica serves
            idx = next((i for i, c in enumerate(self._ctx_list) if c.device_typeid in (1, 3, 5)), None)
        if idx is None:
            raise RuntimeError("Parameter '%s' was not initialized on context %s. It was only initialized on %s."
                               % (self.name, str(ctx), str(self._ctx_list)))
        return arrays[idx]

    # ------------------------------------------------------------------ initialisation
    def initialize(self, init=None, ctx=None, default_init=initializer.Uniform(), force_reinit=False):
        """Create the replicas on ``ctx`` with ``init`` (else this parameter's own init, else
        ``default_init``); defer until the shape is known when allowed."""
        if self._data is not None and not force_reinit:
            warnings.warn("Parameter '%s' is already initialized, ignoring. Set force_reinit=True to "
                          "re-initialize." % self.name, stacklevel=2)
            return
        self._data = self._grad = None
        pending = _PendingInit(init if init is not None else (self.init if self.init is not None else default_init),
                               _as_ctx_list(ctx), default_init)
        if not _shape_known(self.shape):
            if not self._allow_deferred_init:
                raise ValueError("Cannot initialize Parameter '%s' because it has invalid shape: %s." %
                                 (self.name, str(self.shape)))
            self._deferred_init = pending
            return
        self._deferred_init = pending
        self._finish_deferred_init()

    def _finish_deferred_init(self):
        """Materialise a deferred parameter (its shape has been inferred by now)."""
        pending, self._deferred_init = self._deferred_init, None
        if pending is None:
            return
        if not _shape_known(self.shape):
            raise AssertionError("Cannot initialize Parameter '%s' because it has invalid shape: %s. Please "
                                 "specify in_units, in_channels, etc for `Block`s." % (self.name, str(self.shape)))
        with autograd.pause():
            data = pending.data
            if data is None:
                data = nd.zeros(self.shape, dtype=self.dtype, ctx=cpu())
                initializer.create(pending.default_init)(
                    initializer.InitDesc(self.name, {'__init__': pending.init}), data)
            self._init_impl(data, pending.ctx)

    def _init_impl(self, data, ctx_list):
        """One replica of ``data`` per context (cast to this parameter's dtype), then gradients."""
        self._ctx_list = list(ctx_list)
        self._slot = {}
        for i, c in enumerate(self._ctx_list):
            self._slot.setdefault(_ctx_key(c), i)
        src = data._data.detach() if isinstance(data, NDArray) else torch.as_tensor(np.asarray(data))
        td = torch_dtype(self.dtype)
        # replicas are dense tensors (autograd and the kvstore work on them); a sparse parameter's
        # replicas carry its storage type
        self._data = [_tag_host_ctx(NDArray(src.to(device=c.torch_device, dtype=td, copy=True)), c)
                      for c in self._ctx_list]
        for arr in self._data:
            arr._stype = self._stype
        self._init_grad()

    def _init_grad(self):
        if self._grad_req == 'null':
            self._grad = None
            return
        gst = self._grad_stype
        if not self._data[0]._data.is_floating_point():
            # integer parameters (e.g. quantized weights) have a gradient buffer that autograd never
            # writes (torch cannot differentiate integer tensors)
            self._grad = [NDArray(torch.zeros_like(arr._data)) for arr in self._data]
        else:
            for arr in self._data:
                arr.attach_grad(self._grad_req, stype=gst)
            self._grad = [arr._grad for arr in self._data]
        for arr, c in zip(self._grad, self._ctx_list):
            if arr is not None:
                _tag_host_ctx(arr, c)
        if self._trainer is not None and hasattr(self._trainer, '_on_param_grad_reset'):
            self._trainer._on_param_grad_reset(self)

    def _load_init(self, data, ctx, cast_dtype=False, dtype_source='current'):
        """Initialise (or overwrite) from loaded ``data``, checking shape and dtype."""
        if cast_dtype and dtype_source not in ('current', 'saved'):
            raise AssertionError("dtype_source must be 'current' or 'saved'")
        if self.shape:
            wildcard = -1 if -1 in self.shape else 0
            if len(self.shape) != len(data.shape) or any(
                    mine not in (wildcard, got) for mine, got in zip(self.shape, data.shape)):
                raise AssertionError("Failed loading Parameter '%s' from saved params: shape incompatible expected "
                                     "%s vs saved %s" % (self.name, str(self.shape), str(data.shape)))
            self.shape = tuple(got if mine == wildcard else mine for mine, got in zip(self.shape, data.shape))
        if self.dtype and dtype_name(self.dtype) != dtype_name(data.dtype):
            if not cast_dtype:
                raise AssertionError(
                    "Failed loading Parameter '%s' from saved params: dtype incompatible expected %s vs saved %s. "
                    "Set cast_dtype=True to cast the dtype of saved params." % (self.name, str(self.dtype),
                                                                                 str(data.dtype)))
            if dtype_source == 'current':
                data = data.astype(self.dtype, copy=False)
            else:
                self.cast(data.dtype)      # the replicas take the saved dtype too
        want = None if ctx is None else _as_ctx_list(ctx)
        if self._data is None:
            if self._deferred_init is not None:
                have = self._deferred_init.ctx
                if want is not None and set(want) != set(have):
                    raise AssertionError("Failed to load Parameter '%s' on %s because it was previous initialized "
                                         "on %s." % (self.name, str(want), str(have)))
                want = have
            self._init_impl(data, want or [cpu()])
        else:
            if want is not None and set(want) != set(self.list_ctx()):
                raise AssertionError("Failed to load Parameter '%s' on %s because it was previous initialized on %s."
                                     % (self.name, str(want), str(self.list_ctx())))
            self.set_data(data)
        self._deferred_init = None
        # weights held by the kvstore are stale now: the trainer re-initialises its store
        tr = self._trainer
        if (tr is not None and getattr(tr, '_kv_initialized', False) and getattr(tr, '_update_on_kvstore', False)
                and self not in tr._params_to_init):
            tr._reset_kvstore()

    def _reduce(self):
        """One host copy of the value (replicas averaged; a row_sparse parameter as a RowSparseNDArray
        holding every row)."""
        host = cpu()
        reps = self._all_data()
        tr = self._trainer
        if self._stype == 'row_sparse' and tr is not None and getattr(tr, '_kvstore', None) is not None:
            # the kvstore holds the authoritative weight: pull every row first (reference parameter.py:400-403)
            all_rows = nd.arange(0, self.shape[0], dtype='int64', ctx=reps[0].context)
            tr._row_sparse_pull(self, reps if len(reps) > 1 else reps[0], all_rows, full_idx=True)
        if len(reps) == 1:
            val = NDArray(reps[0]._data.detach().to('cpu', copy=True))
        else:
            val = nd.add_n(*[NDArray(r._data.detach().to('cpu', copy=True)) for r in reps]) / len(reps)
        if self._stype == 'row_sparse':
            from ..ndarray import sparse as _sp
            return _sp.RowSparseNDArray(val._data, ctx=host)
        return val

    def reset_ctx(self, ctx):
        """Move the replicas (or the pending initialisation) to ``ctx``."""
        ctx = _as_ctx_list(ctx)
        if self._data:
            value = self._reduce()
            with autograd.pause():
                self._init_impl(value, ctx)
        elif self._deferred_init is not None:
            self._deferred_init.ctx = list(ctx)
        else:
            raise ValueError("Cannot reset context for Parameter '%s' because it has not been initialized."
                             % self.name)

    def set_data(self, data):
        """Overwrite every replica with ``data`` (or stash it for a pending initialisation)."""
        self.shape = data.shape
        if self._data is None:
            if self._deferred_init is None:
                raise AssertionError("Parameter '%s' has not been initialized" % self.name)
            self._deferred_init.data = data
            return
        src = data._data if isinstance(data, NDArray) else torch.as_tensor(np.asarray(data))
        with torch.no_grad():
            for arr in self._all_data():
                arr._data.copy_(src.to(arr._data.device, arr._data.dtype))

    # ------------------------------------------------------------------ access
    def _get_row_sparse(self, ctx, row_id):
        if not isinstance(row_id, NDArray):
            raise TypeError('row_id must have NDArray type, but %s is given' % type(row_id))
        if self._trainer is None:
            raise RuntimeError("Cannot get row_sparse data for Parameter '%s' when no Trainer is created with "
                               "it." % self.name)
        got = self._check_and_get(self._data, ctx)
        # only the requested rows are fetched from the kvstore into the local copies
        self._trainer._row_sparse_pull(self, got, row_id)
        if _state.STATE.recording:
            # inside autograd.record() the replica itself (the leaf whose gradient the trainer reads)
            return got
        # outside record(): a copy holding only the pulled rows, like the reference's pulled row_sparse
        # array; the replica itself keeps every row (it is what _reduce / save_parameters read)
        if isinstance(got, list):
            return [self._masked_rows(a, row_id) for a in got]
        return self._masked_rows(got, row_id)

    @staticmethod
    def _masked_rows(arr, row_id):
        """A new array equal to replica ``arr`` on the rows ``row_id`` and zero elsewhere."""
        t = arr._data
        rows = row_id._data.to(device=t.device, dtype=torch.int64).reshape(-1)
        with torch.no_grad():
            out = torch.zeros_like(t)
            out[rows] = t[rows]
        return NDArray(out)

    def row_sparse_data(self, row_id):
        """The rows ``row_id`` of a row_sparse parameter, on ``row_id``'s context."""
        if self._stype != 'row_sparse':
            raise RuntimeError("Cannot return a copy of Parameter %s via row_sparse_data() because its storage "
                               "type is %s. Please use data() instead." % (self.name, self._stype))
        return self._get_row_sparse(row_id.context, row_id)

    def list_row_sparse_data(self, row_id):
        if self._stype != 'row_sparse':
            raise RuntimeError("Cannot return copies of Parameter '%s' on all contexts via "
                               "list_row_sparse_data() because its storage type is %s. Please use data() "
                               "instead." % (self.name, self._stype))
        return self._get_row_sparse(list, row_id)

    def data(self, ctx=None):
        if self._stype != 'default':
            raise RuntimeError("Cannot return a copy of Parameter '%s' on ctx %s via data() because its storage "
                               "type is %s. Please use row_sparse_data() instead." % (self.name, str(ctx), self._stype))
        return self._check_and_get(self._data, ctx)

    def _all_data(self):
        """Per-context data arrays whatever the storage type (framework-internal accessor)."""
        return self._check_and_get(self._data, list)

    def list_data(self):
        if self._stype != 'default':
            raise RuntimeError("Cannot return copies of Parameter '%s' on all contexts via list_data() because its "
                               "storage type is %s. Please use row_sparse_data() instead." % (self.name, self._stype))
        return self._all_data()

    def _grads_or_raise(self):
        if self._data is not None and self._grad is None:
            raise RuntimeError("Cannot get gradient array for Parameter '%s' because grad_req='null'" % self.name)
        return self._grad

    def grad(self, ctx=None):
        return self._check_and_get(self._grads_or_raise(), ctx)

    def list_grad(self):
        return self._check_and_get(self._grads_or_raise(), list)

    def list_ctx(self):
        if self._data is not None:
            return self._ctx_list
        if self._deferred_init is not None:
            return self._deferred_init.ctx
        raise RuntimeError("Parameter '%s' has not been initialized" % self.name)

    def zero_grad(self):
        if self._grad is not None:
            with torch.no_grad():
                torch._foreach_zero_([g._data for g in self._grad])

    def var(self):
        """The Symbol variable standing for this parameter in hybridized graphs."""
        if self._var is None:
            from .. import symbol
            self._var = symbol.var(self.name, shape=self.shape, dtype=self.dtype, lr_mult=self.lr_mult,
                                   wd_mult=self.wd_mult, init=self.init, stype=self._stype)
        return self._var

    def cast(self, dtype):
        self._dtype = dtype
        if self._data is None:
            return
        td = torch_dtype(dtype)
        with autograd.pause():
            for arr in self._data:
                arr._data = arr._data.detach().to(td)
            self._init_grad()


class Constant(Parameter):
    """A constant parameter (grad_req='null') initialised with ``value``."""

    def __init__(self, name, value):
        value = value if isinstance(value, NDArray) else nd.array(value)
        self.value = value

        class _ConstInit(initializer.Initializer):
            def _init_weight(self, _, arr):
                initializer.Initializer._set(arr, value._data)
        key = 'Constant_{}_{}'.format(name, id(self))
        initializer._REGISTRY[key.lower()] = _ConstInit
        super().__init__(name, grad_req='null', shape=value.shape, dtype=value.dtype, init=key)

    def __repr__(self):
        return 'Constant {} (shape={}, dtype={})'.format(self.name, self.shape, self.dtype)

    @property
    def grad_req(self):
        return 'null'

    @grad_req.setter
    def grad_req(self, req):
        if req != 'null':
            warnings.warn('Constant parameter "{}" does not support grad_req other than "null", and new value '
                          '"{}" is ignored.'.format(self.name, req))
        self._grad_req = 'null'


def _merge_shapes(wanted, stored):
    """Unify a requested and a stored shape (0 / -1 = unknown); None when they conflict."""
    if len(wanted) != len(stored):
        return None
    out = []
    for a, b in zip(wanted, stored):
        if a == b or a in (0, -1):
            out.append(b)
        elif b in (0, -1):
            out.append(a)
        else:
            return None
    return tuple(out)


class ParameterDict:
    """An ordered dictionary of Parameters with a shared name prefix.  ``shared``: another
    ParameterDict whose entries are adopted (by reference) when asked for by name."""

    def __init__(self, prefix='', shared=None):
        self._prefix = prefix
        self._params = OrderedDict()
        self._shared = shared

    def __repr__(self):
        head = self._prefix + ' ' if self._prefix else ''
        return '{}(\n{}\n)'.format(head, '\n'.join('  ' + repr(p) for p in self.values()))

    def __getitem__(self, key):
        return self._params[key]

    def __iter__(self):
        return iter(self._params)

    def __len__(self):
        return len(self._params)

    def __contains__(self, key):
        return key in self._params

    def items(self):
        return self._params.items()

    def keys(self):
        return self._params.keys()

    def values(self):
        return self._params.values()

    @property
    def prefix(self):
        return self._prefix

    def _lookup(self, full_name):
        p = self._params.get(full_name)
        if p is None and self._shared is not None:
            p = self._shared._params.get(full_name)
            if p is not None:
                self._params[full_name] = p
        return p

    # kept for code written against the reference's private name
    _get_impl = _lookup

    def get(self, name, **kwargs):
        """The parameter ``prefix + name``: created with ``kwargs`` if new, else checked against them
        (unknown dimensions of a stored shape are filled in from a requested one)."""
        full = self._prefix + name
        p = self._lookup(full)
        if p is None:
            p = self._params[full] = Parameter(full, **kwargs)
            return p
        for attr, want in kwargs.items():
            have = getattr(p, attr, None)
            if have is None:
                setattr(p, attr, want)
                continue
            if attr == 'shape':
                merged = _merge_shapes(tuple(want), tuple(have)) if want is not None else have
                if merged is not None:
                    p._shape = merged
                    continue
            elif attr == 'dtype' and np.dtype(want) == np.dtype(have):
                continue
            if want is not None and want != have:
                raise AssertionError("Cannot retrieve Parameter '%s' because desired attribute does not match with "
                                     "stored for attribute '%s': desired '%s' vs stored '%s'."
                                     % (full, attr, str(want), str(have)))
        return p

    def get_constant(self, name, value=None):
        full = self._prefix + name
        p = self._lookup(full)
        if p is None:
            if value is None:
                raise KeyError("No constant named '{}'. Please specify value if you want to create a new "
                               "constant.".format(full))
            p = self._params[full] = Constant(full, value)
        elif value is not None and not isinstance(p, Constant):
            raise AssertionError("Parameter '{}' already exists but it is not a constant.".format(full))
        return p

    def update(self, other):
        """Adopt every entry of ``other``; the same name must mean the same Parameter."""
        clash = next((k for k, v in other.items() if k in self._params and self._params[k] is not v), None)
        if clash is not None:
            raise AssertionError("Cannot update self with other because they have different Parameters with the "
                                 "same name '%s'" % clash)
        self._params.update(other.items())

    def initialize(self, init=initializer.Uniform(), ctx=None, verbose=False, force_reinit=False):
        if verbose:
            init.set_verbosity(verbose=verbose)
        for p in self.values():
            p.initialize(None, ctx, init, force_reinit=force_reinit)

    def zero_grad(self):
        grads = [g._data for p in self.values() if p._grad is not None for g in p._grad]
        if grads:
            with torch.no_grad():
                torch._foreach_zero_(grads)

    def reset_ctx(self, ctx):
        for p in self.values():
            p.reset_ctx(ctx)

    def list_ctx(self):
        seen = []
        for p in self.values():
            for c in p.list_ctx():
                if c not in seen:
                    seen.append(c)
        return seen

    def setattr(self, name, value):
        for p in self.values():
            setattr(p, name, value)

    def save(self, filename, strip_prefix=''):
        """Save every parameter under its name minus ``strip_prefix``."""
        out = {}
        for p in self.values():
            if not p.name.startswith(strip_prefix):
                raise ValueError("Prefix '%s' is to be striped before saving, but Parameter's name '%s' does not "
                                 "start with '%s'." % (strip_prefix, p.name, strip_prefix))
            out[p.name[len(strip_prefix):]] = p._reduce()
        nd.save(filename, out)

    def load(self, filename, ctx=None, allow_missing=False, ignore_extra=False, restore_prefix='',
             cast_dtype=False, dtype_source='current'):
        if restore_prefix:
            bad = next((k for k in self.keys() if not k.startswith(restore_prefix)), None)
            if bad is not None:
                raise AssertionError("restore_prefix is '%s' but Parameters name '%s' does not start with '%s'"
                                     % (restore_prefix, bad, restore_prefix))
        loaded = nd.load(filename) if isinstance(filename, str) else filename
        self.load_dict(loaded, ctx, allow_missing, ignore_extra, restore_prefix, filename, cast_dtype, dtype_source)

    def load_dict(self, param_dict, ctx=None, allow_missing=False, ignore_extra=False, restore_prefix='',
                  filename=None, cast_dtype=False, dtype_source='current'):
        """Load ``{name: NDArray}`` (names relative to ``restore_prefix``; ``arg:`` / ``aux:`` tags of
        Module checkpoints are dropped)."""
        pairs = param_dict.items() if isinstance(param_dict, dict) else param_dict
        values = {}
        for k, v in pairs:
            if k.startswith(('arg:', 'aux:')):
                k = k[4:]
            values[restore_prefix + k] = v
        where = "file: %s" % filename if filename else "param_dict"
        cut = len(restore_prefix)
        if not allow_missing:
            missing = next((k for k in self.keys() if k not in values), None)
            if missing is not None:
                raise AssertionError("Parameter '%s' is missing in %s, which contains parameters: %s. Please make "
                                     "sure source and target networks have the same prefix."
                                     % (missing[cut:], where, str(list(values)[:10])))
        for k, v in values.items():
            if k in self._params:
                self._params[k]._load_init(v, ctx, cast_dtype=cast_dtype, dtype_source=dtype_source)
            elif not ignore_extra:
                raise AssertionError("Parameter '%s' loaded from %s is not present in ParameterDict, choices are: "
                                     "%s. Set ignore_extra to True to ignore. Please make sure source and target "
                                     "networks have the same prefix." % (k[cut:], where, str(list(self._params)[:10])))
