"""Gluon parameters.

Parity: python/mxnet/gluon/parameter.py (Parameter, Constant, ParameterDict,
DeferredInitializationError, deferred init, multi-context replicas, grad_req,
lr_mult/wd_mult, save/load, cast, var, zero_grad, reset_ctx).
"""
import re
import warnings
from collections import OrderedDict

import numpy as np
import torch

from .. import _state, autograd, initializer
from ..base import MXNetError, np_dtype, torch_dtype, dtype_name
from ..context import Context, cpu, current_context
from ..ndarray.ndarray import NDArray
from .. import ndarray as nd

__all__ = ['DeferredInitializationError', 'Parameter', 'Constant', 'ParameterDict', 'tensor_types']

tensor_types = (NDArray,)


class DeferredInitializationError(MXNetError):
    """Raised when a parameter is used before its deferred initialisation ran."""


def _shape_known(shape):
    return shape is not None and all(d > 0 for d in shape) and len(shape) > 0


def _to_np_class(arrs):
    """Under ``npx.set_np()`` parameters hand out ``mx.np.ndarray`` (same object, NumPy semantics)."""
    from ..numpy import ndarray as _npnd
    for a in arrs:
        if a is not None and a.__class__ is NDArray:
            a.__class__ = _npnd


class Parameter:
    """A Block's parameter: replicated data (+grad) on one or more contexts."""

    def __init__(self, name, grad_req='write', shape=None, dtype=np.float32, lr_mult=1.0, wd_mult=1.0,
                 init=None, allow_deferred_init=False, differentiable=True, stype='default',
                 grad_stype='default'):
        self._var = None
        self._data = None
        self._grad = None
        self._ctx_list = None
        self._ctx_map = None
        self._trainer = None
        self._deferred_init = ()
        self._differentiable = differentiable
        self._allow_deferred_init = allow_deferred_init
        self._grad_req = None
        if isinstance(shape, int):
            shape = (shape,)
        self._shape = shape
        self.name = name
        self._dtype = dtype
        self.lr_mult = lr_mult
        self.wd_mult = wd_mult
        self.grad_req = grad_req
        self.init = init
        valid = ('default', 'row_sparse', 'csr')
        assert stype in valid, "Invalid stype '%s' for Parameter '%s', expected one of %s" % (stype, name, valid)
        assert grad_stype in valid, \
            "Invalid grad_stype '%s' for Parameter '%s', expected one of %s" % (grad_stype, name, valid)
        self._stype = stype
        self._grad_stype = grad_stype

    def __repr__(self):
        s = 'Parameter {name} (shape={shape}, dtype={dtype})'
        return s.format(name=self.name, shape=self.shape, dtype=self.dtype)

    @property
    def grad_req(self):
        return self._grad_req

    @grad_req.setter
    def grad_req(self, req):
        assert req in ['write', 'add', 'null'], \
            "grad_req must be one of 'write', 'add', or 'null', but got '%s'" % req
        if not self._differentiable:
            req = 'null'
        if self._grad_req == req:
            return
        self._grad_req = req
        if req == 'null' and self._grad is not None:
            self._grad = None
            if self._data is not None:
                for d in self._data:
                    d.attach_grad('null')
        elif self._data is not None:
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
        if self._shape is None:
            self._shape = tuple(new_shape)
            return
        assert len(self._shape) == len(new_shape) and \
            all(j in (0, -1, i) for i, j in zip(new_shape, self._shape)), \
            "Expected shape %s is incompatible with given shape %s." % (str(new_shape), str(self._shape))
        self._shape = tuple(new_shape)

    def _set_trainer(self, trainer):
        """Attach the Trainer that updates this parameter (a sparse parameter allows only one)."""
        if self._stype != 'default' and getattr(self, '_trainer', None) is not None and trainer is not None \
                and self._trainer is not trainer:
            raise RuntimeError("Failed to set the trainer for Parameter '%s' because it was already set. More "
                               "than one trainers for a %s Parameter is not supported." % (self.name, self._stype))
        self._trainer = trainer

    @property
    def stype(self):
        return self._stype

    @property
    def grad_stype(self):
        return self._grad_stype

    # ------------------------------------------------------------------ data
    def _check_and_get(self, arr_list, ctx):
        if arr_list is not None and _state.STATE.np_array:
            _to_np_class(arr_list)
        if arr_list is not None:
            if ctx is list:
                return arr_list
            if ctx is None:
                if len(arr_list) == 1:
                    return arr_list[0]
                ctx = current_context()
            ctx_list = self._ctx_map[ctx.device_typeid & 1]
            if ctx.device_id < len(ctx_list):
                idx = ctx_list[ctx.device_id]
                if idx is not None:
                    return arr_list[idx]
            raise RuntimeError("Parameter '%s' was not initialized on context %s. It was only initialized on %s."
                               % (self.name, str(ctx), str(self._ctx_list)))
        if self._deferred_init:
            raise DeferredInitializationError(
                "Parameter '%s' has not been initialized yet because initialization was deferred. Actual "
                "initialization happens during the first forward pass. Please pass one batch of data through "
                "the network before accessing Parameters." % self.name)
        raise RuntimeError("Parameter '%s' has not been initialized. Note that you should initialize "
                           "parameters and create Trainer with Block.collect_params() instead of Block.params "
                           "because the later does not include Parameters of nested child Blocks" % self.name)

    def _load_init(self, data, ctx, cast_dtype=False, dtype_source='current'):
        if cast_dtype:
            assert dtype_source in ['current', 'saved']
        if self.shape:
            unknown_dim_size = -1 if self.shape and -1 in self.shape else 0
            for self_dim, data_dim in zip(self.shape, data.shape):
                assert self_dim in (unknown_dim_size, data_dim), \
                    "Failed loading Parameter '%s' from saved params: shape incompatible expected %s vs saved %s" % (
                        self.name, str(self.shape), str(data.shape))
            self.shape = tuple(i if i != unknown_dim_size else j for i, j in zip(self.shape, data.shape))
        if self.dtype:
            if cast_dtype and dtype_name(self.dtype) != dtype_name(data.dtype):
                if dtype_source == 'current':
                    data = data.astype(self.dtype, copy=False)
                elif dtype_source == 'saved':
                    self._dtype = data.dtype
            else:
                assert dtype_name(self.dtype) == dtype_name(data.dtype), \
                    "Failed loading Parameter '%s' from saved params: dtype incompatible expected %s vs saved %s. " \
                    "Set cast_dtype=True to cast the dtype of saved params." % (
                        self.name, str(self.dtype), str(data.dtype))
        if isinstance(ctx, Context):
            ctx = [ctx]
        if self._data is None:
            if self._deferred_init:
                assert ctx is None or set(ctx) == set(self._deferred_init[1]), \
                    "Failed to load Parameter '%s' on %s because it was previous initialized on %s." % (
                        self.name, str(ctx), str(self.list_ctx()))
                ctx = self._deferred_init[1]
            elif ctx is None:
                ctx = [cpu()]
            self._init_impl(data, ctx)
        else:
            assert ctx is None or set(ctx) == set(self.list_ctx()), \
                "Failed to load Parameter '%s' on %s because it was previous initialized on %s." % (
                    self.name, str(ctx), str(self.list_ctx()))
            self.set_data(data)
        self._deferred_init = ()
        # weights held by the kvstore are stale now: the trainer re-initialises its store
        tr = getattr(self, '_trainer', None)
        if tr is not None and getattr(tr, '_kv_initialized', False) and getattr(tr, '_update_on_kvstore', False) \
                and self not in tr._params_to_init:
            tr._reset_kvstore()

    def _finish_deferred_init(self):
        if not self._deferred_init:
            return
        init, ctx, default_init, data = self._deferred_init
        self._deferred_init = ()
        assert _shape_known(self.shape), \
            "Cannot initialize Parameter '%s' because it has invalid shape: %s. Please specify in_units, " \
            "in_channels, etc for `Block`s." % (self.name, str(self.shape))
        with autograd.pause():
            if data is None:
                data = nd.zeros(self.shape, dtype=self.dtype, ctx=cpu())
                initializer.create(default_init)(
                    initializer.InitDesc(self.name, {'__init__': init}), data)
            self._init_impl(data, ctx)

    def _init_impl(self, data, ctx_list):
        self._ctx_list = list(ctx_list)
        self._ctx_map = [[], []]
        for i, ctx in enumerate(self._ctx_list):
            dev_list = self._ctx_map[ctx.device_typeid & 1]
            while len(dev_list) <= ctx.device_id:
                dev_list.append(None)
            dev_list[ctx.device_id] = i
        td = torch_dtype(self.dtype)
        self._data = [NDArray(data._data.detach().to(device=c.torch_device, dtype=td, copy=True))
                      for c in self._ctx_list]
        self._init_grad()

    def _init_grad(self):
        if self.grad_req == 'null':
            self._grad = None
            return
        for d in self._data:
            d.attach_grad(self.grad_req, stype=None if self._grad_stype == 'default' else self._grad_stype)
        self._grad = [d._grad for d in self._data]
        if self._trainer is not None and hasattr(self._trainer, '_on_param_grad_reset'):
            self._trainer._on_param_grad_reset(self)

    def _reduce(self):
        ctx = cpu()
        if self._stype == 'default':
            block = self._all_data()
            if len(block) > 1:
                data = nd.add_n(*[w.copyto(ctx) for w in block]) / len(block)
            else:
                data = self.data().copyto(ctx)
        else:
            data = self.row_sparse_data(nd.arange(self.shape[0], ctx=ctx))
        return data

    def initialize(self, init=None, ctx=None, default_init=initializer.Uniform(), force_reinit=False):
        if self._data is not None and not force_reinit:
            warnings.warn("Parameter '%s' is already initialized, ignoring. Set force_reinit=True to "
                          "re-initialize." % self.name, stacklevel=2)
            return
        self._data = self._grad = None
        if ctx is None:
            ctx = [current_context()]
        if isinstance(ctx, Context):
            ctx = [ctx]
        if init is None:
            init = default_init if self.init is None else self.init
        if not _shape_known(self.shape):
            if self._allow_deferred_init:
                self._deferred_init = (init, ctx, default_init, None)
                return
            raise ValueError("Cannot initialize Parameter '%s' because it has invalid shape: %s." %
                             (self.name, str(self.shape)))
        self._deferred_init = (init, ctx, default_init, None)
        self._finish_deferred_init()

    def reset_ctx(self, ctx):
        if ctx is None:
            ctx = [current_context()]
        if isinstance(ctx, Context):
            ctx = [ctx]
        if self._data:
            data = self._reduce()
            with autograd.pause():
                self._init_impl(data, ctx)
        elif self._deferred_init:
            init, _, default_init, data = self._deferred_init
            self._deferred_init = (init, ctx, default_init, data)
        else:
            raise ValueError("Cannot reset context for Parameter '%s' because it has not been initialized."
                             % self.name)

    def set_data(self, data):
        self.shape = data.shape
        if self._data is None:
            assert self._deferred_init, "Parameter '%s' has not been initialized" % self.name
            self._deferred_init = self._deferred_init[:3] + (data,)
            return
        src = data._data if isinstance(data, NDArray) else torch.as_tensor(np.asarray(data))
        with torch.no_grad():
            for arr in self._check_and_get(self._data, list):
                arr._data.copy_(src.to(arr._data.device, arr._data.dtype))

    def _get_row_sparse(self, ctx, row_id):
        if not isinstance(row_id, NDArray):
            raise TypeError('row_id must have NDArray type, but %s is given' % type(row_id))
        if self._trainer is None:
            raise RuntimeError("Cannot get row_sparse data for Parameter '%s' when no Trainer is created with "
                               "it." % self.name)
        results = self._check_and_get(self._data, ctx)
        # only the requested rows are fetched from the kvstore into the local copies
        self._trainer._row_sparse_pull(self, results, row_id)
        return results

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
        return self._check_and_get(self._data, list)

    def grad(self, ctx=None):
        if self._data is not None and self._grad is None:
            raise RuntimeError("Cannot get gradient array for Parameter '%s' because grad_req='null'" % self.name)
        return self._check_and_get(self._grad, ctx)

    def list_grad(self):
        if self._data is not None and self._grad is None:
            raise RuntimeError("Cannot get gradient array for Parameter '%s' because grad_req='null'" % self.name)
        return self._check_and_get(self._grad, list)

    def list_ctx(self):
        if self._data is None:
            if self._deferred_init:
                return self._deferred_init[1]
            raise RuntimeError("Parameter '%s' has not been initialized" % self.name)
        return self._ctx_list

    def zero_grad(self):
        if self._grad is None:
            return
        with torch.no_grad():
            torch._foreach_zero_([g._data for g in self._grad])

    def var(self):
        from .. import symbol
        if self._var is None:
            self._var = symbol.var(self.name, shape=self.shape, dtype=self.dtype, lr_mult=self.lr_mult,
                                   wd_mult=self.wd_mult, init=self.init, stype=self._stype)
        return self._var

    def cast(self, dtype):
        self._dtype = dtype
        if self._data is None:
            return
        td = torch_dtype(dtype)
        with autograd.pause():
            for d in self._data:
                d._data = d._data.detach().to(td)
            self._init_grad()


class Constant(Parameter):
    """A constant parameter (grad_req='null') initialised with ``value``."""

    def __init__(self, name, value):
        if not isinstance(value, NDArray):
            value = nd.array(value)
        self.value = value

        class Init(initializer.Initializer):
            def _init_weight(self, _, arr):
                initializer.Initializer._set(arr, value._data)
        init_name = 'Constant_{}_{}'.format(name, id(self))
        initializer._INIT_REGISTRY[init_name.lower()] = Init
        super().__init__(name, grad_req='null', shape=value.shape, dtype=value.dtype, init=init_name)

    def __repr__(self):
        return 'Constant {name} (shape={shape}, dtype={dtype})'.format(name=self.name, shape=self.shape,
                                                                        dtype=self.dtype)

    @property
    def grad_req(self):
        return 'null'

    @grad_req.setter
    def grad_req(self, req):
        if req != 'null':
            warnings.warn('Constant parameter "{}" does not support grad_req other than "null", and new value '
                          '"{}" is ignored.'.format(self.name, req))
        self._grad_req = 'null'


class ParameterDict:
    """An ordered dictionary of Parameters with a shared name prefix."""

    def __init__(self, prefix='', shared=None):
        self._prefix = prefix
        self._params = OrderedDict()
        self._shared = shared

    def __repr__(self):
        s = '{name}(\n{content}\n)'
        name = self._prefix + ' ' if self._prefix else ''
        return s.format(name=name, content='\n'.join(['  ' + repr(v) for v in self.values()]))

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

    def _get_impl(self, name):
        if name in self._params:
            return self._params[name]
        if self._shared is not None and name in self._shared._params:
            self._params[name] = self._shared._params[name]
            return self._shared._params[name]
        return None

    def get(self, name, **kwargs):
        name = self.prefix + name
        param = self._get_impl(name)
        if param is None:
            param = Parameter(name, **kwargs)
            self._params[name] = param
        else:
            for k, v in kwargs.items():
                if hasattr(param, k) and getattr(param, k) is not None:
                    existing = getattr(param, k)
                    if k == 'shape' and len(v) == len(existing):
                        inferred_shape = []
                        matched = True
                        for dim1, dim2 in zip(v, existing):
                            if dim1 != dim2 and dim1 > 0 and dim2 > 0:
                                matched = False
                                break
                            elif dim1 == dim2:
                                inferred_shape.append(dim1)
                            elif dim1 in (0, -1):
                                inferred_shape.append(dim2)
                            else:
                                inferred_shape.append(dim1)
                        if matched:
                            param._shape = tuple(inferred_shape)
                            continue
                    elif k == 'dtype' and np.dtype(v) == np.dtype(existing):
                        continue
                    assert v is None or v == existing, \
                        "Cannot retrieve Parameter '%s' because desired attribute does not match with stored for " \
                        "attribute '%s': desired '%s' vs stored '%s'." % (name, k, str(v), str(getattr(param, k)))
                else:
                    setattr(param, k, v)
        return param

    def get_constant(self, name, value=None):
        name = self.prefix + name
        param = self._get_impl(name)
        if param is None:
            if value is None:
                raise KeyError("No constant named '{}'. Please specify value if you want to create a new "
                               "constant.".format(name))
            param = Constant(name, value)
            self._params[name] = param
        elif value is not None:
            assert isinstance(param, Constant), \
                "Parameter '{}' already exists but it is not a constant.".format(name)
        return param

    def update(self, other):
        for k, v in other.items():
            if k in self._params:
                assert self._params[k] is v, \
                    "Cannot update self with other because they have different Parameters with the same name '%s'" % k
        for k, v in other.items():
            self._params[k] = v

    def initialize(self, init=initializer.Uniform(), ctx=None, verbose=False, force_reinit=False):
        if verbose:
            init.set_verbosity(verbose=verbose)
        for _, v in self.items():
            v.initialize(None, ctx, init, force_reinit=force_reinit)

    def zero_grad(self):
        grads = []
        for p in self.values():
            if p._grad is not None:
                grads.extend(g._data for g in p._grad)
        if grads:
            with torch.no_grad():
                torch._foreach_zero_(grads)

    def reset_ctx(self, ctx):
        for i in self.values():
            i.reset_ctx(ctx)

    def list_ctx(self):
        s = set()
        for i in self.values():
            s.update(i.list_ctx())
        return list(s)

    def setattr(self, name, value):
        for i in self.values():
            setattr(i, name, value)

    def save(self, filename, strip_prefix=''):
        arg_dict = {}
        for param in self.values():
            weight = param._reduce()
            if not param.name.startswith(strip_prefix):
                raise ValueError("Prefix '%s' is to be striped before saving, but Parameter's name '%s' does not "
                                 "start with '%s'." % (strip_prefix, param.name, strip_prefix))
            arg_dict[param.name[len(strip_prefix):]] = weight
        nd.save(filename, arg_dict)

    def load(self, filename, ctx=None, allow_missing=False, ignore_extra=False, restore_prefix='',
             cast_dtype=False, dtype_source='current'):
        if restore_prefix:
            for name in self.keys():
                assert name.startswith(restore_prefix), \
                    "restore_prefix is '%s' but Parameters name '%s' does not start with '%s'" % (
                        restore_prefix, name, restore_prefix)
        ndarray_load = nd.load(filename) if isinstance(filename, str) else filename
        self.load_dict(ndarray_load, ctx, allow_missing, ignore_extra, restore_prefix, filename,
                       cast_dtype, dtype_source)

    def load_dict(self, param_dict, ctx=None, allow_missing=False, ignore_extra=False, restore_prefix='',
                  filename=None, cast_dtype=False, dtype_source='current'):
        lprefix = len(restore_prefix)
        loaded = [(k[4:] if k.startswith('arg:') or k.startswith('aux:') else k, v) for k, v in param_dict.items()] \
            if isinstance(param_dict, dict) else param_dict
        arg_dict = {restore_prefix + k: v for k, v in loaded}
        error_str = "file: %s" % (filename) if filename else "param_dict"
        if not allow_missing:
            for name in self.keys():
                assert name in arg_dict, \
                    "Parameter '%s' is missing in %s, which contains parameters: %s. Please make sure source and " \
                    "target networks have the same prefix." % (name[lprefix:], error_str, str(list(arg_dict)[:10]))
        for name in arg_dict:
            if name not in self._params:
                assert ignore_extra, \
                    "Parameter '%s' loaded from %s is not present in ParameterDict, choices are: %s. Set " \
                    "ignore_extra to True to ignore. Please make sure source and target networks have the same " \
                    "prefix." % (name[lprefix:], error_str, str(list(self._params)[:10]))
                continue
            self[name]._load_init(arg_dict[name], ctx, cast_dtype=cast_dtype, dtype_source=dtype_source)
