"""User-defined operators in Python (parity: python/mxnet/operator.py, src/operator/custom/custom.cc).

::

    class Sigmoid(mx.operator.CustomOp):
        def forward(self, is_train, req, in_data, out_data, aux):
            self.assign(out_data[0], req[0], 1 / (1 + mx.nd.exp(-in_data[0])))
        def backward(self, req, out_grad, in_data, out_data, in_grad, aux):
            y = out_data[0]
            self.assign(in_grad[0], req[0], out_grad[0] * y * (1 - y))

    @mx.operator.register('sigmoid')
    class SigmoidProp(mx.operator.CustomOpProp):
        def create_operator(self, ctx, shapes, dtypes):
            return Sigmoid()

    y = mx.nd.Custom(x, op_type='sigmoid')      # or mx.sym.Custom(...)

The ``Custom`` operator is registered like any other op, so it works
imperatively (with autograd), symbolically (infer_shape via the prop's
``infer_shape``) and inside hybridized blocks.
"""
import collections
import warnings
import ctypes  # noqa: F401  (part of the reference module's star-import surface)
import torch

from . import _state
from . import profiler as _profiler
from .base import MXNetError, NDArrayHandle  # noqa: F401
from .ndarray.ndarray import NDArray  # noqa: F401
from .ops import registry

__all__ = ['CustomOp', 'CustomOpProp', 'register', 'get_all_registered_operators', 'get_operator_arguments',
           'OperatorArguments', 'ctypes', 'NDArrayHandle', 'NDArray', 'NDArrayOp', 'NumpyOp',
           'PythonOp']

_REGISTRY = {}


class CustomOp:
    """Base class for the computation of a custom operator."""

    def forward(self, is_train, req, in_data, out_data, aux):
        raise NotImplementedError

    def backward(self, req, out_grad, in_data, out_data, in_grad, aux):
        raise NotImplementedError

    def assign(self, dst, req, src):
        """Write ``src`` into ``dst`` according to ``req`` (null / write / inplace / add)."""
        if req == 'null':
            return
        if req in ('write', 'inplace'):
            dst[:] = src
        elif req == 'add':
            dst[:] = dst + src


class CustomOpProp:
    """Describes a custom operator: arguments, outputs, shape/type inference and the op factory."""

    def __init__(self, need_top_grad=True):
        self.need_top_grad_ = need_top_grad

    def infer_shape(self, in_shape):
        return in_shape, (in_shape[0],) * len(self.list_outputs()), ()

    def infer_type(self, in_type):
        return in_type, [in_type[0]] * len(self.list_outputs()), [in_type[0]] * len(self.list_auxiliary_states())

    def infer_storage_type(self, in_stype):
        return in_stype, ['default'] * len(self.list_outputs()), ['default'] * len(self.list_auxiliary_states())

    def infer_storage_type_backward(self, ograd_stype, in_stype, out_stype, igrad_stype, aux_stype):
        return (ograd_stype, in_stype, out_stype, ['default'] * len(igrad_stype),
                ['default'] * len(aux_stype))

    def list_outputs(self):
        return ['output']

    def list_arguments(self):
        return ['data']

    def list_auxiliary_states(self):
        return []

    def declare_backward_dependency(self, out_grad, in_data, out_data):
        deps = []
        if self.need_top_grad_:
            deps.extend(out_grad)
        deps.extend(in_data)
        deps.extend(out_data)
        return deps

    def create_operator(self, ctx, in_shapes, in_dtypes):
        return CustomOp()


def register(reg_name):
    """Class decorator registering a CustomOpProp subclass under ``reg_name``."""
    def do_register(prop_cls):
        _REGISTRY[reg_name] = prop_cls
        return prop_cls
    return do_register


def get_all_registered_operators():
    """Names of every registered operator (built-in and Custom)."""
    from .ops import registry as _ops_registry, load_all
    load_all()
    return sorted(set(_ops_registry.list_ops()) | set(_REGISTRY))


OperatorArguments = collections.namedtuple('OperatorArguments', ['narg', 'names', 'types'])


def _type_doc(spec):
    kind, default = spec[0], spec[1]
    if kind == 'str' and isinstance(default, str) and default.startswith('{'):
        return default
    return '%s, %s' % (kind.rstrip('?'), 'optional, default=%r' % (default,) if default is not None
                       else 'required')


def get_operator_arguments(op_name):
    """OperatorArguments(narg, names, types) of a registered operator: its array inputs
    ('NDArray-or-Symbol') followed by its parameters."""
    from .ops import registry as _ops_registry, load_all
    load_all()
    op = _ops_registry.get(op_name)
    names = list(op.get_arg_names({}) if not callable(op.arg_names) else op.get_arg_names({}))
    types = ['NDArray-or-Symbol'] * len(names)
    enums = _ENUM_DOCS.get(op.name, {})
    for k, spec in op.params.items():
        names.append(k)
        types.append(enums.get(k) or _type_doc(spec))
    return OperatorArguments(len(names), names, types)


# documented choices of enumerated parameters (the reference's dmlc enum type strings)
_ENUM_DOCS = {'Activation': {'act_type': "{'relu', 'sigmoid', 'softrelu', 'softsign', 'tanh'}, required"}}


def _make_prop(attrs):
    op_type = attrs.get('op_type')
    if op_type not in _REGISTRY:
        raise MXNetError('Custom operator %s is not registered' % op_type)
    kw = {k: (v if isinstance(v, str) else str(v)) for k, v in attrs.items() if k != 'op_type'
          and not (k.startswith('__') and k.endswith('__'))}
    prop = _REGISTRY[op_type](**kw)
    prop._op_type_name = op_type
    return prop


def _custom_args(attrs):
    return _make_prop(attrs).list_arguments()


def _custom_aux(attrs):
    return _make_prop(attrs).list_auxiliary_states()


def _custom_nout(attrs):
    return len(_make_prop(attrs).list_outputs())


def _custom_infer(in_shapes, attrs):
    prop = _make_prop(attrs)
    if any(s is None for s in in_shapes[:1]):
        return {}
    n_args = len(prop.list_arguments())
    shapes = [list(s) if s is not None else None for s in in_shapes[:n_args]]
    try:
        ins, _, auxs = _infer3(prop, shapes)
    except Exception:
        return {}
    res = {i: tuple(s) for i, s in enumerate(ins) if s is not None}
    res.update({n_args + i: tuple(s) for i, s in enumerate(auxs)})
    return res


def _infer3(prop, shapes):
    """prop.infer_shape -> (in, out, aux); the aux list may be omitted by user props."""
    res = prop.infer_shape(shapes)
    if len(res) == 2:
        return res[0], res[1], []
    return res


def _out_types(prop, in_types, n_out):
    """Output dtypes from prop.infer_type when it is overridden, else the first input's dtype."""
    from .base import torch_dtype
    if type(prop).infer_type is not CustomOpProp.infer_type:
        import numpy as _np
        res = prop.infer_type([_np.dtype(str(t).replace('torch.', '')) for t in in_types])
        outs = res[1] if len(res) > 1 else []
        if len(outs) == n_out:
            return [torch_dtype(_np.dtype(t).name) for t in outs]
    return [in_types[0] if in_types else torch.float32] * n_out


class _CustomFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, op, prop, n_in, is_train, *tensors):
        from .ndarray.ndarray import NDArray
        ins = [NDArray(t.detach()) for t in tensors[:n_in]]
        aux = [NDArray(t) for t in tensors[n_in:]]
        in_shapes = [list(t.shape) for t in tensors[:n_in]]
        _, out_shapes, _ = _infer3(prop, in_shapes)
        out_types = _out_types(prop, [t.dtype for t in tensors[:n_in]], len(out_shapes))
        dev = tensors[0].device if tensors else torch.device('cpu')
        outs = [NDArray(torch.zeros(tuple(s), dtype=dt, device=dev)) for s, dt in zip(out_shapes, out_types)]
        with torch.no_grad(), _profiler.custom_op_scope(prop._op_type_name):
            op.forward(is_train=is_train, req=['write'] * len(outs), in_data=ins, out_data=outs, aux=aux)
        for o in outs:
            box = getattr(o, '_exc', None)
            if box is not None and box[0] is not None:
                from . import engine
                engine.rethrow(box)       # an operator inside the body failed
        ctx.op, ctx.n_in, ctx.op_type = op, n_in, prop._op_type_name
        ctx.save_for_backward(*tensors)
        ctx.outs = [o._data for o in outs]
        return tuple(o._data for o in outs)

    @staticmethod
    def backward(ctx, *grads):
        from .ndarray.ndarray import NDArray
        tensors = ctx.saved_tensors
        n_in = ctx.n_in
        ins = [NDArray(t) for t in tensors[:n_in]]
        aux = [NDArray(t) for t in tensors[n_in:]]
        outs = [NDArray(t) for t in ctx.outs]
        ograds = [NDArray(g if g is not None else torch.zeros_like(o)) for g, o in zip(grads, ctx.outs)]
        igrads = [NDArray(torch.zeros_like(t)) for t in tensors[:n_in]]
        with torch.no_grad(), _profiler.custom_op_scope(ctx.op_type, backward=True):
            ctx.op.backward(req=['write'] * n_in, out_grad=ograds, in_data=ins, out_data=outs, in_grad=igrads,
                            aux=aux)
        return (None, None, None, None) + tuple(g._data for g in igrads) + (None,) * (len(tensors) - n_in)


_OP_CACHE = {}


def _custom_fn(*inputs, op_type=None, **kwargs):
    attrs = dict(kwargs, op_type=op_type)
    prop = _make_prop(attrs)
    n_in = len(prop.list_arguments())
    tensors = [t for t in inputs if t is not None]
    if tensors and tensors[0].device.type == 'meta':
        _, out_shapes, _ = _infer3(prop, [list(t.shape) for t in tensors[:n_in]])
        outs = [torch.empty(tuple(s), dtype=tensors[0].dtype, device='meta') for s in out_shapes]
        return outs[0] if len(outs) == 1 else tuple(outs)
    from .context import context_from_torch
    dev = tensors[0].device if tensors else torch.device('cpu')
    key = (op_type, tuple(sorted((k, str(v)) for k, v in kwargs.items())),
           tuple(tuple(t.shape) for t in tensors), tuple(str(t.dtype) for t in tensors), str(dev))
    op = _OP_CACHE.get(key)
    if op is None:
        op = prop.create_operator(context_from_torch(dev), [list(t.shape) for t in tensors[:n_in]],
                                  [t.dtype for t in tensors[:n_in]])
        _OP_CACHE[key] = op
    try:
        outs = _CustomFunction.apply(op, prop, n_in, bool(_state.STATE.training), *tensors)
    except MXNetError:
        raise
    except Exception as e:      # pylint: disable=broad-except
        # an exception in the Python body surfaces as MXNetError, like the reference's custom op worker
        raise MXNetError('Error in CustomOp %s: %s: %s' % (op_type, type(e).__name__, e)) from e
    return outs[0] if len(outs) == 1 else tuple(outs)


registry.register('Custom', _custom_fn, arg_names=_custom_args, aux_names=_custom_aux, num_outputs=_custom_nout,
                  infer_params=_custom_infer, params={'op_type': ('str', None)}, extra_params=True)


# ---------------------------------------------------------------------------
# deprecated numpy/ndarray op front-ends of the reference (NumpyOp / NDArrayOp):
# kept as thin CustomOp adapters so old code keeps running.
# ---------------------------------------------------------------------------

class PythonOp:
    """Deprecated operator front-end (reference python/mxnet/operator.py:51-152). ``get_symbol``
    registers a private CustomOpProp that forwards shape inference and forward/backward to this
    instance, so the op runs through the same Custom-op path as :class:`CustomOp`."""

    _array_kind = 'ndarray'
    _count = 0

    def __init__(self, need_top_grad=True):
        self.info_ = None
        self.need_top_grad_ = need_top_grad
        warnings.warn('PythonOp has been deprecated. Please use CustomOp')

    def __call__(self, *args, **kwargs):
        return self.get_symbol(*args, **kwargs)

    def get_symbol(self, *args, **kwargs):
        """Symbol applying this operator to ``args`` (call once per stateful instance)."""
        if self.info_ is None:
            PythonOp._count += 1
            self.info_ = '_pythonop_%s_%d' % (type(self).__name__, PythonOp._count)
            register(self.info_)(_python_op_prop(self))
        from . import symbol as _sym
        return _sym.Custom(*args, op_type=self.info_, **kwargs)

    def forward(self, in_data, out_data):
        out_data[0][:] = in_data[0]

    def backward(self, out_grad, in_data, out_data, in_grad):
        in_grad[0][:] = 1.0

    def list_outputs(self):
        return ['output']

    def list_arguments(self):
        return ['data']

    def infer_shape(self, in_shape):
        return in_shape, [in_shape[0]]

    def need_top_grad(self):
        return self.need_top_grad_


class NDArrayOp(PythonOp):
    """PythonOp whose forward/backward receive NDArrays (reference operator.py:255-362)."""

    def __init__(self, need_top_grad=True):
        super().__init__(need_top_grad)
        warnings.warn('NDArrayOp has been deprecated. Please use CustomOp')

    def declare_backward_dependency(self, out_grad, in_data, out_data):
        deps = []
        if self.need_top_grad():
            deps.extend(out_grad)
        deps.extend(in_data)
        deps.extend(out_data)
        return deps


class NumpyOp(PythonOp):
    """PythonOp whose forward/backward receive numpy arrays, written back after the call
    (reference operator.py:155-252)."""

    _array_kind = 'numpy'

    def __init__(self, need_top_grad=True):
        super().__init__(need_top_grad)
        warnings.warn('NumpyOp has been deprecated. Please use CustomOp')


def _python_op_prop(pyop):
    """CustomOpProp class bound to one PythonOp instance."""
    as_numpy = pyop._array_kind == 'numpy'

    def _call(fn, groups, written):
        if not as_numpy:
            fn(*groups)
            return
        host = [[a.asnumpy() for a in g] for g in groups]
        fn(*host)
        for gi in written:
            for dst, src in zip(groups[gi], host[gi]):
                dst[:] = src

    class _Op(CustomOp):
        def forward(self, is_train, req, in_data, out_data, aux):
            _call(pyop.forward, [in_data, out_data], written=(1,))

        def backward(self, req, out_grad, in_data, out_data, in_grad, aux):
            _call(pyop.backward, [out_grad, in_data, out_data, in_grad], written=(3,))

    class _Prop(CustomOpProp):
        def __init__(self):
            super().__init__(need_top_grad=pyop.need_top_grad())

        def list_arguments(self):
            return pyop.list_arguments()

        def list_outputs(self):
            return pyop.list_outputs()

        def infer_shape(self, in_shape):
            ins, outs = pyop.infer_shape(in_shape)[:2]
            return ins, outs, []

        def create_operator(self, ctx, in_shapes, in_dtypes):
            return _Op()

    return _Prop
