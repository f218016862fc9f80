"""NumPy-semantics operators (``_npi_*`` / ``_np_*``) behind ``mx.np`` / ``mx.npx``.

Parity: src/operator/numpy/** (np_elemwise_broadcast_op*, np_broadcast_reduce_op*,
np_matrix_op*, np_init_op*, np_dot*, np_einsum_op*, linalg/np_*, random/np_*)
and python/mxnet/numpy/multiarray.py.  Every op is an ordinary registry entry, so
the same definition serves imperative ``mx.np.*`` calls, ``mx.sym.np.*``
graph construction (hybridized blocks) and meta-tensor shape inference.

Semantics follow MXNet's NumPy interface: float32 is the default floating
type (``np.array([1, 2])`` and ``np.arange(3)`` are float32), integer true
division promotes to float32, comparisons return ``bool``.
"""
import math

import numpy as onp
import torch

from ..base import MXNetError, torch_dtype
from .registry import register

_FLOAT = torch.float32


def _td(dtype, default=None):
    if dtype is None:
        return default
    return torch_dtype(dtype)


def _dev(ctx):
    from .tensor import _dev as d
    return d(ctx)


def _axes(axis, ndim):
    if axis is None:
        return tuple(range(ndim))
    if isinstance(axis, int):
        axis = (axis,)
    return tuple(a % max(ndim, 1) for a in axis)


def _fl(x):
    """Promote integer/bool input to the default float type (numpy's float ufunc rule, float32 default)."""
    return x if x.is_floating_point() or x.is_complex() else x.to(_FLOAT)


# ---------------------------------------------------------------------------
# elementwise unary
# ---------------------------------------------------------------------------

def _rint(x):
    return torch.round(x)


def _fix(x):
    return torch.trunc(_fl(x))


_UNARY = {
    'negative': torch.neg, 'absolute': torch.abs, 'abs': torch.abs, 'fabs': lambda x: torch.abs(_fl(x)),
    'sign': torch.sign, 'rint': lambda x: torch.round(_fl(x)), 'ceil': lambda x: torch.ceil(_fl(x)),
    'floor': lambda x: torch.floor(_fl(x)), 'trunc': lambda x: torch.trunc(_fl(x)), 'fix': _fix,
    'square': torch.square, 'sqrt': lambda x: torch.sqrt(_fl(x)), 'cbrt': lambda x: torch.sign(_fl(x)) *
    torch.abs(_fl(x)).pow(1.0 / 3), 'exp': lambda x: torch.exp(_fl(x)), 'expm1': lambda x: torch.expm1(_fl(x)),
    'log': lambda x: torch.log(_fl(x)), 'log2': lambda x: torch.log2(_fl(x)), 'log10': lambda x: torch.log10(_fl(x)),
    'log1p': lambda x: torch.log1p(_fl(x)), 'sin': lambda x: torch.sin(_fl(x)), 'cos': lambda x: torch.cos(_fl(x)),
    'tan': lambda x: torch.tan(_fl(x)), 'arcsin': lambda x: torch.asin(_fl(x)),
    'arccos': lambda x: torch.acos(_fl(x)), 'arctan': lambda x: torch.atan(_fl(x)),
    'sinh': lambda x: torch.sinh(_fl(x)), 'cosh': lambda x: torch.cosh(_fl(x)), 'tanh': lambda x: torch.tanh(_fl(x)),
    'arcsinh': lambda x: torch.asinh(_fl(x)), 'arccosh': lambda x: torch.acosh(_fl(x)),
    'arctanh': lambda x: torch.atanh(_fl(x)), 'degrees': lambda x: torch.rad2deg(_fl(x)),
    'rad2deg': lambda x: torch.rad2deg(_fl(x)), 'radians': lambda x: torch.deg2rad(_fl(x)),
    'deg2rad': lambda x: torch.deg2rad(_fl(x)), 'reciprocal': lambda x: torch.reciprocal(x) if x.is_floating_point()
    else torch.div(1, x, rounding_mode='trunc'),
    'logical_not': torch.logical_not, 'bitwise_not': torch.bitwise_not, 'invert': torch.bitwise_not,
    'isnan': torch.isnan, 'isinf': torch.isinf, 'isfinite': torch.isfinite, 'isposinf': torch.isposinf,
    'isneginf': torch.isneginf, 'signbit': torch.signbit, 'positive': lambda x: x.clone(),
    'sigmoid': lambda x: torch.sigmoid(_fl(x)),
}

for _n, _f in _UNARY.items():
    register('_npi_' + _n, arg_names=('x',))(lambda x, _f=_f: _f(x))


@register('_npi_around', aliases=('_npi_round',), arg_names=('x',), params={'decimals': ('int', 0)})
def _around(x, decimals=0):
    if not x.is_floating_point():
        if decimals >= 0:
            return x.clone()
        f = 10 ** (-decimals)
        return (torch.round(x.double() / f) * f).to(x.dtype)
    return torch.round(x, decimals=decimals)


@register('_npi_nan_to_num', arg_names=('x',), params={'copy': ('bool', True), 'nan': ('float', 0.0),
                                                       'posinf': ('float?', None), 'neginf': ('float?', None)})
def _nan_to_num(x, copy=True, nan=0.0, posinf=None, neginf=None):
    if not x.is_floating_point():
        return x.clone()
    return torch.nan_to_num(x, nan=nan, posinf=posinf, neginf=neginf)


# ---------------------------------------------------------------------------
# elementwise binary (tensor-tensor with broadcasting, tensor-scalar)
# ---------------------------------------------------------------------------

def _fbin(f):
    def g(a, b):
        rt = torch.result_type(a, b)
        if not (rt.is_floating_point or rt.is_complex):
            rt = _FLOAT
        return f(a.to(rt), b.to(rt))
    return g


def _sub(a, b):
    # numpy: a bool operand is promoted to the other's type (bool - bool is a TypeError there too)
    if a.dtype == torch.bool and b.dtype != torch.bool:
        a = a.to(b.dtype)
    elif b.dtype == torch.bool and a.dtype != torch.bool:
        b = b.to(a.dtype)
    return torch.sub(a, b)


def _floor_divide(a, b):
    return torch.floor_divide(a, b)


def _mod(a, b):
    return torch.remainder(a, b)


def _power(a, b):
    return torch.pow(a, b)


def _ldexp(a, b):
    return _fl(a) * torch.pow(2.0, b.to(_fl(a).dtype))


def _heaviside(a, b):
    rt = torch.result_type(a, b)
    return torch.heaviside(a.to(rt), b.to(rt))


def _maxmin(is_max):
    def f(a, b):
        from .tensor import _maximum, _minimum
        if a.dtype != b.dtype:
            rt = torch.promote_types(a.dtype, b.dtype)
            a, b = a.to(rt), b.to(rt)
        return _maximum(a, b) if is_max else _minimum(a, b)
    return f


_BINARY = {
    'add': torch.add, 'subtract': _sub, 'multiply': torch.mul, 'true_divide': torch.true_divide,
    'floor_divide': _floor_divide, 'mod': _mod, 'fmod': torch.fmod, 'power': _power,
    'maximum': _maxmin(True), 'minimum': _maxmin(False), 'fmax': torch.fmax, 'fmin': torch.fmin,
    'arctan2': _fbin(torch.atan2), 'hypot': _fbin(torch.hypot), 'copysign': _fbin(torch.copysign),
    'ldexp': _ldexp, 'lcm': torch.lcm, 'gcd': torch.gcd, 'bitwise_and': torch.bitwise_and,
    'bitwise_or': torch.bitwise_or, 'bitwise_xor': torch.bitwise_xor, 'logical_and': torch.logical_and,
    'logical_or': torch.logical_or, 'logical_xor': torch.logical_xor, 'equal': torch.eq, 'not_equal': torch.ne,
    'greater': torch.gt, 'greater_equal': torch.ge, 'less': torch.lt, 'less_equal': torch.le,
    'float_power': lambda a, b: torch.float_power(a, b).to(torch.float64), 'heaviside': _heaviside,
    'bitwise_left_shift': torch.bitwise_left_shift, 'bitwise_right_shift': torch.bitwise_right_shift,
}
BINARY_NAMES = tuple(_BINARY)


def _scalar_tensor(x, scalar):
    """A 0-d tensor for a python scalar using numpy/MXNet weak-scalar promotion."""
    if isinstance(scalar, bool):
        dt = x.dtype if x.dtype == torch.bool else x.dtype
    elif isinstance(scalar, int):
        dt = x.dtype if x.dtype != torch.bool else torch.int64
    else:
        dt = x.dtype if (x.is_floating_point() or x.is_complex()) else _FLOAT
    return torch.tensor(scalar, dtype=dt, device=x.device)


for _n, _f in _BINARY.items():
    register('_npi_' + _n, arg_names=('x1', 'x2'))(lambda a, b, _f=_f: _f(a, b))

    def _sc(x, scalar=0.0, reverse=False, _f=_f):
        s = _scalar_tensor(x, scalar)
        if s.dtype != x.dtype:
            x = x.to(s.dtype)
        return _f(s, x) if reverse else _f(x, s)
    register('_npi_' + _n + '_scalar', arg_names=('x',), params={'scalar': ('any', 0.0), 'reverse': ('bool', False)})(_sc)


@register('_npi_divide', arg_names=('x1', 'x2'))
def _divide(a, b):
    return torch.true_divide(a, b)


# ---------------------------------------------------------------------------
# reductions
# ---------------------------------------------------------------------------

_RED = {'axis': ('axis', None), 'keepdims': ('bool', False), 'dtype': ('dtype', None)}


def _red_dims(x, axis):
    return list(_axes(axis, x.dim())) if x.dim() else []


@register('_np_sum', aliases=('_npi_sum',), arg_names=('a',), params=dict(_RED, initial=('float?', None)))
def _sum(a, axis=None, keepdims=False, dtype=None, initial=None):
    dt = _td(dtype)
    if dt is None and (a.dtype == torch.bool):
        dt = torch.int64
    d = _red_dims(a, axis)
    if dt is not None and not dt.is_floating_point and a.requires_grad:
        a = a.detach()                      # an integer result carries no gradient
    if d and a.dtype in (torch.float16, torch.bfloat16, torch.float32) and (dt is None or dt.is_floating_point):
        # accumulate one precision up (fp16 -> fp32, fp32 -> fp64: the reference's AccType), then cast
        acc = torch.float64 if a.dtype == torch.float32 else torch.float32
        r = torch.sum(a, dim=d, keepdim=keepdims, dtype=acc).to(dt or a.dtype)
    elif d and dt is not None and dt.is_floating_point and a.is_floating_point() and \
            torch.finfo(a.dtype).bits > torch.finfo(dt).bits:
        r = torch.sum(a, dim=d, keepdim=keepdims).to(dt)    # accumulate in the wider input type
    else:
        r = torch.sum(a, dim=d, keepdim=keepdims, dtype=dt) if d else (a.to(dt) if dt else a.clone())
    return r + initial if initial is not None else r


@register('_np_prod', aliases=('_npi_prod',), arg_names=('a',), params=dict(_RED, initial=('float?', None)))
def _prod(a, axis=None, keepdims=False, dtype=None, initial=None):
    dt = _td(dtype)
    r = a.to(dt) if dt is not None else a
    for d in sorted(_red_dims(a, axis), reverse=True):
        r = torch.prod(r, dim=d, keepdim=keepdims)
    return r * initial if initial is not None else r


@register('_npi_mean', arg_names=('a',), params=_RED)
def _mean(a, axis=None, keepdims=False, dtype=None):
    dt = _td(dtype) or (a.dtype if a.is_floating_point() else _FLOAT)
    d = _red_dims(a, axis)
    acc = dt if dt.is_floating_point else torch.float64     # integer dtype: float mean, then cast
    if a.is_floating_point() and acc.is_floating_point and torch.finfo(a.dtype).bits > torch.finfo(acc).bits:
        acc = a.dtype          # narrowing dtype: reduce (and differentiate) in the input precision
    if not dt.is_floating_point and not a.is_floating_point() and d:
        # integer input and result: numpy sums in the result type (wrapping) and truncates the quotient
        n = 1
        for k in d:
            n *= a.shape[k]
        s_ = torch.sum(a.to(dt), dim=d, keepdim=keepdims, dtype=dt)
        return torch.trunc(s_.to(torch.float64) / max(n, 1)).to(dt)
    r = torch.mean(a.to(acc), dim=d, keepdim=keepdims) if d else a.to(acc).clone()
    return r.to(dt)


def _std_var(fn):
    def f(a, axis=None, keepdims=False, dtype=None, ddof=0):
        dt = _td(dtype) or (a.dtype if a.is_floating_point() else _FLOAT)
        d = _red_dims(a, axis)
        if not d and a.dim():
            # no axes: one element per reduction, so sum((x - mean)^2) = 0 over n - ddof = 1 - ddof
            v = (0 * a.to(dt)) / (1 - ddof) if ddof != 1 else (0 * a.to(dt)) / 0.0
            return torch.sqrt(v) if fn is torch.std else v
        return fn(a.to(dt), dim=d, correction=ddof, keepdim=keepdims)
    return f


register('_npi_std', arg_names=('a',), params=dict(_RED, ddof=('int', 0)))(_std_var(torch.std))
register('_npi_var', arg_names=('a',), params=dict(_RED, ddof=('int', 0)))(_std_var(torch.var))


def _minmax(fn):
    def f(a, axis=None, keepdims=False, initial=None):
        d = _red_dims(a, axis)
        r = fn(a, dim=d, keepdim=keepdims) if d else a.clone()
        return r
    return f


register('_np_max', aliases=('_npi_max', '_npi_amax'), arg_names=('a',),
         params={'axis': ('axis', None), 'keepdims': ('bool', False), 'initial': ('float?', None)})(_minmax(torch.amax))
register('_np_min', aliases=('_npi_min', '_npi_amin'), arg_names=('a',),
         params={'axis': ('axis', None), 'keepdims': ('bool', False), 'initial': ('float?', None)})(_minmax(torch.amin))


@register('_np_all', aliases=('_npi_all',), arg_names=('a',), params={'axis': ('axis', None), 'keepdims': ('bool', False)})
def _all(a, axis=None, keepdims=False):
    r = a.bool()
    for d in sorted(_red_dims(a, axis), reverse=True):
        r = torch.all(r, dim=d, keepdim=keepdims)
    return r


@register('_np_any', aliases=('_npi_any',), arg_names=('a',), params={'axis': ('axis', None), 'keepdims': ('bool', False)})
def _any(a, axis=None, keepdims=False):
    r = a.bool()
    for d in sorted(_red_dims(a, axis), reverse=True):
        r = torch.any(r, dim=d, keepdim=keepdims)
    return r


def _arg(fn):
    def f(a, axis=None, keepdims=False):
        if axis is None:
            r = fn(a.reshape(-1))
            return r.reshape([1] * a.dim()) if keepdims else r
        return fn(a, dim=axis, keepdim=keepdims)
    return f


register('_npi_argmax', arg_names=('a',), params={'axis': ('int?', None), 'keepdims': ('bool', False)})(_arg(torch.argmax))
register('_npi_argmin', arg_names=('a',), params={'axis': ('int?', None), 'keepdims': ('bool', False)})(_arg(torch.argmin))


@register('_np_cumsum', aliases=('_npi_cumsum',), arg_names=('a',), params={'axis': ('int?', None), 'dtype': ('dtype', None)})
def _cumsum(a, axis=None, dtype=None):
    if axis is None:
        a, axis = a.reshape(-1), 0
    dt = _td(dtype) or a.dtype
    if dt in (torch.float16, torch.bfloat16) and 0 < a.shape[axis] <= 4096:
        # the reference's kernel accumulates in the output type (out[i] = out[i-1] + in[i]); torch
        # widens half-precision scans internally, which rounds differently
        x = a.to(dt).movedim(axis, 0)
        outs = [x[0]]
        for i in range(1, x.shape[0]):
            outs.append(outs[-1] + x[i])
        return (torch.stack(outs) if outs else x.clone()).movedim(0, axis)
    return torch.cumsum(a, dim=axis, dtype=_td(dtype))


@register('_npi_cumprod', arg_names=('a',), params={'axis': ('int?', None), 'dtype': ('dtype', None)})
def _cumprod(a, axis=None, dtype=None):
    if axis is None:
        a, axis = a.reshape(-1), 0
    return torch.cumprod(a, dim=axis, dtype=_td(dtype))


@register('_npi_average', arg_names=lambda a: ['a', 'weights'] if a.get('weighted', False) else ['a'],
          num_outputs=lambda a: 2 if a.get('returned', False) else 1,
          params={'axis': ('axis', None), 'returned': ('bool', False), 'weighted': ('bool', False)})
def _average(a, weights=None, axis=None, returned=False, weighted=False):
    a = _fl(a)
    d = _red_dims(a, axis)
    if weights is None:
        avg = a.mean(dim=d) if d else a.clone()
        n = torch.full_like(avg, float(a.numel() // max(avg.numel(), 1)))
    else:
        w = weights.to(a.dtype)
        if w.dim() == 1 and a.dim() > 1 and isinstance(axis, int):
            shape = [1] * a.dim()
            shape[axis % a.dim()] = -1
            w = w.reshape(shape)
        w = w.expand_as(a)
        n = w.sum(dim=d)
        avg = (a * w).sum(dim=d) / n
    return (avg, n) if returned else avg


@register('_npi_quantile', arg_names=('a',), params={'q': ('any', 0.5), 'axis': ('axis', None),
                                                     'interpolation': ('str', 'linear'), 'keepdims': ('bool', False)})
def _quantile(a, q=0.5, axis=None, interpolation='linear', keepdims=False):
    if a.dtype not in (torch.float32, torch.float64):
        # torch.quantile takes float/double only: half and integer inputs go through float64
        out_dt = a.dtype if a.is_floating_point() else _FLOAT
        return _quantile(a.double(), q, axis, interpolation, keepdims).to(out_dt)
    qt = q.to(a.device, a.dtype) if torch.is_tensor(q) else torch.as_tensor(q, dtype=a.dtype, device=a.device)
    x = a
    if axis is None:
        r = torch.quantile(x.reshape(-1), qt, interpolation=interpolation)
        if keepdims:
            r = r.reshape(tuple(qt.shape) + (1,) * a.dim())
        return r
    if isinstance(axis, tuple):
        if len(axis) != 1:
            red = _axes(axis, x.dim())
            keep = [i for i in range(x.dim()) if i not in red]
            full = [1 if i in red else x.shape[i] for i in range(x.dim())]
            x = x.permute(keep + list(red)).reshape([x.shape[i] for i in keep] + [-1])
            r = torch.quantile(x, qt, dim=-1, interpolation=interpolation)
            return r.reshape(tuple(qt.shape) + tuple(full)) if keepdims else r
        axis = axis[0]
    return torch.quantile(x, qt, dim=axis, keepdim=keepdims, interpolation=interpolation)


@register('_npi_percentile', arg_names=('a',), params={'q': ('any', 50.0), 'axis': ('axis', None),
                                                       'interpolation': ('str', 'linear'), 'keepdims': ('bool', False)})
def _percentile(a, q=50.0, axis=None, interpolation='linear', keepdims=False):
    qq = (torch.as_tensor(q, dtype=torch.float64) / 100.0).tolist()
    return _quantile(a, qq, axis, interpolation, keepdims)


@register('_npi_quantile_q', arg_names=('a', 'q'), params={'axis': ('axis', None), 'interpolation': ('str', 'linear'),
                                                          'keepdims': ('bool', False), 'percent': ('bool', False)})
def _quantile_q(a, q, axis=None, interpolation='linear', keepdims=False, percent=False):
    """quantile / percentile with the quantiles as an array input (a graph input when hybridized)."""
    q = q.double() / 100.0 if percent else q.double()
    return _quantile(a, q, axis, interpolation, keepdims)


@register('_npi_median', arg_names=('a',), params={'axis': ('axis', None), 'keepdims': ('bool', False)})
def _median(a, axis=None, keepdims=False):
    return _quantile(a, 0.5, axis, 'linear', keepdims)


# ---------------------------------------------------------------------------
# creation
# ---------------------------------------------------------------------------

_INIT = {'shape': ('shape', ()), 'ctx': ('any', None), 'dtype': ('dtype', 'float32')}


@register('_npi_zeros', arg_names=(), params=_INIT)
def _zeros(shape=(), ctx=None, dtype='float32'):
    return torch.zeros(shape, dtype=_td(dtype, _FLOAT), device=_dev(ctx))


@register('_npi_ones', arg_names=(), params=_INIT)
def _ones(shape=(), ctx=None, dtype='float32'):
    return torch.ones(shape, dtype=_td(dtype, _FLOAT), device=_dev(ctx))


@register('_npi_full', arg_names=(), params=dict(_INIT, value=('any', 0.0)))
def _full(shape=(), ctx=None, dtype='float32', value=0.0):
    return torch.full(shape, value, dtype=_td(dtype, _FLOAT), device=_dev(ctx))


@register('_npi_full_like', arg_names=('a',), params={'fill_value': ('any', 0.0), 'dtype': ('dtype', None),
                                                      'ctx': ('any', None)})
def _full_like(a, fill_value=0.0, dtype=None, ctx=None):
    return torch.full(a.shape, fill_value, dtype=_td(dtype, a.dtype), device=a.device)


@register('_npi_zeros_like', arg_names=('a',), params={'dtype': ('dtype', None)})
def _zeros_like(a, dtype=None):
    return torch.zeros(a.shape, dtype=_td(dtype, a.dtype), device=a.device)


@register('_npi_ones_like', arg_names=('a',), params={'dtype': ('dtype', None)})
def _ones_like(a, dtype=None):
    return torch.ones(a.shape, dtype=_td(dtype, a.dtype), device=a.device)


@register('_npi_arange', arg_names=(), params={'start': ('float', 0.0), 'stop': ('float?', None),
                                              'step': ('float', 1.0), 'ctx': ('any', None), 'dtype': ('dtype', 'float32')})
def _arange(start=0.0, stop=None, step=1.0, ctx=None, dtype='float32'):
    if stop is None:
        start, stop = 0.0, start
    n = max(int(math.ceil((stop - start) / step)), 0)
    r = start + step * torch.arange(n, dtype=torch.float64, device=_dev(ctx))
    return r.to(_td(dtype, _FLOAT))


@register('_npi_linspace', arg_names=(), params={'start': ('float', 0.0), 'stop': ('float', 1.0), 'num': ('int', 50),
                                                'endpoint': ('bool', True), 'ctx': ('any', None),
                                                'dtype': ('dtype', 'float32')})
def _linspace(start=0.0, stop=1.0, num=50, endpoint=True, ctx=None, dtype='float32'):
    if endpoint:
        r = torch.linspace(start, stop, num, dtype=torch.float64)
    else:
        r = start + (stop - start) / max(num, 1) * torch.arange(num, dtype=torch.float64)
    dt = _td(dtype, _FLOAT)
    if not (dt.is_floating_point or dt.is_complex):
        r = torch.floor(r)          # numpy floors integer linspace
    return r.to(dt).to(_dev(ctx))


@register('_npi_logspace', arg_names=(), params={'start': ('float', 0.0), 'stop': ('float', 1.0), 'num': ('int', 50),
                                                'endpoint': ('bool', True), 'base': ('float', 10.0),
                                                'ctx': ('any', None), 'dtype': ('dtype', 'float32')})
def _logspace(start=0.0, stop=1.0, num=50, endpoint=True, base=10.0, ctx=None, dtype='float32'):
    e = _linspace(start, stop, num, endpoint, ctx, 'float64')
    return torch.pow(base, e).to(_td(dtype, _FLOAT))


@register('_npi_eye', aliases=('_npi_identity',), arg_names=(),
          params={'N': ('int', 1), 'M': ('int?', None), 'k': ('int', 0), 'ctx': ('any', None),
                  'dtype': ('dtype', 'float32')})
def _eye(N=1, M=None, k=0, ctx=None, dtype='float32'):
    M = N if M is None else M
    r = torch.ones(N, M, dtype=_td(dtype, _FLOAT), device=_dev(ctx))
    return torch.triu(torch.tril(r, k), k)


@register('_npi_tri', arg_names=(), params={'N': ('int', 1), 'M': ('int?', None), 'k': ('int', 0),
                                           'ctx': ('any', None), 'dtype': ('dtype', 'float32')})
def _tri(N=1, M=None, k=0, ctx=None, dtype='float32'):
    M = N if M is None else M
    return torch.tril(torch.ones(N, M, dtype=_td(dtype, _FLOAT), device=_dev(ctx)), k)


@register('_npi_indices', arg_names=(), params={'dimensions': ('shape', ()), 'ctx': ('any', None),
                                               'dtype': ('dtype', 'int64')})
def _indices(dimensions=(), ctx=None, dtype='int64'):
    g = torch.meshgrid(*[torch.arange(d, device=_dev(ctx)) for d in dimensions], indexing='ij')
    return torch.stack(g).to(_td(dtype, torch.int64))


# ---------------------------------------------------------------------------
# shape manipulation
# ---------------------------------------------------------------------------

@register('_np_reshape', aliases=('_npi_reshape',), arg_names=('a',), params={'newshape': ('any', ()), 'order': ('str', 'C')})
def _reshape(a, newshape=(), order='C'):
    if isinstance(newshape, int):
        newshape = (newshape,)
    if order == 'F':
        return a.permute(*reversed(range(a.dim()))).reshape(tuple(reversed(newshape))).permute(
            *reversed(range(len(newshape))))
    return a.reshape(tuple(newshape))


@register('_np_transpose', aliases=('_npi_transpose',), arg_names=('a',), params={'axes': ('shape?', None)})
def _transpose(a, axes=None):
    if a.dim() == 0:
        return a.clone()
    if not axes:
        axes = tuple(reversed(range(a.dim())))
    if len(axes) != a.dim() or any(not -a.dim() <= x < a.dim() for x in axes):
        from ..base import MXNetError
        raise MXNetError('transpose: axes %s do not match an array of %d dimensions' % (tuple(axes), a.dim()))
    perm = [x % a.dim() for x in axes]
    if len(set(perm)) != len(perm):
        raise ValueError('transpose: repeated axis in %s' % (tuple(axes),))
    return a.permute(*perm)


@register('_npi_swapaxes', aliases=('_np_swapaxes',), arg_names=('a',), params={'axis1': ('int', 0), 'axis2': ('int', 0)})
def _swapaxes(a, axis1=0, axis2=0):
    return a.transpose(axis1, axis2)


@register('_npi_moveaxis', arg_names=('a',), params={'source': ('any', 0), 'destination': ('any', 0)})
def _moveaxis(a, source=0, destination=0):
    return torch.movedim(a, source, destination)


@register('_npi_rollaxis', arg_names=('a',), params={'axis': ('int', 0), 'start': ('int', 0)})
def _rollaxis(a, axis=0, start=0):
    n = a.dim()
    axis %= n
    if start < 0:
        start += n
    if axis < start:
        start -= 1
    return torch.movedim(a, axis, start)


@register('_npi_expand_dims', arg_names=('a',), params={'axis': ('axis', 0)})
def _expand_dims(a, axis=0):
    axes = (axis,) if isinstance(axis, int) else axis
    out_nd = a.dim() + len(axes)
    for ax in sorted(x % out_nd for x in axes):
        a = a.unsqueeze(ax)
    return a


@register('_np_squeeze', aliases=('_npi_squeeze',), arg_names=('a',), params={'axis': ('axis', None)})
def _squeeze(a, axis=None):
    if axis is None:
        return a.squeeze()
    if a.dim() == 0:
        return a.clone()        # numpy accepts axis 0 / -1 on a 0-d array
    for ax in sorted(_axes(axis, a.dim()), reverse=True):
        if a.shape[ax] != 1:
            raise ValueError('cannot select an axis to squeeze out which has size not equal to one')
        a = a.squeeze(ax)
    return a


@register('_npi_flip', arg_names=('a',), params={'axis': ('axis', None)})
def _flip(a, axis=None):
    return torch.flip(a, _axes(axis, a.dim()))


@register('_npi_roll', arg_names=('a',), params={'shift': ('any', 0), 'axis': ('axis', None)})
def _roll(a, shift=0, axis=None):
    if axis is None:
        return torch.roll(a.reshape(-1), shift).reshape(a.shape)
    axes = tuple(axis) if isinstance(axis, (tuple, list)) else (axis,)
    shifts = tuple(shift) if isinstance(shift, (tuple, list)) else (shift,)
    if len(shifts) == 1 and len(axes) > 1:
        shifts = shifts * len(axes)        # numpy broadcasts one shift over several axes
    elif len(axes) == 1 and len(shifts) > 1:
        axes = axes * len(shifts)
    return torch.roll(a, shifts, axes)


@register('_npi_rot90', arg_names=('a',), params={'k': ('int', 1), 'axes': ('shape', (0, 1))})
def _rot90(a, k=1, axes=(0, 1)):
    return torch.rot90(a, k, list(axes))


@register('_npi_tile', aliases=('_np_tile',), arg_names=('a',), params={'reps': ('shape', ())})
def _tile(a, reps=()):
    return torch.tile(a, tuple(reps))


@register('_np_repeat', aliases=('_npi_repeat', '_npi_repeats'), arg_names=('a',),
          params={'repeats': ('any', 1), 'axis': ('int?', None)})
def _repeat(a, repeats=1, axis=None):
    if axis is None:
        a, axis = a.reshape(-1), 0
    if isinstance(repeats, (list, tuple)):
        repeats = torch.as_tensor(repeats, device=a.device)
    return torch.repeat_interleave(a, repeats, dim=axis)


@register('_npi_broadcast_to', aliases=('_np_broadcast_to',), arg_names=('a',), params={'shape': ('shape', ())})
def _broadcast_to(a, shape=()):
    shape = list(shape)
    if any(d == -2 for d in shape):
        # npx semantics: -2 keeps the input's size of the dimension it aligns with (right-aligned)
        off = len(shape) - a.dim()
        for i, d in enumerate(shape):
            if d == -2:
                if i - off < 0:
                    raise ValueError('broadcast_to: -2 at axis %d has no input dimension to copy' % i)
                shape[i] = a.shape[i - off]
    return a.expand(tuple(shape)).clone()


@register('_npi_ravel', aliases=('_np_ravel',), arg_names=('a',), params={'order': ('str', 'C')})
def _ravel(a, order='C'):
    return a.reshape(-1) if order == 'C' else a.t().reshape(-1) if a.dim() == 2 else \
        a.permute(*reversed(range(a.dim()))).reshape(-1)


@register('_npi_tril', arg_names=('a',), params={'k': ('int', 0)})
def _tril(a, k=0):
    if a.dim() == 1:        # numpy: a vector is broadcast to its square matrix first
        a = a.unsqueeze(0).expand(a.shape[0], a.shape[0])
    return torch.tril(a, k)


@register('_npi_triu', arg_names=('a',), params={'k': ('int', 0)})
def _triu(a, k=0):
    if a.dim() == 1:
        a = a.unsqueeze(0).expand(a.shape[0], a.shape[0])
    return torch.triu(a, k)


@register('_np_diag', aliases=('_npi_diag',), arg_names=('a',), params={'k': ('int', 0)})
def _diag(a, k=0):
    return torch.diag(a, k)


@register('_np_diagflat', aliases=('_npi_diagflat',), arg_names=('a',), params={'k': ('int', 0)})
def _diagflat(a, k=0):
    return torch.diagflat(a, k)


@register('_np_diagonal', aliases=('_npi_diagonal',), arg_names=('a',),
          params={'offset': ('int', 0), 'axis1': ('int', 0), 'axis2': ('int', 1)})
def _diagonal(a, offset=0, axis1=0, axis2=1):
    return torch.diagonal(a, offset, axis1, axis2).clone()


@register('_np_trace', aliases=('_npi_trace',), arg_names=('a',),
          params={'offset': ('int', 0), 'axis1': ('int', 0), 'axis2': ('int', 1)})
def _trace(a, offset=0, axis1=0, axis2=1):
    return torch.diagonal(a, offset, axis1, axis2).sum(-1)


@register('_npi_pad', arg_names=('a',), params={'pad_width': ('any', ()), 'mode': ('str', 'constant'),
                                               'constant_values': ('float', 0.0), 'reflect_type': ('str', 'even')})
def _pad(a, pad_width=(), mode='constant', constant_values=0.0, reflect_type='even'):
    """numpy.pad (src/operator/numpy/np_pad_op-inl.h).  Constant padding is one device op; the
    index-permuting modes (reflect, symmetric, edge, wrap) gather through a host-computed index
    map (numpy's own rules applied to element codes); the statistic modes pad axis by axis."""
    pw = onp.broadcast_to(onp.asarray(pad_width, dtype=onp.int64).reshape(-1, 2) if onp.ndim(pad_width) else
                          onp.full((1, 2), pad_width), (a.dim(), 2))
    if mode == 'constant':
        flat = []
        for lo, hi in reversed(pw.tolist()):
            flat += [lo, hi]
        return torch.nn.functional.pad(a, flat, value=constant_values)
    if mode in ('reflect', 'symmetric', 'edge', 'wrap'):
        if reflect_type != 'even' and mode in ('reflect', 'symmetric'):
            raise NotImplementedError("pad: reflect_type='odd'")
        return _gather_map(onp.pad(_codes(tuple(a.shape)), pw, mode=mode), a)
    stat = {'minimum': lambda x, d: x.amin(d, keepdim=True), 'maximum': lambda x, d: x.amax(d, keepdim=True),
            'mean': lambda x, d: x.mean(d, keepdim=True) if x.is_floating_point() else
            x.double().mean(d, keepdim=True).round().to(x.dtype)}.get(mode)
    if stat is None:
        raise MXNetError('pad: unsupported mode %s' % mode)
    x = a
    for d, (lo, hi) in enumerate(pw.tolist()):
        if not (lo or hi):
            continue
        s_ = stat(x, d)
        shp = list(x.shape)
        parts = []
        if lo:
            shp[d] = lo
            parts.append(s_.expand(shp))
        parts.append(x)
        if hi:
            shp[d] = hi
            parts.append(s_.expand(shp))
        x = torch.cat(parts, d)
    return x


@register('_npi_clip', aliases=('_np_clip',), arg_names=('a',), params={'a_min': ('float?', None), 'a_max': ('float?', None)})
def _clip(a, a_min=None, a_max=None):
    return torch.clamp(a, a_min, a_max)


def _where_cast(x, y):
    rt = torch.result_type(x, y)
    return x.to(rt), y.to(rt)


@register('_npi_where', arg_names=('condition', 'x', 'y'))
def _where(condition, x, y):
    x, y = _where_cast(x, y)
    return torch.where(condition.bool(), x, y)


@register('_npi_where_lscalar', arg_names=('condition', 'y'), params={'scalar': ('any', 0.0)})
def _where_l(condition, y, scalar=0.0):
    s = _scalar_tensor(y, scalar)
    return torch.where(condition.bool(), s.to(y.dtype) if s.dtype == y.dtype else s, y.to(s.dtype))


@register('_npi_where_rscalar', arg_names=('condition', 'x'), params={'scalar': ('any', 0.0)})
def _where_r(condition, x, scalar=0.0):
    s = _scalar_tensor(x, scalar)
    return torch.where(condition.bool(), x.to(s.dtype), s)


@register('_npi_where_scalar2', arg_names=('condition',), params={'x': ('any', 0.0), 'y': ('any', 0.0)})
def _where_ss(condition, x=0.0, y=0.0):
    dt = _FLOAT if isinstance(x, float) or isinstance(y, float) else torch.int64
    return torch.where(condition.bool(), torch.tensor(x, dtype=dt, device=condition.device),
                       torch.tensor(y, dtype=dt, device=condition.device))


@register('_npi_take', arg_names=('a', 'indices'), params={'axis': ('int?', None), 'mode': ('str', 'raise')})
def _take(a, indices, axis=None, mode='raise'):
    idx = indices.long()
    if axis is None:
        a, axis = a.reshape(-1), 0
    axis %= max(a.dim(), 1)
    n = a.shape[axis]
    if mode == 'wrap':
        idx = idx % n
    elif mode == 'clip':
        idx = idx.clamp(0, n - 1)
    else:
        idx = torch.where(idx < 0, idx + n, idx)
    out = torch.index_select(a, axis, idx.reshape(-1))
    return out.reshape(tuple(a.shape[:axis]) + tuple(idx.shape) + tuple(a.shape[axis + 1:]))


@register('_npi_take_along_axis', arg_names=('arr', 'indices'), params={'axis': ('int?', None)})
def _take_along_axis(arr, indices, axis=None):
    if axis is None:
        return torch.take_along_dim(arr.reshape(-1), indices.long().reshape(-1))
    return torch.take_along_dim(arr, indices.long(), dim=axis)


def _cat_dtype(ts):
    rt = ts[0].dtype
    for t in ts[1:]:
        rt = torch.promote_types(rt, t.dtype)
    return [t.to(rt) for t in ts]


@register('_npi_concatenate', aliases=('_np_concatenate',), arg_names=lambda a: ['data%d' % i for i in range(int(a.get('num_args', 1)))],
          key_var_num_args='num_args', params={'num_args': ('int', 1), 'axis': ('int?', 0)})
def _concatenate(*arrays, num_args=1, axis=0):
    ts = _cat_dtype(list(arrays))
    if axis is None:
        return torch.cat([t.reshape(-1) for t in ts])
    return torch.cat(ts, dim=axis)


@register('_npi_stack', arg_names=lambda a: ['data%d' % i for i in range(int(a.get('num_args', 1)))],
          key_var_num_args='num_args', params={'num_args': ('int', 1), 'axis': ('int', 0)})
def _stack(*arrays, num_args=1, axis=0):
    return torch.stack(_cat_dtype(list(arrays)), dim=axis)


def _atleast(t, n):
    while t.dim() < n:
        t = t.unsqueeze(0) if n < 3 or t.dim() == 0 else (t.unsqueeze(0).unsqueeze(-1) if t.dim() == 1 else t.unsqueeze(-1))
    return t


for _nd in (1, 2, 3):
    register('_npi_atleast_%dd' % _nd, arg_names=('a',))(lambda a, _nd=_nd: _atleast(a, _nd).clone()
                                                       if a.dim() >= _nd else _atleast(a, _nd))


@register('_npi_vstack', aliases=('_npi_row_stack',), arg_names=lambda a: ['data%d' % i for i in range(int(a.get('num_args', 1)))],
          key_var_num_args='num_args', params={'num_args': ('int', 1)})
def _vstack(*arrays, num_args=1):
    return torch.cat(_cat_dtype([_atleast(t, 2) for t in arrays]), 0)


@register('_npi_hstack', arg_names=lambda a: ['data%d' % i for i in range(int(a.get('num_args', 1)))],
          key_var_num_args='num_args', params={'num_args': ('int', 1)})
def _hstack(*arrays, num_args=1):
    ts = _cat_dtype([_atleast(t, 1) for t in arrays])
    return torch.cat(ts, 0 if ts[0].dim() == 1 else 1)


@register('_npi_dstack', arg_names=lambda a: ['data%d' % i for i in range(int(a.get('num_args', 1)))],
          key_var_num_args='num_args', params={'num_args': ('int', 1)})
def _dstack(*arrays, num_args=1):
    return torch.cat(_cat_dtype([_atleast(t, 3) for t in arrays]), 2)


@register('_npi_column_stack', arg_names=lambda a: ['data%d' % i for i in range(int(a.get('num_args', 1)))],
          key_var_num_args='num_args', params={'num_args': ('int', 1)})
def _column_stack(*arrays, num_args=1):
    ts = [t.reshape(-1, 1) if t.dim() < 2 else t for t in arrays]
    return torch.cat(_cat_dtype(ts), 1)


def _split_sizes(n, ios, even):
    if isinstance(ios, int):
        if even and n % ios:
            raise ValueError('array split does not result in an equal division')
        q, r = divmod(n, ios)
        return [q + (1 if i < r else 0) for i in range(ios)]
    bounds = [0] + [min(max(int(i) if i >= 0 else n + int(i), 0), n) for i in ios] + [n]
    return [max(b - a, 0) for a, b in zip(bounds[:-1], bounds[1:])]


def _split_nout(a):
    ios = a.get('indices_or_sections', 1)
    if isinstance(ios, str):
        import ast
        ios = ast.literal_eval(ios)
    return ios if isinstance(ios, int) else len(ios) + 1


def _make_split(name, even, default_axis):
    def f(a, indices_or_sections=1, axis=default_axis):
        ax = axis
        if name in ('dsplit',):
            ax = 2
        elif name == 'hsplit':
            ax = 0 if a.dim() == 1 else 1
        sizes = _split_sizes(a.shape[ax], indices_or_sections, even)
        return tuple(torch.split(a, sizes, dim=ax))
    register('_npi_' + name, arg_names=('a',), num_outputs=_split_nout,
             params={'indices_or_sections': ('any', 1), 'axis': ('int', default_axis)})(f)


for _n, _e, _ax in (('split', True, 0), ('array_split', False, 0), ('hsplit', True, 1), ('vsplit', True, 0),
                    ('dsplit', True, 2)):
    _make_split(_n, _e, _ax)


@register('_npi_sort', arg_names=('a',), params={'axis': ('int?', -1), 'kind': ('str?', None), 'order': ('any', None),
                                                 'descending': ('bool', False)})
def _sort(a, axis=-1, kind=None, order=None, descending=False):
    if axis is None:
        a, axis = a.reshape(-1), 0
    return torch.sort(a, dim=axis, descending=descending, stable=True).values


@register('_npi_argsort', arg_names=('a',), params={'axis': ('int?', -1), 'kind': ('str?', None), 'order': ('any', None),
                                                    'descending': ('bool', False), 'dtype': ('dtype', 'int64')})
def _argsort(a, axis=-1, kind=None, order=None, descending=False, dtype='int64'):
    if axis is None:
        a, axis = a.reshape(-1), 0
    return torch.argsort(a, dim=axis, descending=descending, stable=True).to(_td(dtype, torch.int64))


@register('_npi_diff', arg_names=('a',), params={'n': ('int', 1), 'axis': ('int', -1)})
def _diff(a, n=1, axis=-1):
    return torch.diff(a, n=n, dim=axis)


@register('_npi_cross', arg_names=('a', 'b'), params={'axisa': ('int', -1), 'axisb': ('int', -1), 'axisc': ('int', -1),
                                                     'axis': ('int?', None)})
def _cross(a, b, axisa=-1, axisb=-1, axisc=-1, axis=None):
    if axis is not None:
        axisa = axisb = axisc = axis
    a = torch.movedim(a, axisa, -1)
    b = torch.movedim(b, axisb, -1)
    if a.shape[-1] == 2 and b.shape[-1] == 2:
        return a[..., 0] * b[..., 1] - a[..., 1] * b[..., 0]
    if a.shape[-1] == 2:
        a = torch.nn.functional.pad(a, (0, 1))
    if b.shape[-1] == 2:
        b = torch.nn.functional.pad(b, (0, 1))
    a, b = torch.broadcast_tensors(a, b)
    return torch.movedim(torch.linalg.cross(a, b), -1, axisc)


def _gather_map(idx, arr, values=None):
    """Gather ``arr`` (codes >= 0) and ``values`` (codes < 0, value element ``-code - 1``) into the
    layout described by the int64 code array ``idx`` -- differentiable in both sources."""
    t = torch.as_tensor(onp.ascontiguousarray(idx), dtype=torch.long, device=arr.device)
    src = arr.reshape(-1)
    if values is not None:
        src = torch.cat([src, values.to(arr.dtype).reshape(-1)])
        t = torch.where(t >= 0, t, arr.numel() - 1 - t)
    return src[t.reshape(-1)].reshape(t.shape)


def _codes(shape):
    return onp.arange(int(onp.prod(shape, dtype=onp.int64)), dtype=onp.int64).reshape(shape)


@register('_npi_delete', arg_names=('arr',), params={'obj': ('any', 0), 'axis': ('int?', None)})
def _delete(arr, obj=0, axis=None):
    """numpy.delete via an index map computed on the host (src/operator/numpy/np_delete_op-inl.h):
    out-of-range entries of an index list are ignored, as in the reference."""
    codes = _codes(tuple(arr.shape))
    n = codes.size if axis is None else codes.shape[axis]
    if isinstance(obj, slice):
        o = obj
    elif onp.ndim(obj) == 0:
        o = int(obj)
    else:
        o = onp.asarray(obj, dtype=onp.int64).reshape(-1)
        o = o[(o >= 0) & (o < n)]
    return _gather_map(onp.delete(codes, o, axis=axis), arr)


@register('_npi_insert_scalar', arg_names=('arr',), params={'obj': ('any', 0), 'values': ('any', 0.0),
                                                            'axis': ('int?', None)})
def _insert(arr, obj=0, values=0.0, axis=None):
    return _insert_t(arr, torch.as_tensor(values, dtype=arr.dtype, device=arr.device), obj, axis)


@register('_npi_insert_tensor', arg_names=('arr', 'values'), params={'obj': ('any', 0), 'axis': ('int?', None)})
def _insert_tensor(arr, values, obj=0, axis=None):
    return _insert_t(arr, values.to(arr.dtype), obj, axis)


def _insert_t(arr, values, obj, axis):
    """numpy.insert: the host computes where every output element comes from (numpy's own
    placement and broadcasting rules on index codes), the device gathers."""
    o = obj if isinstance(obj, slice) or onp.ndim(obj) == 0 else onp.asarray(obj, dtype=onp.int64)
    if onp.ndim(o) == 0 and not isinstance(o, slice):
        o = int(o)
    vcodes = -1 - _codes(tuple(values.shape))
    return _gather_map(onp.insert(_codes(tuple(arr.shape)), o, vcodes, axis=axis), arr, values)


# ---------------------------------------------------------------------------
# products / linear algebra
# ---------------------------------------------------------------------------

def _promote2(a, b):
    rt = torch.promote_types(a.dtype, b.dtype)
    return a.to(rt), b.to(rt)


@register('_np_dot', aliases=('_npi_dot',), arg_names=('a', 'b'))
def _dot(a, b):
    a, b = _promote2(a, b)
    if a.dim() == 0 or b.dim() == 0:
        return a * b
    if b.dim() == 1:
        return torch.matmul(a, b)
    if a.dim() <= 2 and b.dim() <= 2:
        return torch.matmul(a, b)
    return torch.tensordot(a, b, dims=([a.dim() - 1], [b.dim() - 2]))


@register('_npi_matmul', arg_names=('a', 'b'))
def _matmul(a, b):
    a, b = _promote2(a, b)
    return torch.matmul(a, b)


@register('_npi_tensordot', arg_names=('a', 'b'), params={'axes': ('any', 2)})
def _tensordot(a, b, axes=2):
    a, b = _promote2(a, b)
    if isinstance(axes, (list, tuple)):
        axes = [list(x) if isinstance(x, (list, tuple)) else [x] for x in axes]
    return torch.tensordot(a, b, dims=axes)


@register('_npi_inner', arg_names=('a', 'b'))
def _inner(a, b):
    a, b = _promote2(a, b)
    if a.dim() == 0 or b.dim() == 0:
        return a * b
    return torch.inner(a, b)


@register('_npi_outer', arg_names=('a', 'b'))
def _outer(a, b):
    a, b = _promote2(a, b)
    return torch.outer(a.reshape(-1), b.reshape(-1))


@register('_npi_vdot', arg_names=('a', 'b'))
def _vdot(a, b):
    a, b = _promote2(a, b)
    return torch.dot(a.reshape(-1), b.reshape(-1))


@register('_npi_kron', arg_names=('a', 'b'))
def _kron(a, b):
    a, b = _promote2(a, b)
    return torch.kron(a, b)


@register('_npi_einsum', arg_names=lambda a: ['data%d' % i for i in range(int(a.get('num_args', 1)))],
          key_var_num_args='num_args', params={'num_args': ('int', 1), 'subscripts': ('str', ''),
                                               'optimize': ('any', False)})
def _einsum(*operands, num_args=1, subscripts='', optimize=False):
    return torch.einsum(subscripts, *_cat_dtype(list(operands)))


@register('_npi_norm', arg_names=('x',), params={'ord': ('any', None), 'axis': ('axis', None), 'keepdims': ('bool', False)})
def _norm(x, ord=None, axis=None, keepdims=False):
    x = _fl(x)
    if axis is None and ord is None:
        return torch.linalg.vector_norm(x, 2, keepdim=keepdims)
    if isinstance(ord, str) and ord in ('inf', '-inf'):
        ord = float(ord)
    if axis is not None and (isinstance(axis, int) or len(axis) == 1):
        return torch.linalg.vector_norm(x, 2 if ord is None else ord, dim=axis, keepdim=keepdims)
    if axis is None:
        if x.dim() == 1:
            return torch.linalg.vector_norm(x, 2 if ord is None else ord, keepdim=keepdims)
        axis = (-2, -1)
    return torch.linalg.matrix_norm(x, 'fro' if ord is None else ord, dim=axis, keepdim=keepdims)


def _lin(name, fn, nout=1, params=None, args=('A',)):
    register('_npi_' + name, arg_names=args, num_outputs=nout, params=params or {})(fn)


_lin('svd', lambda A: tuple(torch.linalg.svd(_fl(A), full_matrices=False)), 3)
_lin('cholesky', lambda A: torch.linalg.cholesky(_fl(A)))
_lin('inv', lambda A: torch.linalg.inv(_fl(A)))
_lin('det', lambda A: torch.linalg.det(_fl(A)))
_lin('slogdet', lambda A: tuple(torch.linalg.slogdet(_fl(A))), 2)
_lin('solve', lambda A, B: torch.linalg.solve(_fl(A), _fl(B)) if B.dim() != A.dim() - 1 else
     torch.linalg.solve(_fl(A), _fl(B).unsqueeze(-1)).squeeze(-1), args=('A', 'B'))
_lin('pinv_scalar_rcond', lambda A, rcond=1e-15, hermitian=False: torch.linalg.pinv(_fl(A), rtol=rcond,
                                                                                     hermitian=hermitian),
     params={'rcond': ('float', 1e-15), 'hermitian': ('bool', False)})
# rcond as an array broadcast over the batch of matrices (numpy.linalg.pinv)
_lin('pinv', lambda A, rcond, hermitian=False: torch.linalg.pinv(_fl(A), rtol=rcond.to(_fl(A).dtype),
                                                                 hermitian=hermitian),
     params={'hermitian': ('bool', False)}, args=('A', 'rcond'))
_lin('eigvals', lambda A: torch.linalg.eigvals(_fl(A)).real)
_lin('eig', lambda A: tuple(t.real for t in torch.linalg.eig(_fl(A))), 2)
_lin('eigvalsh', lambda A, UPLO='L': torch.linalg.eigvalsh(_fl(A), UPLO=UPLO), params={'UPLO': ('str', 'L')})
_lin('eigh', lambda A, UPLO='L': tuple(torch.linalg.eigh(_fl(A), UPLO=UPLO)), 2, params={'UPLO': ('str', 'L')})
_lin('qr', lambda A, mode='reduced': tuple(torch.linalg.qr(_fl(A), mode=mode)), 2, params={'mode': ('str', 'reduced')})
_lin('matrix_rank', lambda A, tol=None, hermitian=False: torch.linalg.matrix_rank(_fl(A), atol=tol, hermitian=hermitian),
     params={'tol': ('float?', None), 'hermitian': ('bool', False)})
_lin('matrix_power', lambda A, n=1: torch.linalg.matrix_power(A, n), params={'n': ('int', 1)})
_lin('lstsq', lambda A, B, rcond=None: _lstsq(A, B, rcond), 4, params={'rcond': ('float?', None)}, args=('A', 'B'))
_lin('cond', lambda A, p=None: torch.linalg.cond(_fl(A), p), params={'p': ('any', None)})


def _lstsq(A, B, rcond):
    A, B = _fl(A), _fl(B)
    vec = B.dim() == 1
    Bm = B.unsqueeze(-1) if vec else B
    sol = torch.linalg.pinv(A, rtol=rcond if rcond is not None else 1e-15 * max(A.shape)) @ Bm
    r = torch.linalg.matrix_rank(A)
    s = torch.linalg.svdvals(A)
    res = ((A @ sol - Bm) ** 2).sum(0) if A.shape[0] > A.shape[1] and int(r) == A.shape[1] else \
        torch.zeros(0, dtype=A.dtype, device=A.device)
    return (sol.squeeze(-1) if vec else sol), res, r, s


@register('_npi_tensorinv', arg_names=('a',), params={'ind': ('int', 2)})
def _tensorinv(a, ind=2):
    return torch.linalg.tensorinv(_fl(a), ind=ind)


@register('_npi_tensorsolve', arg_names=('a', 'b'), params={'a_axes': ('shape?', None)})
def _tensorsolve(a, b, a_axes=None):
    """numpy.linalg.tensorsolve's reshaping rules, including 0-d operands and a.ndim == b.ndim."""
    a, b = _fl(a), _fl(b)
    an = a.dim()
    if a_axes is not None:
        order = [k for k in range(an) if k not in [x % an for x in a_axes]] + [x % an for x in a_axes]
        a = a.permute(order)
    tail = tuple(a.shape)[-(an - b.dim()):]
    n = int(onp.prod(tail, dtype=onp.int64))
    if n * n != a.numel() or n != b.numel():
        raise MXNetError('tensorsolve: a of shape %s is not square for b of shape %s' % (tuple(a.shape), tuple(b.shape)))
    return torch.linalg.solve(a.reshape(n, n), b.reshape(n)).reshape(tail)


@register('_npi_multi_dot', arg_names=lambda a: ['data%d' % i for i in range(int(a.get('num_args', 1)))],
          key_var_num_args='num_args', params={'num_args': ('int', 1)})
def _multi_dot(*arrays, num_args=1):
    return torch.linalg.multi_dot(_cat_dtype(list(arrays)))


# ---------------------------------------------------------------------------
# random (graph-capable samplers; the host-side rest lives in mx.np.random)
# ---------------------------------------------------------------------------

_RND = {'size': ('shape?', None), 'ctx': ('any', None), 'dtype': ('dtype', 'float32')}


def _size(size):
    return () if size is None else tuple(size)


@register('_npi_uniform', arg_names=(), params=dict(_RND, low=('float', 0.0), high=('float', 1.0)))
def _uniform(low=0.0, high=1.0, size=None, ctx=None, dtype='float32'):
    r = torch.rand(_size(size), dtype=_td(dtype, _FLOAT), device=_dev(ctx))
    return r * (high - low) + low


@register('_npi_normal', arg_names=(), params=dict(_RND, loc=('float', 0.0), scale=('float', 1.0)))
def _normal(loc=0.0, scale=1.0, size=None, ctx=None, dtype='float32'):
    if scale < 0:
        from ..base import AsyncOpError
        raise AsyncOpError('Check failed: scale >= 0 (normal sampler: scale=%s)' % scale)
    return torch.randn(_size(size), dtype=_td(dtype, _FLOAT), device=_dev(ctx)) * scale + loc


@register('_npi_random_randint', arg_names=(), params=dict(_RND, low=('int', 0), high=('int?', None), dtype=('dtype', 'int64')))
def _randint(low=0, high=None, size=None, ctx=None, dtype='int64'):
    if high is None:
        low, high = 0, low
    return torch.randint(low, high, _size(size), device=_dev(ctx)).to(_td(dtype, torch.int64))


@register('_npi_bernoulli', arg_names=(), params=dict(_RND, prob=('float', 0.5)))
def _bernoulli(prob=0.5, size=None, ctx=None, dtype='float32'):
    return (torch.rand(_size(size), device=_dev(ctx)) < prob).to(_td(dtype, _FLOAT))


@register('_npi_uniform_like', arg_names=('a',), params={'low': ('float', 0.0), 'high': ('float', 1.0)})
def _uniform_like(a, low=0.0, high=1.0):
    return torch.rand_like(_fl(a)) * (high - low) + low


@register('_npi_normal_like', arg_names=('a',), params={'loc': ('float', 0.0), 'scale': ('float', 1.0)})
def _normal_like(a, loc=0.0, scale=1.0):
    return torch.randn_like(_fl(a)) * scale + loc


# ---------------------------------------------------------------------------
# npx-only operators
# ---------------------------------------------------------------------------

def _masked(x, mask, axis, temperature, log):
    m = mask.bool()
    z = x.float() / temperature
    z = z.masked_fill(~m, float('-inf'))
    if log:
        r = torch.log_softmax(z, dim=axis)
    else:
        r = torch.softmax(z, dim=axis)
    return torch.where(m, r, torch.zeros_like(r) if not log else torch.full_like(r, float('-inf'))).to(x.dtype)


@register('masked_softmax', aliases=('_npx_masked_softmax',), arg_names=('data', 'mask'),
          params={'axis': ('int', -1), 'temperature': ('float', 1.0), 'normalize': ('bool', True)})
def masked_softmax(data, mask, axis=-1, temperature=1.0, normalize=True):
    return _masked(data, mask, axis, temperature, False)


@register('masked_log_softmax', aliases=('_npx_masked_log_softmax',), arg_names=('data', 'mask'),
          params={'axis': ('int', -1), 'temperature': ('float', 1.0), 'normalize': ('bool', True)})
def masked_log_softmax(data, mask, axis=-1, temperature=1.0, normalize=True):
    return _masked(data, mask, axis, temperature, True)


@register('_contrib_index_add', aliases=('_npx_index_add',), arg_names=('a', 'ind', 'val'))
def index_add(a, ind, val):
    idx = tuple(ind.long())
    out = a.clone()
    return out.index_put(idx, val.to(a.dtype).expand(out[idx].shape) if val.dim() < out[idx].dim() else val.to(a.dtype),
                         accumulate=True)


@register('_contrib_index_update', aliases=('_npx_index_update',), arg_names=('a', 'ind', 'val'))
def index_update(a, ind, val):
    idx = tuple(ind.long())
    out = a.clone()
    return out.index_put(idx, val.to(a.dtype).expand(out[idx].shape) if val.dim() < out[idx].dim() else val.to(a.dtype))


@register('_npx_constraint_check', arg_names=('input',), params={'msg': ('str', 'Constraint violated.')})
def constraint_check(input, msg='Constraint violated.'):  # noqa: A002
    if input.device.type != 'meta' and not bool(torch.all(input.bool())):
        raise ValueError(msg)
    return torch.ones((), dtype=torch.bool, device=input.device)


@register('_npx_reshape', arg_names=('a',), params={'newshape': ('any', ()), 'reverse': ('bool', False),
                                                   'order': ('str', 'C')})
def npx_reshape(a, newshape=(), reverse=False, order='C'):
    """npx.reshape special codes: -1 infer, -2 copy dim, -3 drop a size-1 dim, -4 copy the rest,
    -5 merge two dims, -6 split one dim into the next two values (one may be -1)."""
    src = list(a.shape)
    spec = list(newshape) if isinstance(newshape, (list, tuple)) else [newshape]
    if reverse:
        src, spec = src[::-1], spec[::-1]
    out, i, j = [], 0, 0
    infer_at = None
    while j < len(spec):
        s = spec[j]
        if s == -1:
            infer_at = len(out)
            out.append(-1)
            i += 1
        elif s == -2:
            out.append(src[i])
            i += 1
        elif s == -3:
            if src[i] != 1:
                raise ValueError('npx.reshape -3 requires a size-1 dimension')
            i += 1
        elif s == -4:
            out.extend(src[i:])
            i = len(src)
        elif s == -5:
            out.append(src[i] * src[i + 1])
            i += 2
        elif s == -6:
            d1, d2 = spec[j + 1], spec[j + 2]
            if d1 == -1:
                d1 = src[i] // d2
            if d2 == -1:
                d2 = src[i] // d1
            out.extend([d1, d2])
            i += 1
            j += 2
        else:
            out.append(s)
            i += 1
        j += 1
    if reverse:
        out = out[::-1]
    return a.reshape(out)


# ---------------------------------------------------------------------------
# mx.np.random samplers with array parameters (reference: src/operator/numpy/random/np_*_op.cc).
# One registered op for every distribution so samplers work on NDArrays, in hybridized graphs
# (Symbol parameters) and under autograd: the draws are reparameterised (x = f(params, u) with u
# from a parameter-free base distribution), which gives the reference's pathwise gradients w.r.t.
# loc / scale / shape parameters.
# ---------------------------------------------------------------------------
_SAMPLER_ARITY = {'normal': 2, 'uniform': 2, 'lognormal': 2, 'logistic': 2, 'gumbel': 2, 'laplace': 2,
                  'exponential': 1, 'rayleigh': 1, 'weibull': 1, 'pareto': 1, 'power': 1, 'gamma': 2,
                  'beta': 2, 'chisquare': 1}


def _sampler_args(attrs):
    return ['p%d' % i for i, s in enumerate(attrs.get('pscal') or ()) if s is None]


def _sampler_draw(kind, ps, shape, dev, dt):
    u = lambda: torch.rand(shape, device=dev, dtype=dt).clamp_(1e-7, 1 - 1e-7)  # noqa: E731
    if kind == 'normal':
        return ps[0] + ps[1] * torch.randn(shape, device=dev, dtype=dt)
    if kind == 'uniform':
        return ps[0] + (ps[1] - ps[0]) * torch.rand(shape, device=dev, dtype=dt)
    if kind == 'lognormal':
        return torch.exp(ps[0] + ps[1] * torch.randn(shape, device=dev, dtype=dt))
    if kind == 'logistic':
        v = u()
        return ps[0] + ps[1] * torch.log(v / (1 - v))
    if kind == 'gumbel':
        return ps[0] - ps[1] * torch.log(-torch.log(u()))
    if kind == 'laplace':
        v = u() - 0.5
        return ps[0] - ps[1] * torch.sign(v) * torch.log1p(-2 * v.abs())
    if kind == 'exponential':
        return -torch.log1p(-u()) * ps[0]
    if kind == 'rayleigh':
        return ps[0] * torch.sqrt(-2.0 * torch.log1p(-u()))
    if kind == 'weibull':
        return torch.pow(-torch.log1p(-u()), 1.0 / ps[0])
    if kind == 'pareto':
        return torch.pow(1 - u(), -1.0 / ps[0]) - 1
    if kind == 'power':
        return torch.pow(u(), 1.0 / ps[0])
    if kind == 'gamma':
        k = ps[0].expand(shape)
        return torch.distributions.Gamma(k, torch.ones_like(k)).rsample() * ps[1]
    if kind == 'beta':
        return torch.distributions.Beta(ps[0].expand(shape), ps[1].expand(shape)).rsample()
    if kind == 'chisquare':
        k = (ps[0] / 2).expand(shape)
        return torch.distributions.Gamma(k, torch.ones_like(k)).rsample() * 2
    raise MXNetError('unknown sampler %s' % kind)


def _sampler_check(kind, ps):
    from ..base import AsyncValueError

    def positive(t, name, strict=True):
        bad = (t <= 0) if strict else (t < 0)
        if bool(bad.any()):
            # a ValueError in the reference (CHECK -> "ValueError:" prefixed MXNetError)
            raise AsyncValueError('Check failed: %s %s 0 (%s sampler)' % (name, '>' if strict else '>=', kind))
    if kind in ('normal', 'lognormal', 'logistic', 'gumbel', 'laplace'):
        positive(ps[1], 'scale', strict=False)
    elif kind in ('exponential', 'rayleigh'):
        positive(ps[0], 'scale', strict=False)
    elif kind in ('weibull', 'pareto', 'power', 'chisquare'):
        positive(ps[0], 'a')
    elif kind == 'gamma':
        positive(ps[0], 'shape')
        positive(ps[1], 'scale')
    elif kind == 'beta':
        positive(ps[0], 'a')
        positive(ps[1], 'b')


@register('_npi_sampler', arg_names=_sampler_args,
          params={'kind': ('str', 'normal'), 'pscal': ('any', ()), 'size': ('any', None), 'ctx': ('any', None),
                  'dtype': ('str', 'float32'), 'batch': ('bool', False)})
def _np_sampler(*arrays, kind='normal', pscal=(), size=None, ctx=None, dtype='float32', batch=False):
    """``batch``: ``size`` is a batch shape prepended to the parameters' broadcast shape (npx *_n)."""
    dt = _td(dtype if dtype not in (None, 'None') else 'float32', _FLOAT)
    dev = arrays[0].device if arrays else _dev(ctx)
    it = iter(arrays)
    ps = []
    for s in pscal:
        if s is None:
            a = next(it)
            ps.append(a.to(dt) if a.dtype != dt else a)
        else:
            ps.append(torch.tensor(float(s), device=dev, dtype=dt))
    pshape = tuple(torch.broadcast_shapes(*[tuple(p.shape) for p in ps])) if ps else ()
    if size is None or size == ():
        shape = pshape
    else:
        shape = (int(size),) if isinstance(size, int) else tuple(int(d) for d in size)
        if batch:
            shape = shape + pshape
    _sampler_check(kind, ps)
    if 0 in shape:
        z = torch.zeros(shape, device=dev, dtype=dt)
        # keep the (empty) result on the autograd tape of the parameters
        return z + sum(p.sum() for p in ps if p.requires_grad) * 0 if any(p.requires_grad for p in ps) else z
    cdt = torch.float32 if dt in (torch.float16, torch.bfloat16) and dev.type == 'cpu' else dt
    ps = [(p.expand(shape) if p.dim() else p).to(cdt) for p in ps]
    return _sampler_draw(kind, ps, shape, dev, cdt).to(dt)



# ---------------------------------------------------------------------------
# generic node for host-computed / data-dependent numpy functions in graphs (see
# numpy/multiarray.py _host_graph): the function is looked up by name at run time
# ---------------------------------------------------------------------------
@register('_npi_host_call', arg_names=lambda a: ['data%d' % i for i in range(int(a.get('num_args', 0) or 0))],
          key_var_num_args='num_args', num_outputs=lambda a: int(a.get('nout', 1) or 1),
          params={'fn': ('str', ''), 'names': ('str', '[]'), 'kwargs': ('str', '{}'), 'nout': ('int', 1),
                  'num_args': ('int', 0)})
def np_host_call(*data, fn='', names='[]', kwargs='{}', nout=1, num_args=0):
    from ..numpy import multiarray as _ma
    return _ma._run_host_call(list(data), fn, names, kwargs)


@register('_npi_polyval', arg_names=['p', 'x'])
def npi_polyval(p, x):
    """Horner evaluation of the coefficient vector ``p`` at ``x`` (src/operator/numpy/np_polynomial_op.cc)."""
    dt = torch.promote_types(p.dtype, x.dtype)
    r = torch.zeros_like(x, dtype=dt)
    for i in range(p.shape[0]):
        r = r * x + p[i]
    return r


# ---------------------------------------------------------------------------
# boolean-mask assignment (a[mask] = v with the mask starting at ``start_axis``)
# src/operator/numpy/np_boolean_mask_assign.cc
# ---------------------------------------------------------------------------
def _mask_assign(data, mask, value, start_axis):
    start_axis %= max(data.dim(), 1)
    if tuple(data.shape[start_axis:start_axis + mask.dim()]) != tuple(mask.shape):
        raise MXNetError('boolean_mask_assign: mask of shape %s does not match data %s at axis %d'
                         % (tuple(mask.shape), tuple(data.shape), start_axis))
    out = data.clone()
    out[(slice(None),) * start_axis + (mask.to(torch.bool),)] = value.to(out.dtype)   # broadcasts
    return out


@register('_npi_boolean_mask_assign_scalar', arg_names=('data', 'mask'),
          params={'value': ('float', 0.0), 'start_axis': ('int', 0)})
def _bool_assign_scalar(data, mask, value=0.0, start_axis=0):
    return _mask_assign(data, mask, torch.tensor(value, device=data.device), start_axis)


@register('_npi_boolean_mask_assign_tensor', arg_names=('data', 'mask', 'value'), params={'start_axis': ('int', 0)})
def _bool_assign_tensor(data, mask, value, start_axis=0):
    return _mask_assign(data, mask, value, start_axis)
