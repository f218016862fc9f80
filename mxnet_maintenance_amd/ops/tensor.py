"""Tensor operators: elementwise, broadcast, scalar, reduce, matrix, indexing, init.

Parity: src/operator/tensor/*.cc (elemwise_unary_op_*.cc, elemwise_binary_*.cc,
elemwise_binary_scalar_op_*.cc, broadcast_reduce_op_*.cc, matrix_op.cc,
indexing_op.cc, init_op.cc, ordering_op.cc, dot.cc, control_flow_op.cc).
Semantics follow MXNet 1.x "legacy" shapes: a full reduction returns shape (1,),
comparison operators return 0/1 in the input dtype.

These are the torch reference implementations; the GPU hot path for fused
elementwise work lives in ops/hip_ops.py and is selected by the callers that
can fuse (BatchNorm+ReLU+add, softmax-CE, optimizer updates).
"""
import math

import numpy as np
import torch

from .. import _state
from ..base import torch_dtype, MXNetError
from .registry import register, alias


def _legacy(t):
    """MXNet 1.x legacy shape semantics: no 0-d arrays."""
    if t.dim() == 0 and not _state.STATE.np_shape:
        return t.reshape(1)
    return t


def _float_like(t):
    return t if t.is_floating_point() else t.to(torch.float32)


# ---------------------------------------------------------------------------
# unary math
# ---------------------------------------------------------------------------

def _rcbrt(x):
    return torch.sign(x) * torch.abs(x).pow(-1.0 / 3)


class _Cbrt(torch.autograd.Function):
    """Real cube root with the reference gradient 1 / (3 cbrt(x)^2) (inf at 0; the
    sign * |x|^(1/3) composition gives 0 * inf = NaN there)."""

    @staticmethod
    def forward(ctx, x):
        y = torch.sign(x) * torch.abs(x).pow(1.0 / 3)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, g):
        y, = ctx.saved_tensors
        return g / (3 * y * y)


def _cbrt(x):
    return _Cbrt.apply(x) if x.requires_grad else torch.sign(x) * torch.abs(x).pow(1.0 / 3)


class _Relu(torch.autograd.Function):
    """relu whose gradient propagates NaN inputs (reference: mshadow_op relu_grad returns NaN for a
    NaN input, test_ndarray.py:test_ndarray_nan_comparison); torch's threshold gradient zeroes them."""

    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return torch.relu(x)

    @staticmethod
    def backward(ctx, g):
        x, = ctx.saved_tensors
        return torch.where(x > 0, g, torch.where(torch.isnan(x), x, torch.zeros_like(g)))


def _relu(x):
    if x.is_cuda:
        from . import hip_ops
        return hip_ops.relu(x)         # src/kernels/pointwise.hip
    return _Relu.apply(x) if x.requires_grad and x.is_floating_point() else torch.relu(x)


def _tgamma(x):
    """Gamma function with C tgamma's signs and poles: negative between odd/even negative integers,
    +inf at +0, nan at negative integers."""
    x = x if x.is_floating_point() else x.to(torch.float32)
    mag = torch.exp(torch.lgamma(x))
    neg_odd = (x < 0) & (torch.remainder(torch.ceil(-x), 2) == 1)
    r = torch.where(neg_odd, -mag, mag)
    return torch.where((x < 0) & (x == torch.floor(x)), torch.full_like(r, float('nan')), r)


class _Gamma(torch.autograd.Function):
    """d/dx gamma = gamma(x) * psi(x), with psi = +inf at the non-positive integers (the reference's
    psi, src/operator/mshadow_op.h special_functions::cephes::psi)."""

    @staticmethod
    def forward(ctx, x):
        y = _tgamma(x)
        ctx.save_for_backward(x, y)
        return y

    @staticmethod
    def backward(ctx, g):
        x, y = ctx.saved_tensors
        return g * y * _psi_ref(x)


def _gamma(x):
    return _Gamma.apply(x) if x.requires_grad else _tgamma(x)


def _psi_ref(x):
    return torch.where((x <= 0) & (x == torch.floor(x)), torch.full_like(x, float('inf')), torch.digamma(x))


class _Gammaln(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return torch.lgamma(x)

    @staticmethod
    def backward(ctx, g):
        x, = ctx.saved_tensors
        return g * _psi_ref(x)


def _gammaln(x):
    return _Gammaln.apply(x) if x.requires_grad else torch.lgamma(x)


class _ArcsinhPrime(torch.autograd.Function):
    """f'(x) = (x^2 + 1)^(-1/2) of arcsinh, differentiated the way the reference's second-order
    gradient does it: src/operator/tensor/elemwise_unary_op_trig.cc:506 writes
    f''(x) = f'(x) * x / (x^2 + 1) = x / (x^2 + 1)^(3/2) (mathematically -x / (x^2 + 1)^(3/2)); models
    and tests that use arcsinh's higher-order gradient see the reference's values."""

    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return torch.rsqrt(x * x + 1)

    @staticmethod
    def backward(ctx, g):
        x, = ctx.saved_tensors
        fp = _ArcsinhPrime.apply(x)
        return g * fp * fp * fp * x


class _Arcsinh(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return torch.asinh(x)

    @staticmethod
    def backward(ctx, g):
        x, = ctx.saved_tensors
        return g * _ArcsinhPrime.apply(x)


def _arcsinh(x):
    return _Arcsinh.apply(x) if x.requires_grad else torch.asinh(x)


_UNARY = {
    'abs': torch.abs, 'sign': torch.sign, 'round': torch.round,
    'rint': torch.round, 'ceil': torch.ceil, 'floor': torch.floor, 'trunc': torch.trunc,
    'fix': torch.trunc, 'square': torch.square, 'sqrt': torch.sqrt, 'rsqrt': torch.rsqrt,
    'cbrt': _cbrt, 'rcbrt': _rcbrt,
    'exp': torch.exp, 'log': torch.log, 'log10': torch.log10, 'log2': torch.log2,
    'log1p': torch.log1p, 'expm1': torch.expm1, 'gamma': _gamma,
    'gammaln': _gammaln, 'erf': torch.erf, 'erfinv': torch.erfinv,
    'sin': torch.sin, 'cos': torch.cos, 'tan': torch.tan, 'arcsin': torch.asin,
    'arccos': torch.acos, 'arctan': torch.atan, 'degrees': torch.rad2deg,
    'radians': torch.deg2rad, 'sinh': torch.sinh, 'cosh': torch.cosh, 'tanh': torch.tanh,
    'arcsinh': _arcsinh, 'arccosh': torch.acosh, 'arctanh': torch.atanh,
    'reciprocal': torch.reciprocal, 'negative': torch.neg, 'relu': _relu,
    'sigmoid': torch.sigmoid, 'softsign': lambda x: x / (1 + torch.abs(x)),
    'logical_not': lambda x: (x == 0).to(x.dtype),
    'log_sigmoid': torch.nn.functional.logsigmoid,
    'mish': lambda x: x * torch.tanh(torch.nn.functional.softplus(x)),
    'digamma': torch.digamma,
}

for _n, _f in _UNARY.items():
    register(_n, (lambda f: lambda data: f(data))(_f))
alias('negative', '_np_negative')


def encode_basic_index(key):
    """A basic (view) index -- ints, slices, None, Ellipsis, or a tuple of them -- as a JSON string,
    the ``key`` attribute of ``_npi_basic_index``."""
    import json
    items = key if isinstance(key, tuple) else (key,)
    enc = []
    for k in items:
        if isinstance(k, slice):
            enc.append(['s', k.start, k.stop, k.step])
        elif k is None:
            enc.append(['n'])
        elif k is Ellipsis:
            enc.append(['e'])
        elif isinstance(k, (int, np.integer)) and not isinstance(k, bool):
            enc.append(['i', int(k)])
        else:
            raise TypeError('symbolic numpy indexing supports ints, slices, None and Ellipsis, got %r' % (k,))
    return json.dumps(enc)


def _decode_basic_index(enc):
    import json
    out = []
    for item in json.loads(enc):
        tag = item[0]
        out.append(slice(*item[1:]) if tag == 's' else None if tag == 'n' else Ellipsis if tag == 'e'
                   else item[1])
    return tuple(out)


@register('_npi_basic_index', params={'key': ('str', '[]')})
def _npi_basic_index(data, key='[]'):
    """x[key] for a basic index in a numpy-mode symbol graph (reference: numpy _Symbol.__getitem__,
    python/mxnet/symbol/numpy/_symbol.py, lowered there to slice / reshape / expand_dims ops)."""
    from ..ndarray.ndarray import _index_fn
    return _index_fn(data, _decode_basic_index(key)).contiguous()


@register('hard_sigmoid', params={'alpha': ('float', 0.2), 'beta': ('float', 0.5)})
def hard_sigmoid(data, alpha=0.2, beta=0.5):
    return torch.clamp(data * alpha + beta, 0, 1)


@register('_copy', aliases=('identity', '_identity_with_attr_like_rhs_dummy'))
def _copy(data):
    return data.clone()


@register('BlockGrad', aliases=('stop_gradient',))
def block_grad(data):
    return data.detach()


@register('zeros_like')
def zeros_like(data):
    return torch.zeros_like(data)


@register('ones_like')
def ones_like(data):
    return torch.ones_like(data)


@register('Cast', aliases=('cast', 'amp_cast'), params={'dtype': ('str', 'float32')})
def cast(data, dtype='float32'):
    return data.to(torch_dtype(dtype))


@register('amp_multicast', arg_names=lambda a: ['data_%d' % i for i in range(int(a.get('num_outputs', 1)))],
          num_outputs=lambda a: int(a.get('num_outputs', 1)),
          params={'num_outputs': ('int', 1), 'cast_narrow': ('bool', False)})
def amp_multicast(*data, num_outputs=1, cast_narrow=False):
    dts = [d.dtype for d in data]
    order = [torch.float16, torch.bfloat16, torch.float32, torch.float64]
    key = min if cast_narrow else max
    tgt = key(dts, key=lambda d: order.index(d) if d in order else 2)
    return tuple(d.to(tgt) for d in data)


@register('clip', params={'a_min': ('float', None), 'a_max': ('float', None)})
def clip(data, a_min=None, a_max=None):
    return torch.clamp(data, a_min, a_max)


@register('smooth_l1', params={'scalar': ('float', 1.0)})
def smooth_l1(data, scalar=1.0):
    s2 = scalar * scalar
    a = torch.abs(data)
    return torch.where(a < 1.0 / s2, 0.5 * s2 * data * data, a - 0.5 / s2)


# ---------------------------------------------------------------------------
# binary (same shape / broadcast) and scalar variants
# ---------------------------------------------------------------------------

def _cmp(f):
    def g(a, b):
        r = f(a, b)
        return r.to(a.dtype if torch.is_tensor(a) else b.dtype)
    return g


def _mod(a, b):
    """Python-sign modulo; x % 0 is 0 (reference mshadow_op::mod), also for integers."""
    if not torch.is_tensor(b):
        if b == 0:
            return torch.zeros_like(a)
        return torch.remainder(a, b)
    zero = b == 0
    if not torch.is_tensor(a):
        a = torch.full_like(b, a)
    r = torch.remainder(a, torch.where(zero, torch.ones_like(b), b))
    return torch.where(zero, torch.zeros_like(r), r)


def _logical(f):
    def g(a, b):
        dt = a.dtype if torch.is_tensor(a) else b.dtype
        return f(a != 0, b != 0).to(dt)
    return g


class _MaxMin(torch.autograd.Function):
    """maximum / minimum with the reference's tie rule: the whole gradient goes to the lhs where
    lhs >= rhs (maximum) or lhs <= rhs (minimum) -- mshadow_op::ge / le, not torch's even split."""

    @staticmethod
    def forward(ctx, a, b, is_max):
        ctx.is_max = is_max
        ctx.save_for_backward(a, b)
        return torch.maximum(a, b) if is_max else torch.minimum(a, b)

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        take_a = (a >= b) if ctx.is_max else (a <= b)
        ga = torch.where(take_a, g, torch.zeros_like(g))
        gb = g - ga
        return _sum_to(ga, a.shape).to(a.dtype), _sum_to(gb, b.shape).to(b.dtype), None


def _sum_to(g, shape):
    if tuple(g.shape) == tuple(shape):
        return g
    lead = g.dim() - len(shape)
    dims = list(range(lead)) + [lead + i for i, n in enumerate(shape) if n == 1 and g.shape[lead + i] != 1]
    return g.sum(dim=dims, keepdim=True).reshape(shape) if dims else g.reshape(shape)


def _maximum(a, b):
    if (a.requires_grad or b.requires_grad) and a.is_floating_point() and b.is_floating_point():
        return _MaxMin.apply(a, b, True)
    return torch.maximum(a, b)


def _minimum(a, b):
    if (a.requires_grad or b.requires_grad) and a.is_floating_point() and b.is_floating_point():
        return _MaxMin.apply(a, b, False)
    return torch.minimum(a, b)


_BINARY = {
    'add': torch.add, 'sub': torch.sub, 'mul': torch.mul,
    'div': lambda a, b: torch.div(a, b) if (a.is_floating_point() if torch.is_tensor(a) else True) else torch.div(a, b, rounding_mode='trunc'),
    'mod': _mod, 'power': torch.pow, 'maximum': _maximum, 'minimum': _minimum,
    'hypot': torch.hypot,
    'equal': _cmp(torch.eq), 'not_equal': _cmp(torch.ne), 'greater': _cmp(torch.gt),
    'greater_equal': _cmp(torch.ge), 'lesser': _cmp(torch.lt), 'lesser_equal': _cmp(torch.le),
    'logical_and': _logical(torch.logical_and), 'logical_or': _logical(torch.logical_or),
    'logical_xor': _logical(torch.logical_xor),
}

_ELEMWISE_NAMES = {'add': ['elemwise_add', '_plus', '_add', '_Plus'],
                   'sub': ['elemwise_sub', '_minus', '_sub', '_Minus'],
                   'mul': ['elemwise_mul', '_mul', '_Mul'],
                   'div': ['elemwise_div', '_div', '_Div'],
                   'mod': ['_mod', '_Mod'], 'power': ['_power', '_Power'],
                   'maximum': ['_maximum', '_Maximum'], 'minimum': ['_minimum', '_Minimum'],
                   'hypot': ['_hypot', '_Hypot'], 'equal': ['_equal'], 'not_equal': ['_not_equal'],
                   'greater': ['_greater'], 'greater_equal': ['_greater_equal'],
                   'lesser': ['_lesser'], 'lesser_equal': ['_lesser_equal'],
                   'logical_and': ['_logical_and'], 'logical_or': ['_logical_or'],
                   'logical_xor': ['_logical_xor']}

_BCAST_NAMES = {'add': ['broadcast_add', 'broadcast_plus'], 'sub': ['broadcast_sub', 'broadcast_minus'],
                'mul': ['broadcast_mul'], 'div': ['broadcast_div'], 'mod': ['broadcast_mod'],
                'power': ['broadcast_power'], 'maximum': ['broadcast_maximum'],
                'minimum': ['broadcast_minimum'], 'hypot': ['broadcast_hypot'],
                'equal': ['broadcast_equal'], 'not_equal': ['broadcast_not_equal'],
                'greater': ['broadcast_greater'], 'greater_equal': ['broadcast_greater_equal'],
                'lesser': ['broadcast_lesser'], 'lesser_equal': ['broadcast_lesser_equal'],
                'logical_and': ['broadcast_logical_and'], 'logical_or': ['broadcast_logical_or'],
                'logical_xor': ['broadcast_logical_xor']}


_HIP_BINARY = ('add', 'sub', 'mul', 'div', 'maximum', 'minimum')


def _make_binary(f, name=None):
    if name not in _HIP_BINARY:
        def op(lhs, rhs):
            return f(lhs, rhs)
        return op

    def op_hip(lhs, rhs):
        # GPU operands of one dtype: the in-tree broadcast kernel (src/kernels/pointwise.hip)
        if lhs.is_cuda:
            from . import hip_ops
            r = hip_ops.binary(name, lhs, rhs)
            if r is not None:
                return r
        return f(lhs, rhs)
    return op_hip


for _k, _f in _BINARY.items():
    names = _ELEMWISE_NAMES[_k]
    register(names[0], _make_binary(_f, _k), arg_names=('lhs', 'rhs'), aliases=names[1:])
    bn = _BCAST_NAMES[_k]
    register(bn[0], _make_binary(_f, _k), arg_names=('lhs', 'rhs'), aliases=bn[1:])


def _make_scalar(f, reverse=False):
    def op(data, scalar=0.0, is_int=None):
        s = scalar
        if not data.is_floating_point() and float(s).is_integer():
            s = int(s)
        return f(s, data) if reverse else f(data, s)
    return op


def _scalar_tensor_first(f):
    # torch functions like maximum/hypot need tensor args
    def g(a, b):
        if not torch.is_tensor(a):
            a = torch.full_like(b, a)
        if not torch.is_tensor(b):
            b = torch.full_like(a, b)
        return f(a, b)
    return g


_SCALAR_NAMES = {'add': ('_plus_scalar', None), 'sub': ('_minus_scalar', '_rminus_scalar'),
                 'mul': ('_mul_scalar', None), 'div': ('_div_scalar', '_rdiv_scalar'),
                 'mod': ('_mod_scalar', '_rmod_scalar'), 'power': ('_power_scalar', '_rpower_scalar'),
                 'maximum': ('_maximum_scalar', None), 'minimum': ('_minimum_scalar', None),
                 'hypot': ('_hypot_scalar', None), 'equal': ('_equal_scalar', None),
                 'not_equal': ('_not_equal_scalar', None), 'greater': ('_greater_scalar', None),
                 'greater_equal': ('_greater_equal_scalar', None), 'lesser': ('_lesser_scalar', None),
                 'lesser_equal': ('_lesser_equal_scalar', None),
                 'logical_and': ('_logical_and_scalar', None), 'logical_or': ('_logical_or_scalar', None),
                 'logical_xor': ('_logical_xor_scalar', None)}

_SCALAR_PARAMS = {'scalar': ('float', 0.0), 'is_int': ('bool?', None)}
for _k, (fwd, rev) in _SCALAR_NAMES.items():
    f = _BINARY[_k]
    if _k in ('maximum', 'minimum', 'hypot', 'mod', 'logical_and', 'logical_or', 'logical_xor'):
        f = _scalar_tensor_first(f)
    if _k == 'div':
        f = lambda a, b: a / b
    register(fwd, _make_scalar(f), params=_SCALAR_PARAMS)
    if rev:
        register(rev, _make_scalar(f, reverse=True), params=_SCALAR_PARAMS)

alias('_plus_scalar', '_PlusScalar')
alias('_minus_scalar', '_MinusScalar')
alias('_rminus_scalar', '_RMinusScalar')
alias('_mul_scalar', '_MulScalar')
alias('_div_scalar', '_DivScalar')
alias('_rdiv_scalar', '_RDivScalar')


@register('add_n', aliases=('ElementWiseSum', '_contrib_add_n'),
          arg_names=lambda a: ['arg%d' % i for i in range(int(a.get('num_args', 1)))],
          params={'num_args': ('int', 1)}, key_var_num_args='num_args')
def add_n(*args, num_args=None):
    out = args[0]
    for a in args[1:]:
        out = out + a
    return out


# ---------------------------------------------------------------------------
# reductions
# ---------------------------------------------------------------------------

def _norm_axes(axis, ndim, exclude=False):
    if axis is None or axis == ():
        axes = list(range(ndim))
        if exclude:
            axes = []
    else:
        if isinstance(axis, int):
            axis = (axis,)
        axes = [a % ndim if ndim else 0 for a in axis]
        if exclude:
            axes = [a for a in range(ndim) if a not in axes]
    return axes


_RED_PARAMS = {'axis': ('axis', None), 'keepdims': ('bool', False), 'exclude': ('bool', False)}


def _make_reduce(kind):
    def op(data, axis=None, keepdims=False, exclude=False):
        axes = _norm_axes(axis, data.dim(), exclude)
        if not axes:
            return data.clone() if kind != 'mean' else data.clone()
        x = data
        if kind == 'sum':
            r = torch.sum(x, dim=axes, keepdim=keepdims)
        elif kind == 'mean':
            r = torch.mean(_float_like(x), dim=axes, keepdim=keepdims).to(x.dtype)
        elif kind == 'prod':
            r = x
            for a in sorted(axes, reverse=True):
                r = torch.prod(r, dim=a, keepdim=keepdims)
        elif kind == 'nansum':
            r = torch.nansum(x, dim=axes, keepdim=keepdims)
        elif kind == 'nanprod':
            r = torch.where(torch.isnan(x), torch.ones_like(x), x)
            for a in sorted(axes, reverse=True):
                r = torch.prod(r, dim=a, keepdim=keepdims)
        elif kind == 'max':
            r = torch.amax(x, dim=axes, keepdim=keepdims)
        elif kind == 'min':
            r = torch.amin(x, dim=axes, keepdim=keepdims)
        else:
            raise ValueError(kind)
        return _legacy(r)
    return op


for _k, _names in {'sum': ['sum', 'sum_axis'], 'mean': ['mean'], 'prod': ['prod'],
                   'nansum': ['nansum'], 'nanprod': ['nanprod'], 'max': ['max', 'max_axis'],
                   'min': ['min', 'min_axis']}.items():
    register(_names[0], _make_reduce(_k), params=_RED_PARAMS, aliases=_names[1:])


@register('norm', params={'ord': ('int', 2), 'axis': ('axis', None), 'keepdims': ('bool', False),
                          'out_dtype': ('str?', None)})
def norm(data, ord=2, axis=None, keepdims=False, out_dtype=None):
    x = _float_like(data)
    dims = None if axis is None else ([axis] if isinstance(axis, int) else list(axis))
    if ord == 1:
        r = torch.sum(torch.abs(x), dim=dims, keepdim=keepdims) if dims is not None else torch.sum(torch.abs(x))
    else:
        r = torch.sqrt(torch.sum(x * x, dim=dims, keepdim=keepdims)) if dims is not None else torch.sqrt(torch.sum(x * x))
    if keepdims and dims is None:
        r = r.reshape([1] * data.dim())
    r = r.to(torch_dtype(out_dtype) if out_dtype else data.dtype)
    return _legacy(r)


def _argred(f):
    def op(data, axis=None, keepdims=False):
        if axis is None:
            r = f(data.reshape(-1), 0)
            if keepdims:
                r = r.reshape([1] * data.dim())
        else:
            r = f(data, axis)
            if keepdims:
                r = r.unsqueeze(axis)
        return _legacy(r.to(data.dtype if data.is_floating_point() else torch.float32))
    return op


register('argmax', _argred(lambda x, a: torch.argmax(x, a)), params={'axis': ('int?', None), 'keepdims': ('bool', False)})
register('argmin', _argred(lambda x, a: torch.argmin(x, a)), params={'axis': ('int?', None), 'keepdims': ('bool', False)})


@register('argmax_channel')
def argmax_channel(data):
    return torch.argmax(data, -1).to(data.dtype)


@register('pick', arg_names=('data', 'index'),
          params={'axis': ('int?', -1), 'keepdims': ('bool', False), 'mode': ('str', 'clip')})
def pick(data, index, axis=-1, keepdims=False, mode='clip'):
    if axis is None:
        data = data.reshape(-1)
        axis = 0
    axis = axis % data.dim()
    n = data.shape[axis]
    idx = index.to(torch.int64)
    idx = torch.remainder(idx, n) if mode == 'wrap' else torch.clamp(idx, 0, n - 1)
    idx = idx.reshape(idx.shape[:axis] + (1,) + idx.shape[axis:]) if idx.dim() < data.dim() else idx
    r = torch.gather(data, axis, idx)
    if not keepdims:
        r = r.squeeze(axis)
    return _legacy(r)


@register('broadcast_to', params={'shape': ('shape', ())})
def broadcast_to(data, shape=()):
    tgt = [d if s == 0 else s for s, d in zip(shape, data.shape)] if len(shape) == data.dim() else list(shape)
    return data.expand(*tgt).contiguous()


@register('broadcast_axis', aliases=('broadcast_axes',), params={'axis': ('axis', ()), 'size': ('shape', ())})
def broadcast_axis(data, axis=(), size=()):
    if isinstance(axis, int):
        axis = (axis,)
    tgt = list(data.shape)
    for a, s in zip(axis, size):
        tgt[a] = s
    return data.expand(*tgt).contiguous()


@register('broadcast_like', arg_names=('lhs', 'rhs'),
          params={'lhs_axes': ('shape?', None), 'rhs_axes': ('shape?', None)})
def broadcast_like(lhs, rhs, lhs_axes=None, rhs_axes=None):
    if lhs_axes is None:
        return lhs.expand_as(rhs).contiguous()
    if len(lhs_axes) == 0 or len(lhs_axes) != len(rhs_axes):
        raise MXNetError('broadcast_like: lhs_axes and rhs_axes must be non-empty and of equal length, got %s / %s'
                         % (tuple(lhs_axes), tuple(rhs_axes)))
    tgt = list(lhs.shape)
    for la, ra in zip(lhs_axes, rhs_axes):
        tgt[la] = rhs.shape[ra]
    return lhs.expand(*tgt).contiguous()


# ---------------------------------------------------------------------------
# shape manipulation
# ---------------------------------------------------------------------------

def infer_reshape(src, shape, reverse=False):
    """MXNet Reshape special codes 0, -1, -2, -3, -4 (matrix_op-inl.h InferReshapeShape)."""
    src = list(src)
    shape = list(shape)
    if reverse:
        # right-to-left: the reversed codes apply to the reversed source shape (a -4 then splits
        # into the two reversed entries after it)
        src = src[::-1]
        shape = shape[::-1]
    out = []
    si = 0
    i = 0
    infer_idx = -1
    while i < len(shape):
        s = shape[i]
        if s == 0:
            out.append(src[si]); si += 1
        elif s == -1:
            infer_idx = len(out); out.append(-1); si += 1
        elif s == -2:
            out.extend(src[si:]); si = len(src)
        elif s == -3:
            out.append(src[si] * src[si + 1]); si += 2
        elif s == -4:
            d1, d2 = shape[i + 1], shape[i + 2]
            cur = src[si]
            if d1 == -1:
                d1 = cur // d2
            if d2 == -1:
                d2 = cur // d1
            out.extend([d1, d2]); si += 1; i += 2
        else:
            out.append(s); si += 1
        i += 1
    if infer_idx >= 0:
        total = int(np.prod(src)) if src else 1
        known = int(np.prod([d for j, d in enumerate(out) if j != infer_idx])) if len(out) > 1 else 1
        out[infer_idx] = total // known if known else 0
    if reverse:
        out = out[::-1]
    return tuple(out)


@register('Reshape', aliases=('reshape',), params={'shape': ('shape', ()), 'reverse': ('bool', False),
                                                   'target_shape': ('shape?', None), 'keep_highest': ('bool', False)})
def reshape(data, shape=(), reverse=False, target_shape=None, keep_highest=False):
    if not shape and target_shape:
        # legacy target_shape: a 0 is the inferred dim; keep_highest fixes the first dim to the input's
        t = [int(d) for d in target_shape]
        if keep_highest:
            t[0] = int(data.shape[0])
        known = int(np.prod([d for d in t if d != 0])) if t else 1
        shape = tuple(d if d != 0 else data.numel() // max(known, 1) for d in t)
        return data.reshape(shape)
    return data.reshape(infer_reshape(data.shape, shape, reverse))


@register('reshape_like', arg_names=('lhs', 'rhs'),
          params={'lhs_begin': ('int?', None), 'lhs_end': ('int?', None),
                  'rhs_begin': ('int?', None), 'rhs_end': ('int?', None)})
def reshape_like(lhs, rhs, lhs_begin=None, lhs_end=None, rhs_begin=None, rhs_end=None):
    if lhs_begin is None and rhs_begin is None and lhs_end is None and rhs_end is None:
        return lhs.reshape(rhs.shape)
    def norm(v, dim, default):
        # negative positions count from the end (python slicing): -1 is the last axis
        return default if v is None else (v + dim if v < 0 else v)
    lb = norm(lhs_begin, lhs.dim(), 0)
    le = norm(lhs_end, lhs.dim(), lhs.dim())
    rb = norm(rhs_begin, rhs.dim(), 0)
    re_ = norm(rhs_end, rhs.dim(), rhs.dim())
    new = list(lhs.shape[:lb]) + list(rhs.shape[rb:re_]) + list(lhs.shape[le:])
    return lhs.reshape(new)


@register('Flatten', aliases=('flatten',))
def flatten(data):
    return data.reshape(data.shape[0], -1) if data.dim() > 0 else data.reshape(1, 1)


@register('transpose', params={'axes': ('shape', ())})
def transpose(data, axes=()):
    if not axes:
        axes = tuple(range(data.dim() - 1, -1, -1))
    return data.permute(*axes).contiguous()


@register('expand_dims', params={'axis': ('int', 0)})
def expand_dims(data, axis=0):
    return data.unsqueeze(axis if axis >= 0 else axis + data.dim() + 1)


@register('squeeze', params={'axis': ('axis', None)})
def squeeze(data, axis=None):
    if axis is None:
        r = data.squeeze()
    else:
        if isinstance(axis, int):
            axis = (axis,)
        r = data
        for a in sorted([a % data.dim() for a in axis], reverse=True):
            r = r.squeeze(a)
    return _legacy(r)


@register('SwapAxis', aliases=('swapaxes',), params={'dim1': ('int', 0), 'dim2': ('int', 0)})
def swapaxes(data, dim1=0, dim2=0):
    return data.transpose(dim1, dim2).contiguous()


def _slice_args(shape, begin, end, step):
    idx = []
    for i in range(len(shape)):
        b = begin[i] if i < len(begin) else None
        e = end[i] if i < len(end) else None
        s = step[i] if step and i < len(step) else None
        idx.append(slice(b, e, s))
    return tuple(idx)


def _neg_step_slice(data, idx):
    # torch does not support negative-step slicing: flip then slice
    out = data
    for ax, sl in enumerate(idx):
        if sl.step is not None and sl.step < 0:
            n = out.shape[ax]
            b, e, s = sl.indices(n)
            ids = torch.tensor(list(range(b, e, s)), dtype=torch.long, device=out.device)
            out = out.index_select(ax, ids)
        else:
            out = out[(slice(None),) * ax + (sl,)]
    return out


@register('slice', aliases=('crop', '_slice'), params={'begin': ('shape', ()), 'end': ('shape', ()), 'step': ('shape', ())})
def slice_op(data, begin=(), end=(), step=()):
    idx = _slice_args(data.shape, begin, end, step)
    return _neg_step_slice(data, idx).contiguous()


@register('slice_axis', params={'axis': ('int', 0), 'begin': ('int', 0), 'end': ('int?', None)})
def slice_axis(data, axis=0, begin=0, end=None):
    axis = axis % data.dim()
    return data[(slice(None),) * axis + (slice(begin, end),)].contiguous()


@register('slice_like', arg_names=('data', 'shape_like'), params={'axes': ('shape', ())})
def slice_like(data, shape_like, axes=()):
    axes = list(axes) if axes else list(range(min(data.dim(), shape_like.dim())))
    idx = [slice(None)] * data.dim()
    for a in axes:
        idx[a % data.dim()] = slice(0, shape_like.shape[a % shape_like.dim()])
    return data[tuple(idx)].contiguous()


@register('_slice_assign', aliases=('_crop_assign',), arg_names=('lhs', 'rhs'),
          params={'begin': ('shape', ()), 'end': ('shape', ()), 'step': ('shape', ())})
def slice_assign(lhs, rhs, begin=(), end=(), step=()):
    out = lhs.clone()
    out[_slice_args(lhs.shape, begin, end, step)] = rhs
    return out


@register('_slice_assign_scalar', aliases=('_crop_assign_scalar',),
          params={'scalar': ('float', 0.0), 'begin': ('shape', ()), 'end': ('shape', ()), 'step': ('shape', ())})
def slice_assign_scalar(data, scalar=0.0, begin=(), end=(), step=()):
    out = data.clone()
    out[_slice_args(data.shape, begin, end, step)] = scalar
    return out


@register('Concat', aliases=('concat',), arg_names=lambda a: ['arg%d' % i for i in range(int(a.get('num_args', 1)))],
          params={'num_args': ('int', 1), 'dim': ('int', 1)}, key_var_num_args='num_args')
def concat(*data, num_args=None, dim=1):
    return torch.cat(data, dim=dim)


@register('_rnn_param_concat', arg_names=lambda a: ['arg%d' % i for i in range(int(a.get('num_args', 1)))],
          params={'num_args': ('int', 1), 'dim': ('int', 0)}, key_var_num_args='num_args')
def rnn_param_concat(*data, num_args=None, dim=0):
    return torch.cat([d.reshape(-1) for d in data], dim=0)


@register('stack', arg_names=lambda a: ['arg%d' % i for i in range(int(a.get('num_args', 1)))],
          params={'num_args': ('int', 1), 'axis': ('int', 0)}, key_var_num_args='num_args')
def stack(*data, num_args=None, axis=0):
    return torch.stack(data, dim=axis)


def _split_nout(a):
    return int(a.get('num_outputs', 1))


@register('SliceChannel', aliases=('split',), num_outputs=_split_nout,
          params={'num_outputs': ('int', 1), 'axis': ('int', 1), 'squeeze_axis': ('bool', False)})
def split(data, num_outputs=1, axis=1, squeeze_axis=False):
    parts = torch.chunk(data, num_outputs, dim=axis)
    if squeeze_axis:
        parts = [p.squeeze(axis) for p in parts]
    return tuple(p.contiguous() for p in parts)


@register('_split_v2', aliases=('split_v2',), num_outputs=lambda a: _nout_v2(a),
          params={'indices': ('shape', ()), 'axis': ('int', 0), 'squeeze_axis': ('bool', False),
                  'sections': ('int', 0), 'indices_or_sections': ('any', None)})
def split_v2(data, indices=(), axis=0, squeeze_axis=False, sections=0, indices_or_sections=None):
    if indices_or_sections is not None:
        if isinstance(indices_or_sections, int):
            sections = indices_or_sections
        else:
            indices = tuple(indices_or_sections)
    if sections:
        parts = torch.chunk(data, sections, dim=axis)
    else:
        idx = [i for i in indices if i != 0] if indices and indices[0] == 0 else list(indices)
        bounds = [0] + idx + [data.shape[axis]]
        parts = [data.narrow(axis, bounds[i], bounds[i + 1] - bounds[i]) for i in range(len(bounds) - 1)]
    if squeeze_axis:
        parts = [p.squeeze(axis) for p in parts]
    return tuple(p.contiguous() for p in parts)


def _nout_v2(a):
    from .registry import _auto_parse
    ios = a.get('indices_or_sections')
    if isinstance(ios, str):
        ios = _auto_parse(ios)
    if ios is not None:
        if isinstance(ios, int):
            return ios
        idx = [i for i in ios if i != 0] if len(ios) and ios[0] == 0 else list(ios)
        return len(idx) + 1
    sec = a.get('sections', 0)
    sec = int(sec) if not isinstance(sec, int) else sec
    if sec:
        return sec
    ind = a.get('indices', ())
    if isinstance(ind, str):
        ind = _auto_parse(ind)
    if isinstance(ind, int):
        ind = (ind,)
    idx = [i for i in ind if i != 0] if len(ind) and ind[0] == 0 else list(ind)
    return len(idx) + 1


@register('repeat', params={'repeats': ('int', 1), 'axis': ('int?', None)})
def repeat(data, repeats=1, axis=None):
    if axis is None:
        return data.reshape(-1).repeat_interleave(repeats)
    return data.repeat_interleave(repeats, dim=axis)


@register('tile', params={'reps': ('shape', ())})
def tile(data, reps=()):
    reps = tuple(int(r) for r in reps)
    from ..util import is_np_shape
    if any(r < 0 for r in reps) or (not is_np_shape() and any(r == 0 for r in reps)):
        # 0 means "unknown" outside numpy shape semantics (reference TileOpShape)
        raise MXNetError('tile: reps must be positive, got %s' % (reps,))
    if len(reps) < data.dim():
        reps = (1,) * (data.dim() - len(reps)) + reps
    return data.repeat(*reps) if len(reps) == data.dim() else data.reshape((1,) * (len(reps) - data.dim()) + tuple(data.shape)).repeat(*reps)


@register('reverse', aliases=('flip',), params={'axis': ('axis', ())})
def reverse(data, axis=()):
    if isinstance(axis, int):
        axis = (axis,)
    return torch.flip(data, dims=list(axis))


@register('depth_to_space', params={'block_size': ('int', 1)})
def depth_to_space(data, block_size=1):
    b = block_size
    if data.dim() != 4 or b <= 0 or data.shape[1] % (b * b) or min(data.shape) == 0:
        raise MXNetError('depth_to_space: need a 4-D input with depth divisible by block_size^2 > 0, got %s '
                         'with block_size %d' % (tuple(data.shape), b))
    n, c, h, w = data.shape
    x = data.reshape(n, b, b, c // (b * b), h, w).permute(0, 3, 4, 1, 5, 2)
    return x.reshape(n, c // (b * b), h * b, w * b)


@register('space_to_depth', params={'block_size': ('int', 1)})
def space_to_depth(data, block_size=1):
    b = block_size
    if data.dim() != 4 or b <= 0 or data.shape[2] % b or data.shape[3] % b or min(data.shape) == 0:
        raise MXNetError('space_to_depth: need a 4-D input whose height and width are divisible by '
                         'block_size > 0, got %s with block_size %d' % (tuple(data.shape), b))
    n, c, h, w = data.shape
    x = data.reshape(n, c, h // b, b, w // b, b).permute(0, 3, 5, 1, 2, 4)
    return x.reshape(n, c * b * b, h // b, w // b)


@register('diag', params={'k': ('int', 0), 'axis1': ('int', 0), 'axis2': ('int', 1)})
def diag(data, k=0, axis1=0, axis2=1):
    if data.dim() >= 2:
        d1, d2 = data.shape[axis1 % data.dim()], data.shape[axis2 % data.dim()]
        if (k > 0 and k >= d2) or (k < 0 and -k >= d1):
            raise MXNetError('diag: k=%d out of range for a %dx%d matrix' % (k, d1, d2))
    if data.dim() == 1:
        return torch.diag(data, k)
    return torch.diagonal(data, offset=k, dim1=axis1, dim2=axis2).contiguous()


@register('where', arg_names=('condition', 'x', 'y'))
def where(condition, x, y):
    if condition.shape != x.shape and condition.dim() == 1:
        condition = condition.reshape((-1,) + (1,) * (x.dim() - 1))
    return torch.where(condition != 0, x, y)


@register('take', arg_names=('a', 'indices'), params={'axis': ('int', 0), 'mode': ('str', 'clip')})
def take(a, indices, axis=0, mode='clip'):
    axis = axis % a.dim()
    n = a.shape[axis]
    idx = indices.to(torch.int64)
    if mode == 'wrap':
        idx = torch.remainder(idx, n)
    elif mode == 'raise':
        if idx.numel() and bool(((idx < 0) | (idx >= n)).any()):
            from ..base import AsyncOpError
            raise AsyncOpError('take: index out of range for axis of size %d (mode=raise)' % n)
        idx = torch.remainder(idx, n)
    else:
        idx = torch.clamp(idx, 0, n - 1)
    out = torch.index_select(a, axis, idx.reshape(-1))
    return out.reshape(a.shape[:axis] + indices.shape + a.shape[axis + 1:])


@register('batch_take', arg_names=('a', 'indices'))
def batch_take(a, indices):
    idx = torch.clamp(indices.to(torch.int64), 0, a.shape[1] - 1)
    return a.gather(1, idx.reshape(-1, 1)).reshape(-1)


@register('one_hot', arg_names=('indices',), params={'depth': ('int', 1), 'on_value': ('float', 1.0),
                                                    'off_value': ('float', 0.0), 'dtype': ('str', 'float32')})
def one_hot(indices, depth=1, on_value=1.0, off_value=0.0, dtype='float32'):
    idx = indices.to(torch.int64)
    if depth == 0:
        return torch.zeros(tuple(idx.shape) + (0,), dtype=torch_dtype(dtype), device=idx.device)
    valid = (idx >= 0) & (idx < depth)
    oh = torch.nn.functional.one_hot(torch.where(valid, idx, torch.zeros_like(idx)), depth)
    oh = oh * valid.unsqueeze(-1)
    dt = torch_dtype(dtype)
    return (oh.to(dt) * (on_value - off_value) + off_value).to(dt)


@register('gather_nd', arg_names=('data', 'indices'))
def gather_nd(data, indices):
    m = indices.shape[0]
    idx = tuple(indices[i].to(torch.int64) for i in range(m))
    return data[idx]


@register('scatter_nd', arg_names=('data', 'indices'), params={'shape': ('shape', ())})
def scatter_nd(data, indices, shape=()):
    out = torch.zeros(shape, dtype=data.dtype, device=data.device)
    m = indices.shape[0]
    idx = tuple(indices[i].to(torch.int64) for i in range(m))
    out[idx] = data
    return out


@register('_scatter_set_nd', arg_names=('lhs', 'rhs', 'indices'), params={'shape': ('shape', ())})
def scatter_set_nd(lhs, rhs, indices, shape=()):
    out = lhs.clone()
    m = indices.shape[0]
    idx = tuple(indices[i].to(torch.int64) for i in range(m))
    out[idx] = rhs
    return out


@register('_backward_gather_nd', arg_names=('data', 'indices'), params={'shape': ('shape', ())})
def backward_gather_nd(data, indices, shape=()):
    out = torch.zeros(shape, dtype=data.dtype, device=data.device)
    m = indices.shape[0]
    idx = tuple(indices[i].to(torch.int64) for i in range(m))
    out.index_put_(idx, data, accumulate=True)
    return out


@register('Pad', aliases=('pad',), params={'mode': ('str', 'constant'), 'pad_width': ('shape', ()),
                                           'constant_value': ('float', 0.0)})
def pad(data, mode='constant', pad_width=(), constant_value=0.0):
    pw = list(pad_width)
    tp = []
    for ax in range(data.dim() - 1, 1, -1):
        tp += [pw[2 * ax], pw[2 * ax + 1]]
    m = {'constant': 'constant', 'edge': 'replicate', 'reflect': 'reflect'}[mode]
    if m == 'constant':
        return torch.nn.functional.pad(data, tp, mode='constant', value=constant_value)
    return torch.nn.functional.pad(data, tp, mode=m)


@register('shape_array')
def shape_array(data):
    return torch.tensor(list(data.shape), dtype=torch.int64, device=data.device)


@register('size_array')
def size_array(data):
    return torch.tensor([data.numel()], dtype=torch.int64, device=data.device)


# ---------------------------------------------------------------------------
# linear algebra
# ---------------------------------------------------------------------------

@register('dot', arg_names=('lhs', 'rhs'), params={'transpose_a': ('bool', False), 'transpose_b': ('bool', False),
                                                    'forward_stype': ('str?', None)})
def dot(lhs, rhs, transpose_a=False, transpose_b=False, forward_stype=None):
    a, b = lhs, rhs
    if a.dim() == 1 and b.dim() == 1:
        return _legacy(torch.dot(a, b))
    if transpose_a:
        a = a.reshape(a.shape[0], -1).t() if a.dim() > 2 else a.t() if a.dim() == 2 else a
    if transpose_b:
        b = b.t() if b.dim() == 2 else b.reshape(-1, b.shape[-1]).t().reshape(b.shape[-1], *b.shape[:-1]) if b.dim() > 2 else b
    if a.shape[-1] != b.shape[0]:
        raise MXNetError('dot: shape mismatch, lhs %s and rhs %s do not share the contracted dimension'
                         % (tuple(lhs.shape), tuple(rhs.shape)))
    return torch.tensordot(a, b, dims=1)


@register('batch_dot', arg_names=('lhs', 'rhs'), params={'transpose_a': ('bool', False), 'transpose_b': ('bool', False),
                                                          'forward_stype': ('str?', None)})
def batch_dot(lhs, rhs, transpose_a=False, transpose_b=False, forward_stype=None):
    a = lhs.transpose(-1, -2) if transpose_a else lhs
    b = rhs.transpose(-1, -2) if transpose_b else rhs
    return torch.matmul(a, b)


@register('khatri_rao', arg_names=lambda a: ['arg%d' % i for i in range(int(a.get('num_args', 1)))],
          params={'num_args': ('int', 1)}, key_var_num_args='num_args')
def khatri_rao(*args, num_args=None):
    out = args[0]
    for m in args[1:]:
        out = (out.unsqueeze(1) * m.unsqueeze(0)).reshape(-1, out.shape[1])
    return out


# ---------------------------------------------------------------------------
# ordering
# ---------------------------------------------------------------------------

@register('sort', params={'axis': ('int?', -1), 'is_ascend': ('bool', True)})
def sort(data, axis=-1, is_ascend=True):
    if axis is None:
        data, axis = data.reshape(-1), 0
    return torch.sort(data, dim=axis, descending=not is_ascend, stable=True)[0]


@register('argsort', params={'axis': ('int?', -1), 'is_ascend': ('bool', True), 'dtype': ('str', 'float32')})
def argsort(data, axis=-1, is_ascend=True, dtype='float32'):
    if axis is None:
        data, axis = data.reshape(-1), 0
    return torch.sort(data, dim=axis, descending=not is_ascend, stable=True)[1].to(torch_dtype(dtype))


def _topk_nout(a):
    r = a.get('ret_typ', 'indices')
    return 2 if r == 'both' else 1


@register('topk', num_outputs=_topk_nout,
          params={'axis': ('int?', -1), 'k': ('int', 1), 'ret_typ': ('str', 'indices'),
                  'is_ascend': ('bool', False), 'dtype': ('str', 'float32')})
def topk(data, axis=-1, k=1, ret_typ='indices', is_ascend=False, dtype='float32'):
    shape = data.shape
    if axis is None:
        data, axis = data.reshape(-1), 0
    if k <= 0:
        k = data.shape[axis]
    v, i = torch.topk(data, k, dim=axis, largest=not is_ascend, sorted=True)
    if ret_typ == 'value':
        return v
    if ret_typ == 'indices':
        return i.to(torch_dtype(dtype))
    if ret_typ == 'mask':
        m = torch.zeros_like(data)
        m.scatter_(axis, i, 1)
        return m.reshape(shape)     # the mask has the input's shape (also for axis=None)
    return v, i.to(torch_dtype(dtype))


@register('_np_cumsum', aliases=('cumsum',), params={'axis': ('int?', None), 'dtype': ('str?', None)})
def cumsum(a, axis=None, dtype=None):
    if axis is None:
        a, axis = a.reshape(-1), 0
    r = torch.cumsum(a, dim=axis)
    return r.to(torch_dtype(dtype)) if dtype else r


@register('_ravel_multi_index', aliases=('ravel_multi_index',), params={'shape': ('shape', ())})
def ravel_multi_index(data, shape=()):
    strides = np.cumprod([1] + list(shape[::-1]))[:-1][::-1]
    st = torch.tensor(strides.copy(), dtype=data.dtype, device=data.device).reshape(-1, *([1] * (data.dim() - 1)))
    return (data * st).sum(0)


@register('_unravel_index', aliases=('unravel_index',), params={'shape': ('shape', ())})
def unravel_index(data, shape=()):
    out = []
    x = data.to(torch.int64)
    for s in reversed(shape[1:]):
        out.append(torch.remainder(x, s))
        x = torch.div(x, s, rounding_mode='floor')
    out.append(x)            # the leading axis takes the quotient (its extent may be -1: unknown)
    return torch.stack(out[::-1]).to(data.dtype)


@register('_histogram', aliases=('histogram',),
          arg_names=lambda a: ['data'] if a.get('bin_cnt') not in (None, 'None') else ['data', 'bins'],
          num_outputs=2,
          params={'bin_cnt': ('int?', None), 'range': ('floats', None)})
def histogram(data, bins=None, bin_cnt=None, range=None):
    if bin_cnt is not None:
        lo, hi = range
        cnt = torch.histc(data.to(torch.float32), bins=bin_cnt, min=lo, max=hi)
        # edges as numpy computes them (exact 0 at the centre of a symmetric range)
        edges = torch.as_tensor(np.linspace(lo, hi, bin_cnt + 1), device=data.device).to(data.dtype)
        return cnt.to(torch.int64), edges
    edges = bins
    idx = torch.bucketize(data, edges, right=True) - 1
    idx = torch.where(data == edges[-1], torch.full_like(idx, len(edges) - 2), idx)
    valid = (idx >= 0) & (idx < len(edges) - 1)
    cnt = torch.bincount(idx[valid], minlength=len(edges) - 1)
    return cnt.to(torch.int64), edges


# ---------------------------------------------------------------------------
# init ops (no tensor inputs)
# ---------------------------------------------------------------------------

def _dev(ctx):
    from ..context import Context
    if ctx is None:
        from ..context import current_context
        ctx = current_context()
    if isinstance(ctx, str):
        from ..context import device
        ctx = device(ctx.replace('(', ':').replace(')', ''))
    return ctx.torch_device if isinstance(ctx, Context) else torch.device(ctx)


_INIT_PARAMS = {'shape': ('shape', ()), 'ctx': ('any', None), 'dtype': ('str', 'float32')}


@register('_zeros', arg_names=(), params=_INIT_PARAMS)
def _zeros(shape=(), ctx=None, dtype='float32'):
    return torch.zeros(shape, dtype=torch_dtype(dtype), device=_dev(ctx))


@register('_ones', arg_names=(), params=_INIT_PARAMS)
def _ones(shape=(), ctx=None, dtype='float32'):
    return torch.ones(shape, dtype=torch_dtype(dtype), device=_dev(ctx))


@register('_full', arg_names=(), params=dict(_INIT_PARAMS, value=('float', 0.0)))
def _full(shape=(), ctx=None, dtype='float32', value=0.0):
    return torch.full(shape, value, dtype=torch_dtype(dtype), device=_dev(ctx))


@register('_arange', arg_names=(), params={'start': ('float', 0.0), 'stop': ('float?', None), 'step': ('float', 1.0),
                                           'repeat': ('int', 1), 'infer_range': ('bool', False),
                                           'ctx': ('any', None), 'dtype': ('str', 'float32')})
def _arange(start=0.0, stop=None, step=1.0, repeat=1, infer_range=False, ctx=None, dtype='float32'):
    if stop is None:
        start, stop = 0.0, start
    td = torch_dtype(dtype)
    n = max(int(math.ceil((stop - start) / step)), 0)
    if td.is_floating_point:
        r = (start + step * torch.arange(n, dtype=torch.float64, device=_dev(ctx))).to(td)
    else:
        # integer ranges as numpy (and the reference kernel) build them: the first two values in the
        # target type fix the step
        first = int(start)
        delta = int(start + step) - first
        r = (first + delta * torch.arange(n, dtype=torch.int64, device=_dev(ctx))).to(td)
    if repeat > 1:
        r = r.repeat_interleave(repeat)
    return r


@register('_linspace', arg_names=(), params={'start': ('float', 0.0), 'stop': ('float', 1.0), 'num': ('int', 50),
                                             'endpoint': ('bool', True), 'ctx': ('any', None), 'dtype': ('str', 'float32')})
def _linspace(start=0.0, stop=1.0, num=50, endpoint=True, ctx=None, dtype='float32'):
    if endpoint:
        r = torch.linspace(start, stop, num, dtype=torch.float64)
    else:
        r = torch.linspace(start, stop, num + 1, dtype=torch.float64)[:-1]
    return r.to(torch_dtype(dtype)).to(_dev(ctx))


@register('_eye', arg_names=(), params={'N': ('int', 1), 'M': ('int', 0), 'k': ('int', 0),
                                        'ctx': ('any', None), 'dtype': ('str', 'float32')})
def _eye(N=1, M=0, k=0, ctx=None, dtype='float32'):
    M = M or N
    out = torch.zeros(N, M, dtype=torch_dtype(dtype), device=_dev(ctx))
    d = torch.diagonal(out, offset=k)
    d.fill_(1)
    return out


@register('_contrib_arange_like', aliases=('arange_like',), params={'start': ('float', 0.0), 'step': ('float', 1.0),
                                                                     'repeat': ('int', 1), 'axis': ('int?', None)})
def arange_like(data, start=0.0, step=1.0, repeat=1, axis=None):
    n = data.numel() if axis is None else data.shape[axis]
    r = (torch.arange(n, device=data.device, dtype=torch.float64) // repeat) * step + start
    r = r.to(data.dtype)
    return r.reshape(data.shape) if axis is None else r


# ---------------------------------------------------------------------------
# misc
# ---------------------------------------------------------------------------

@register('fill_element_0index', arg_names=('lhs', 'mhs', 'rhs'))
def fill_element_0index(lhs, mhs, rhs):
    out = lhs.clone()
    out[torch.arange(lhs.shape[0], device=lhs.device), rhs.to(torch.int64)] = mhs
    return out


@register('_contrib_boolean_mask', aliases=('boolean_mask',), arg_names=('data', 'index'), params={'axis': ('int', 0)})
def boolean_mask(data, index, axis=0):
    return torch.index_select(data, axis, torch.nonzero(index != 0).reshape(-1))


@register('_contrib_index_copy', aliases=('index_copy',), arg_names=('old_tensor', 'index_vector', 'new_tensor'))
def index_copy(old_tensor, index_vector, new_tensor):
    return old_tensor.index_copy(0, index_vector.to(torch.int64), new_tensor)


@register('_contrib_index_array', aliases=('index_array',), params={'axes': ('shape?', None)})
def index_array(data, axes=None):
    if data.dim() == 0:
        return torch.zeros((0,), dtype=torch.int64, device=data.device)
    grids = torch.meshgrid(*[torch.arange(s, device=data.device) for s in data.shape], indexing='ij')
    if axes is not None:
        grids = [grids[a % data.dim()] for a in axes]
    return torch.stack(grids, dim=-1).to(torch.int64)


@register('_contrib_allclose', aliases=('allclose',), arg_names=('a', 'b'),
          params={'rtol': ('float', 1e-5), 'atol': ('float', 1e-8), 'equal_nan': ('bool', True)})
def allclose(a, b, rtol=1e-5, atol=1e-8, equal_nan=True):
    # a 0-d result (reference allclose_op-inl.h: TShape(0, -1))
    return torch.tensor(float(torch.allclose(a, b.to(a.dtype), rtol, atol, equal_nan)), device=a.device)


@register('_contrib_div_sqrt_dim', aliases=('div_sqrt_dim',))
def div_sqrt_dim(data):
    return data / math.sqrt(data.shape[-1])


@register('_contrib_quadratic', aliases=('quadratic',), params={'a': ('float', 0.0), 'b': ('float', 0.0), 'c': ('float', 0.0)})
def quadratic(data, a=0.0, b=0.0, c=0.0):
    return a * data * data + b * data + c


@register('_contrib_getnnz', aliases=('getnnz',), params={'axis': ('int?', None)})
def getnnz(data, axis=None):
    return _legacy((data != 0).sum(dim=axis) if axis is not None else (data != 0).sum()).to(torch.int64)


@register('_contrib_gradientmultiplier', aliases=('gradientmultiplier',), params={'scalar': ('float', 1.0)})
def gradientmultiplier(data, scalar=1.0):
    return _GradMul.apply(data, scalar)


class _GradMul(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, s):
        ctx.s = s
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        return g * ctx.s, None


class _STE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kind):
        return torch.round(x) if kind == 'round' else torch.sign(x)

    @staticmethod
    def backward(ctx, g):
        return g, None


@register('_contrib_round_ste', aliases=('round_ste',))
def round_ste(data):
    return _STE.apply(data, 'round')


@register('_contrib_sign_ste', aliases=('sign_ste',))
def sign_ste(data):
    return _STE.apply(data, 'sign')


@register('_contrib_count_sketch', aliases=('count_sketch',), arg_names=('data', 'h', 's'),
          params={'out_dim': ('int', 1), 'processing_batch_size': ('int', 32)})
def count_sketch(data, h, s, out_dim=1, processing_batch_size=32):
    n = data.shape[0]
    out = torch.zeros(n, out_dim, dtype=data.dtype, device=data.device)
    idx = h.reshape(1, -1).to(torch.int64).expand(n, -1)
    out.scatter_add_(1, idx, data * s.reshape(1, -1))
    return out


@register('_contrib_fft', aliases=('fft',), params={'compute_size': ('int', 128)})
def fft(data, compute_size=128):
    r = torch.fft.fft(data.to(torch.float32), dim=-1)
    return torch.stack([r.real, r.imag], dim=-1).reshape(*data.shape[:-1], data.shape[-1] * 2)


@register('_contrib_ifft', aliases=('ifft',), params={'compute_size': ('int', 128)})
def ifft(data, compute_size=128):
    x = data.reshape(*data.shape[:-1], data.shape[-1] // 2, 2)
    c = torch.complex(x[..., 0].float(), x[..., 1].float())
    return torch.fft.ifft(c, dim=-1).real * c.shape[-1]


@register('_contrib_dgl_adjacency', aliases=('dgl_adjacency',))
def dgl_adjacency(data):
    return (data != 0).to(torch.float32)


@register('_contrib_hawkesll', aliases=('hawkesll',), num_outputs=2,
          arg_names=('lda', 'alpha', 'beta', 'state', 'lags', 'marks', 'valid_length', 'max_time'))
def hawkesll(lda, alpha, beta, state, lags, marks, valid_length, max_time):
    """Log-likelihood of marked Hawkes processes with exponential decay kernels (one sequence per row).

    Semantics of src/operator/contrib/hawkes_ll-inl.h: each mark k keeps its own excitation state
    ``s_k`` and last event time; at an event of mark k after ``d`` time units since that mark's last
    event, ``lambda = mu_k + alpha_k beta_k s_k e^{-beta_k d}`` contributes ``log lambda`` and the
    compensator ``mu_k d + alpha_k s_k (1 - e^{-beta_k d})`` is subtracted, then
    ``s_k <- 1 + s_k e^{-beta_k d}``.  Every mark's remaining compensator up to ``max_time`` closes
    the sequence and the returned states are decayed to ``max_time``.

    All N sequences advance together, one event index per step (rows past their valid length are
    masked), as differentiable tensor ops: autograd gives the exact gradients w.r.t. mu, alpha and
    beta (the reference's hand-written backward) and the initial state."""
    N, T = lags.shape
    K = lda.shape[1]
    dt = lda.dtype
    marks = marks.to(torch.int64)
    vl = valid_length.to(dt)
    rows = torch.arange(N, device=lda.device)
    st = state.to(dt)
    last = torch.zeros(N, K, dtype=dt, device=lda.device)
    t = torch.zeros(N, dtype=dt, device=lda.device)
    ll = torch.zeros(N, dtype=dt, device=lda.device)
    steps = min(T, int(vl.max().item())) if N else 0
    for j in range(steps):
        active = vl > j
        ci = marks[:, j]
        t = t + torch.where(active, lags[:, j].to(dt), torch.zeros_like(t))
        d = t - last[rows, ci]
        b, a = beta[ci], alpha[ci]
        s_c = st[rows, ci]
        mu_c = lda[rows, ci]
        ed = torch.exp(-b * d)
        lam = torch.where(active, mu_c + a * b * s_c * ed, torch.ones_like(mu_c))
        term = torch.log(lam) - (mu_c * d + a * s_c * (1 - ed))
        ll = ll + torch.where(active, term, torch.zeros_like(term))
        hit = torch.nn.functional.one_hot(ci, K).bool() & active[:, None]
        st = torch.where(hit, (1 + s_c * ed)[:, None], st)
        last = torch.where(hit, t[:, None], last)
    d = max_time.to(dt)[:, None] - last
    ed = torch.exp(-beta[None, :] * d)
    ll = ll - (lda * d + alpha[None, :] * st * (1 - ed)).sum(1)
    return ll, ed * st
