"""Host-side NumPy fallbacks (parity: python/mxnet/numpy/fallback.py, fallback_linalg.py).

Like the reference, operators without a device implementation run through
official NumPy on the host: inputs are copied out, the NumPy function runs,
array results come back as ``mx.np.ndarray`` on the first input's context.
They are not differentiable.
"""
import functools

import numpy as onp

from ..ndarray.ndarray import NDArray

_NAMES = ['allclose', 'alltrue', 'apply_along_axis', 'apply_over_axes', 'argpartition', 'argwhere', 'array_equal',
          'array_equiv', 'choose', 'compress', 'corrcoef', 'correlate', 'count_nonzero', 'cov', 'digitize', 'divmod',
          'extract', 'flatnonzero', 'float_power', 'frexp', 'heaviside', 'histogram2d', 'histogram_bin_edges',
          'histogramdd', 'i0', 'in1d', 'interp', 'intersect1d', 'isclose', 'isin', 'ix_', 'lexsort',
          'min_scalar_type', 'modf', 'msort', 'nanargmax', 'nanargmin', 'nancumprod', 'nancumsum', 'nanmax',
          'nanmedian', 'nanmin', 'nanpercentile', 'nanprod', 'nanquantile', 'ndim', 'partition', 'piecewise',
          'packbits', 'poly', 'polyadd', 'polydiv', 'polyfit', 'polyint', 'polymul', 'polysub', 'positive',
          'promote_types', 'ptp', 'real', 'result_type', 'rollaxis', 'roots', 'searchsorted', 'select', 'setdiff1d',
          'setxor1d', 'signbit', 'size', 'spacing', 'take_along_axis', 'trapz', 'tril_indices_from', 'trim_zeros',
          'triu_indices_from', 'union1d', 'unpackbits', 'unwrap', 'vander']
# host fallbacks here that the reference implements as device operators (not part of its fallback list)
_ALSO_HOST = ['nansum', 'nanmean', 'nanstd', 'nanvar', 'convolve', 'gradient', 'sinc', 'angle', 'conj', 'imag',
              'iscomplex', 'isreal', 'fliplr', 'flipud']
_LINALG = ['cond', 'lstsq', 'matrix_power', 'matrix_rank', 'multi_dot', 'qr']
__all__ = list(_NAMES)


def _ctx_of(args):
    for a in args:
        if isinstance(a, NDArray):
            return a.context
        if isinstance(a, (list, tuple)):
            c = _ctx_of(a)
            if c is not None:
                return c
    return None


def _to_host(x):
    if isinstance(x, NDArray):
        return x.asnumpy()
    if isinstance(x, (list, tuple)):
        return type(x)(_to_host(v) for v in x)
    return x


def _to_dev(x, ctx):
    from .multiarray import array
    if isinstance(x, onp.ndarray):
        return array(x, dtype=x.dtype, ctx=ctx)
    if isinstance(x, tuple):
        return tuple(_to_dev(v, ctx) for v in x)
    if isinstance(x, list):
        return [_to_dev(v, ctx) for v in x]
    return x


def make(fn, name):
    @functools.wraps(fn)
    def f(*args, **kwargs):
        ctx = _ctx_of(args) or _ctx_of(list(kwargs.values()))
        res = fn(*_to_host(args), **{k: _to_host(v) for k, v in kwargs.items()})
        return _to_dev(res, ctx)
    f.__name__ = name
    f.__doc__ = 'Host NumPy fallback of ``numpy.%s`` (not differentiable).\n\n' % name + (fn.__doc__ or '')[:400]
    return f


def install(namespace, names=tuple(_NAMES) + tuple(_ALSO_HOST), mod=onp):
    for n in names:
        if n not in namespace and hasattr(mod, n):
            namespace[n] = make(getattr(mod, n), n)
