"""``mx.np.random`` (parity: python/mxnet/numpy/random.py, src/operator/numpy/random/*).

Samplers draw from torch's generator on the array's device (seeded by
``mx.random.seed`` / ``npx.random.seed``).  uniform / normal / randint are
registered ops and therefore also usable inside hybridized graphs.
"""
import numpy as onp
import torch

from ..context import current_context
from ..ndarray.ndarray import NDArray
from .multiarray import _call, ndarray, _is_scalar, _host_graph

__all__ = ['randint', 'uniform', 'normal', 'lognormal', 'logistic', 'gumbel', 'multinomial', 'multivariate_normal',
           'choice', 'rayleigh', 'rand', 'exponential', 'weibull', 'pareto', 'power', 'shuffle', 'gamma', 'beta',
           'chisquare', 'randn', 'laplace', 'permutation', 'seed']


def seed(seed=None, ctx='all', **kwargs):  # pylint: disable=redefined-outer-name
    from .. import random as _r
    _r.seed(seed if seed is not None else kwargs.get('s'), ctx)


def _size(size):
    if size is None:
        return None
    return (size,) if isinstance(size, int) else tuple(size)


def _dev(ctx):
    return (ctx or current_context()).torch_device


def _t(x, dev):
    return x._data.to(dev) if isinstance(x, NDArray) else torch.as_tensor(x, dtype=torch.float32, device=dev)


def _bshape(size, *params):
    if size is not None:
        return _size(size)
    shp = ()
    for p in params:
        if isinstance(p, NDArray):
            shp = tuple(torch.broadcast_shapes(shp, tuple(p.shape)))
    return shp


def _wrap(t, dtype=None):
    if dtype is not None:
        from ..base import torch_dtype
        t = t.to(torch_dtype(dtype))
    return ndarray(t)


# parameter positions that must be > 0 (strict) or >= 0, per distribution
_POSITIVE = {'normal': ((1, False),), 'lognormal': ((1, False),), 'logistic': ((1, False),),
             'gumbel': ((1, False),), 'laplace': ((1, False),), 'exponential': ((0, False),),
             'rayleigh': ((0, False),), 'weibull': ((0, True),), 'pareto': ((0, True),), 'power': ((0, True),),
             'gamma': ((0, True), (1, True)), 'beta': ((0, True), (1, True)), 'chisquare': ((0, True),)}


def _check_scalars(kind, params):
    """Scalar parameters are validated in Python, at the call (reference numpy/random.py raises
    ValueError); array parameters are checked inside the operator."""
    for i, strict in _POSITIVE.get(kind, ()):
        p = params[i]
        if _is_scalar(p) and (p <= 0 if strict else p < 0):
            raise ValueError('%s: parameter %d must be %s 0, got %r' % (kind, i, '>' if strict else '>=', p))


def _sample(kind, params, size, dtype=None, ctx=None, out=None, batch=False):
    """Draw from ``kind`` through the registered sampler op (array or Symbol parameters become op
    inputs; scalars ride along as attributes)."""
    from .multiarray import _is_sym
    _check_scalars(kind, params)
    arrays = [p for p in params if isinstance(p, NDArray) or _is_sym(p)]
    pscal = tuple(None if (isinstance(p, NDArray) or _is_sym(p)) else float(p) for p in params)
    kw = dict(kind=kind, pscal=pscal, size=_size(size), dtype=dtype or 'float32', out=out, batch=bool(batch))
    if not arrays:
        kw['ctx'] = ctx or current_context()
    return _call('_npi_sampler', *arrays, **kw)


def uniform(low=0.0, high=1.0, size=None, dtype=None, ctx=None, out=None):
    if _is_scalar(low) and _is_scalar(high):
        return _call('_npi_uniform', low=float(low), high=float(high), size=_size(size) or (),
                     ctx=ctx or current_context(), dtype=dtype or 'float32', out=out)
    return _sample('uniform', (low, high), size, dtype, ctx, out)


def normal(loc=0.0, scale=1.0, size=None, dtype=None, ctx=None, out=None):
    if _is_scalar(loc) and _is_scalar(scale):
        return _call('_npi_normal', loc=float(loc), scale=float(scale), size=_size(size) or (),
                     ctx=ctx or current_context(), dtype=dtype or 'float32', out=out)
    return _sample('normal', (loc, scale), size, dtype, ctx, out)


def randint(low, high=None, size=None, dtype=None, ctx=None, out=None):
    return _call('_npi_random_randint', low=int(low), high=None if high is None else int(high),
                 size=_size(size) or (), ctx=ctx or current_context(), dtype=dtype or 'int64', out=out)


def rand(*size, **kwargs):
    return uniform(size=size, **kwargs)


def randn(*size, **kwargs):
    return normal(size=size, **kwargs)


def lognormal(mean=0.0, sigma=1.0, size=None, dtype=None, ctx=None, out=None):
    return _sample('lognormal', (mean, sigma), size, dtype, ctx, out)


def logistic(loc=0.0, scale=1.0, size=None, ctx=None, out=None):
    return _sample('logistic', (loc, scale), size, None, ctx, out)


def gumbel(loc=0.0, scale=1.0, size=None, ctx=None, out=None):
    return _sample('gumbel', (loc, scale), size, None, ctx, out)


def laplace(loc=0.0, scale=1.0, size=None, dtype=None, ctx=None, out=None):
    return _sample('laplace', (loc, scale), size, dtype, ctx, out)


def exponential(scale=1.0, size=None, ctx=None, out=None):
    return _sample('exponential', (scale,), size, None, ctx, out)


def rayleigh(scale=1.0, size=None, ctx=None, out=None):
    return _sample('rayleigh', (scale,), size, None, ctx, out)


def weibull(a, size=None, ctx=None, out=None):
    return _sample('weibull', (a,), size, None, ctx, out)


def pareto(a, size=None, ctx=None, out=None):
    return _sample('pareto', (a,), size, None, ctx, out)


def power(a, size=None, ctx=None, out=None):
    return _sample('power', (a,), size, None, ctx, out)


def gamma(shape=1.0, scale=1.0, size=None, dtype=None, ctx=None, out=None):
    return _sample('gamma', (shape, scale), size, dtype, ctx, out)


def beta(a, b, size=None, dtype=None, ctx=None):
    return _sample('beta', (a, b), size, dtype, ctx)


def chisquare(df, size=None, dtype=None, ctx=None):
    return _sample('chisquare', (df,), size, dtype, ctx)


def multinomial(n, pvals, size=None):
    p = torch.as_tensor(pvals.asnumpy() if isinstance(pvals, NDArray) else onp.asarray(pvals), dtype=torch.float64)
    shp = _size(size) or ()
    cnt = int(onp.prod(shp)) if shp else 1
    if p.numel() == 0 or cnt == 0:
        return ndarray(torch.zeros(tuple(shp) + (p.numel(),), dtype=torch.int64))
    draws = torch.multinomial(p.expand(cnt, -1), n, replacement=True)
    counts = torch.zeros(cnt, p.numel(), dtype=torch.int64).scatter_add_(1, draws, torch.ones_like(draws))
    return ndarray(counts.reshape(tuple(shp) + (p.numel(),)))


@_host_graph('random_multivariate_normal')
def multivariate_normal(mean, cov, size=None, check_valid=None, tol=None):
    """Samples of shape ``size + broadcast(mean.shape, cov.shape[:-1])`` in the dtype of ``mean``."""
    dev = mean.context.torch_device if isinstance(mean, NDArray) else torch.device('cpu')
    mt = _t(mean, dev)
    m, c = mt.double(), _t(cov, dev).double()
    d = torch.distributions.MultivariateNormal(m, covariance_matrix=c)
    r = d.sample(_size(size) or ())
    return ndarray(r.to(mt.dtype if mt.is_floating_point() else torch.float32))


@_host_graph('random_choice')
def choice(a, size=None, replace=True, p=None, ctx=None, out=None):
    dev = _dev(ctx)
    if isinstance(a, int):
        n, pool = a, None
    else:
        pool = a._data if isinstance(a, NDArray) else torch.as_tensor(onp.asarray(a))
        n = pool.shape[0]
    shp = _size(size) or ()
    cnt = int(onp.prod(shp)) if shp else 1
    if p is None:
        idx = torch.randint(0, n, (cnt,), device=dev) if replace else torch.randperm(n, device=dev)[:cnt]
    else:
        pt = _t(p, dev).float()
        idx = torch.multinomial(pt, cnt, replacement=replace)
    idx = idx.reshape(shp)
    if pool is None:
        return ndarray(idx)
    return ndarray(pool.to(dev)[idx])


def shuffle(x):
    """Shuffle ``x`` in place along its first axis."""
    perm = torch.randperm(x.shape[0], device=x._data.device)
    with torch.no_grad():
        x._data.copy_(x._data[perm])


def permutation(x):
    if isinstance(x, int):
        return ndarray(torch.randperm(x))
    perm = torch.randperm(x.shape[0], device=x._data.device)
    return ndarray(x._data[perm])
