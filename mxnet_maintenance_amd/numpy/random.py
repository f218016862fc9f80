"""``mx.np.random`` (parity: python/mxnet/numpy/random.py, src/operator/numpy/random/*).

Samplers draw from torch's generator on the array's device (seeded by
``mx.random.seed`` / ``npx.random.seed``).  uniform / normal / randint are
registered ops and therefore also usable inside hybridized graphs.
"""
import numpy as onp
import torch

from ..context import current_context
from ..ndarray.ndarray import NDArray
from .multiarray import _call, ndarray, _is_scalar

__all__ = ['randint', 'uniform', 'normal', 'lognormal', 'logistic', 'gumbel', 'multinomial', 'multivariate_normal',
           'choice', 'rayleigh', 'rand', 'exponential', 'weibull', 'pareto', 'power', 'shuffle', 'gamma', 'beta',
           'chisquare', 'randn', 'laplace', 'permutation', 'seed']


def seed(s, ctx='all'):
    from .. import random as _r
    _r.seed(s, ctx)


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


def uniform(low=0.0, high=1.0, size=None, dtype=None, ctx=None, out=None):
    if _is_scalar(low) and _is_scalar(high):
        return _call('_npi_uniform', low=float(low), high=float(high), size=_size(size) or (),
                     ctx=ctx or current_context(), dtype=dtype or 'float32', out=out)
    dev = _dev(ctx)
    lo, hi = _t(low, dev), _t(high, dev)
    shp = _bshape(size, low, high)
    return _wrap(torch.rand(shp, device=dev) * (hi - lo) + lo, dtype)


def normal(loc=0.0, scale=1.0, size=None, dtype=None, ctx=None, out=None):
    if _is_scalar(loc) and _is_scalar(scale):
        return _call('_npi_normal', loc=float(loc), scale=float(scale), size=_size(size) or (),
                     ctx=ctx or current_context(), dtype=dtype or 'float32', out=out)
    dev = _dev(ctx)
    mu, sd = _t(loc, dev), _t(scale, dev)
    return _wrap(torch.randn(_bshape(size, loc, scale), device=dev) * sd + mu, dtype)


def randint(low, high=None, size=None, dtype=None, ctx=None, out=None):
    return _call('_npi_random_randint', low=int(low), high=None if high is None else int(high),
                 size=_size(size) or (), ctx=ctx or current_context(), dtype=dtype or 'int64', out=out)


def rand(*size, **kwargs):
    return uniform(size=size, **kwargs)


def randn(*size, **kwargs):
    return normal(size=size, **kwargs)


def lognormal(mean=0.0, sigma=1.0, size=None, dtype=None, ctx=None, out=None):
    return _wrap(torch.exp(normal(mean, sigma, size, None, ctx)._data), dtype)


def logistic(loc=0.0, scale=1.0, size=None, ctx=None, out=None):
    u = uniform(1e-7, 1 - 1e-7, _bshape(size, loc, scale), ctx=ctx)._data
    dev = u.device
    return _wrap(_t(loc, dev) + _t(scale, dev) * torch.log(u / (1 - u)))


def gumbel(loc=0.0, scale=1.0, size=None, ctx=None, out=None):
    u = uniform(1e-7, 1 - 1e-7, _bshape(size, loc, scale), ctx=ctx)._data
    dev = u.device
    return _wrap(_t(loc, dev) - _t(scale, dev) * torch.log(-torch.log(u)))


def laplace(loc=0.0, scale=1.0, size=None, dtype=None, ctx=None, out=None):
    dev = _dev(ctx)
    d = torch.distributions.Laplace(_t(loc, dev), _t(scale, dev))
    return _wrap(d.sample(_bshape(size, loc, scale) if size is not None else ()), dtype)


def exponential(scale=1.0, size=None, ctx=None, out=None):
    dev = _dev(ctx)
    u = torch.rand(_bshape(size, scale), device=dev)
    return _wrap(-torch.log1p(-u) * _t(scale, dev))


def rayleigh(scale=1.0, size=None, ctx=None, out=None):
    dev = _dev(ctx)
    u = torch.rand(_bshape(size, scale), device=dev)
    return _wrap(_t(scale, dev) * torch.sqrt(-2.0 * torch.log1p(-u)))


def weibull(a, size=None, ctx=None, out=None):
    dev = _dev(ctx)
    u = torch.rand(_bshape(size, a), device=dev)
    return _wrap(torch.pow(-torch.log1p(-u), 1.0 / _t(a, dev)))


def pareto(a, size=None, ctx=None, out=None):
    dev = _dev(ctx)
    u = torch.rand(_bshape(size, a), device=dev)
    return _wrap(torch.pow(1 - u, -1.0 / _t(a, dev)) - 1)


def power(a, size=None, ctx=None, out=None):
    dev = _dev(ctx)
    u = torch.rand(_bshape(size, a), device=dev)
    return _wrap(torch.pow(u, 1.0 / _t(a, dev)))


def gamma(shape=1.0, scale=1.0, size=None, dtype=None, ctx=None, out=None):
    dev = _dev(ctx)
    k, th = _t(shape, dev), _t(scale, dev)
    shp = _bshape(size, shape, scale)
    d = torch.distributions.Gamma(k.expand(shp) if k.dim() or shp else k, torch.ones((), device=dev))
    return _wrap(d.sample() * th, dtype)


def beta(a, b, size=None, dtype=None, ctx=None):
    dev = _dev(ctx)
    shp = _bshape(size, a, b)
    d = torch.distributions.Beta(_t(a, dev).expand(shp), _t(b, dev).expand(shp))
    return _wrap(d.sample(), dtype)


def chisquare(df, size=None, dtype=None, ctx=None):
    return _wrap(gamma(_t(df, _dev(ctx)) / 2 if isinstance(df, NDArray) else df / 2.0, 2.0, size, None, ctx)._data,
                 dtype)


def multinomial(n, pvals, size=None):
    p = torch.as_tensor(pvals.asnumpy() if isinstance(pvals, NDArray) else onp.asarray(pvals), dtype=torch.float64)
    shp = _size(size) or ()
    cnt = int(onp.prod(shp)) if shp else 1
    draws = torch.multinomial(p.expand(cnt, -1), n, replacement=True)
    counts = torch.zeros(cnt, p.numel(), dtype=torch.int64).scatter_add_(1, draws, torch.ones_like(draws))
    return ndarray(counts.reshape(tuple(shp) + (p.numel(),)))


def multivariate_normal(mean, cov, size=None, check_valid=None, tol=None):
    dev = mean.context.torch_device if isinstance(mean, NDArray) else torch.device('cpu')
    m, c = _t(mean, dev).float(), _t(cov, dev).float()
    d = torch.distributions.MultivariateNormal(m, covariance_matrix=c)
    return ndarray(d.sample(_size(size) or ()))


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
