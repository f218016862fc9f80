"""Random sampling (mx.nd.random).

Parity: python/mxnet/ndarray/random.py and src/operator/random/*.cc
(sample_op, multisample_op, sample_multinomial_op, shuffle_op).  Sampling runs
on the device's torch generator (Philox on HIP).
"""
import numpy as np
import torch

from ..base import torch_dtype, numeric_types
from ..context import current_context
from .ndarray import NDArray

__all__ = ['uniform', 'normal', 'randn', 'randint', 'exponential', 'gamma', 'poisson',
           'negative_binomial', 'generalized_negative_binomial', 'multinomial', 'shuffle',
           'bernoulli', 'uniform_like', 'normal_like', 'categorical']


def _shape(shape):
    if shape is None or shape == ():
        return (1,)
    if isinstance(shape, int):
        return (shape,)
    return tuple(shape)


def _dev(ctx):
    return (ctx or current_context()).torch_device


def _out(t, out):
    if out is not None:
        out._data.copy_(t.reshape(out.shape))
        r = out
    else:
        r = NDArray(t)
    from .. import engine
    box = engine.rng_failure()      # an earlier sampler failed on the shared random resource
    if box is not None:
        r._exc = box
    return r


def _param(p, dev):
    return p._data.to(dev) if isinstance(p, NDArray) else p


def uniform(low=0, high=1, shape=None, dtype=None, ctx=None, out=None, **kwargs):
    if isinstance(low, NDArray) or isinstance(high, NDArray):
        lo = low._data if isinstance(low, NDArray) else torch.tensor(low)
        hi = high._data if isinstance(high, NDArray) else torch.tensor(high)
        s = _shape(shape) if shape else ()
        base = torch.rand(tuple(lo.shape) + s, device=lo.device, dtype=lo.dtype if lo.is_floating_point() else torch.float32)
        lo = lo.reshape(tuple(lo.shape) + (1,) * len(s))
        hi = hi.reshape(tuple(hi.shape) + (1,) * len(s))
        return _out(lo + (hi - lo) * base, out)
    if high < low:
        return _deferred_failure('Check failed: low <= high (uniform sampler: low=%s high=%s)' % (low, high), shape,
                                 dtype, ctx, out)
    dev = _dev(ctx) if out is None else out._data.device
    s = _shape(shape) if out is None else out.shape
    dt = torch_dtype(dtype) if dtype is not None else (out._data.dtype if out is not None else torch.float32)
    t = torch.empty(s, dtype=dt, device=dev).uniform_(low, high)
    return _out(t, out)


def _deferred_failure(msg, shape, dtype, ctx, out):
    """A sampler whose parameter check failed inside the operator: the failure is deferred to the
    next sync point (reference: CHECKs in the sampler kernels run on the engine's workers)."""
    from .. import engine
    from ..base import AsyncOpError
    dev = _dev(ctx) if out is None else out._data.device
    s = _shape(shape) if out is None else out.shape
    dt = torch_dtype(dtype) if dtype is not None else torch.float32
    box = engine.rng_failure() or engine.record_failure(AsyncOpError(msg))
    engine.set_rng_failure(box)
    r = _out(torch.zeros(s, dtype=dt, device=dev), out)
    r._exc = box
    return r


def normal(loc=0, scale=1, shape=None, dtype=None, ctx=None, out=None, **kwargs):
    if isinstance(loc, NDArray) or isinstance(scale, NDArray):
        mu = loc._data if isinstance(loc, NDArray) else torch.tensor(loc)
        sd = scale._data if isinstance(scale, NDArray) else torch.tensor(scale)
        s = _shape(shape) if shape else ()
        base = torch.randn(tuple(mu.shape) + s, device=mu.device, dtype=mu.dtype)
        mu = mu.reshape(tuple(mu.shape) + (1,) * len(s))
        sd = sd.reshape(tuple(sd.shape) + (1,) * len(s))
        return _out(mu + sd * base, out)
    if scale < 0:
        return _deferred_failure('Check failed: scale >= 0 (normal sampler: scale=%s)' % scale, shape, dtype, ctx,
                                 out)
    dev = _dev(ctx) if out is None else out._data.device
    s = _shape(shape) if out is None else out.shape
    dt = torch_dtype(dtype) if dtype is not None else (out._data.dtype if out is not None else torch.float32)
    t = torch.empty(s, dtype=dt, device=dev).normal_(loc, scale)
    return _out(t, out)


def randn(*shape, **kwargs):
    loc = kwargs.pop('loc', 0)
    scale = kwargs.pop('scale', 1)
    return normal(loc, scale, shape or None, **kwargs)


def randint(low, high, shape=None, dtype=None, ctx=None, out=None, **kwargs):
    dt = torch_dtype(dtype or 'int32')
    t = torch.randint(int(low), int(high), _shape(shape), dtype=dt, device=_dev(ctx))
    return _out(t, out)


def exponential(scale=1, shape=None, dtype=None, ctx=None, out=None, **kwargs):
    if isinstance(scale, NDArray):
        s = _shape(shape) if shape else ()
        lam = scale._data.reshape(tuple(scale.shape) + (1,) * len(s))
        e = torch.empty(tuple(scale.shape) + s, device=lam.device, dtype=lam.dtype).exponential_(1.0)
        return _out(e * lam, out)
    t = torch.empty(_shape(shape), dtype=torch_dtype(dtype), device=_dev(ctx)).exponential_(1.0 / scale)
    return _out(t, out)


def gamma(alpha=1, beta=1, shape=None, dtype=None, ctx=None, out=None, **kwargs):
    if isinstance(alpha, NDArray) or isinstance(beta, NDArray):
        a = alpha._data if isinstance(alpha, NDArray) else torch.tensor(float(alpha))
        b = beta._data if isinstance(beta, NDArray) else torch.tensor(float(beta))
        s = _shape(shape) if shape else ()
        a = a.reshape(tuple(a.shape) + (1,) * len(s)).expand(tuple(a.shape) + s)
        b = b.reshape(tuple(b.shape) + (1,) * len(s)).expand(tuple(b.shape) + s)
        return _out(torch.distributions.Gamma(a.float(), 1.0 / b.float()).sample(), out)
    dev = _dev(ctx)
    a = torch.full(_shape(shape), float(alpha), device=dev)
    t = torch._standard_gamma(a) * beta
    return _out(t.to(torch_dtype(dtype)), out)


def poisson(lam=1, shape=None, dtype=None, ctx=None, out=None, **kwargs):
    if isinstance(lam, NDArray):
        s = _shape(shape) if shape else ()
        l = lam._data.reshape(tuple(lam.shape) + (1,) * len(s)).expand(tuple(lam.shape) + s)
        return _out(torch.poisson(l.float()).to(lam._data.dtype), out)
    t = torch.poisson(torch.full(_shape(shape), float(lam), device=_dev(ctx)))
    return _out(t.to(torch_dtype(dtype)), out)


def _per_element(params, shape, dev):
    """Parameters as float tensors of shape param.shape + shape (array parameters draw ``shape``
    samples per element, the reference's _sample_* semantics) plus the output dtype they imply."""
    arrs = [q for q in params if isinstance(q, NDArray)]
    s = _shape(shape) if shape else ()
    if not arrs:
        return [torch.full(_shape(shape), float(q), device=dev) for q in params], None
    base = tuple(arrs[0].shape)
    out = []
    for q in params:
        if isinstance(q, NDArray):
            t = q._data.float().reshape(base + (1,) * len(s)).expand(base + s)
        else:
            t = torch.full(base + s, float(q), device=arrs[0]._data.device)
        out.append(t)
    return out, arrs[0]._data.dtype


def negative_binomial(k=1, p=1, shape=None, dtype=None, ctx=None, out=None, **kwargs):
    (kt, pt), pdt = _per_element([k, p], shape, _dev(ctx))
    g = torch._standard_gamma(kt) * ((1 - pt) / pt)
    return _out(torch.poisson(g).to(pdt or torch_dtype(dtype)), out)


def generalized_negative_binomial(mu=1, alpha=1, shape=None, dtype=None, ctx=None, out=None, **kwargs):
    (mt, at), pdt = _per_element([mu, alpha], shape, _dev(ctx))
    safe = torch.where(at > 0, at, torch.ones_like(at))
    g = torch.where(at > 0, torch._standard_gamma(1.0 / safe) * (mt * safe), mt)
    return _out(torch.poisson(g).to(pdt or torch_dtype(dtype)), out)


def multinomial(data, shape=None, get_prob=False, out=None, dtype='int32', **kwargs):
    p = data._data.float()
    n = int(np.prod(_shape(shape))) if shape else 1
    flat = p.reshape(-1, p.shape[-1])
    if flat.shape[-1] > 2 ** 24:
        from ..base import MXNetError
        raise MXNetError('multinomial: %d categories exceed 2^24 (not exactly representable as float32 indices)'
                         % flat.shape[-1])
    idx = torch.multinomial(flat, n, replacement=True)
    oshape = tuple(p.shape[:-1]) + (_shape(shape) if shape else ())
    idx = idx.reshape(oshape if oshape else (1,))
    res = NDArray(idx.to(torch_dtype(dtype)))
    if get_prob:
        # log-probability of each draw; under autograd its gradient flows to ``data``
        # (d log p_y / d p_y = 1 / p_y, the reference's SampleMultinomialBackward)
        from .. import _state
        rec = bool(_state.STATE.recording)
        with torch.set_grad_enabled(rec):
            src = data._data.reshape(-1, data._data.shape[-1])
            lp = torch.log(torch.gather(src.float(), 1, idx.reshape(flat.shape[0], -1).to(torch.int64)))
            prob = NDArray(lp.reshape(idx.shape).to(data._data.dtype))
        if rec:
            from .register import _note_leaves
            _note_leaves([data])          # grad_req 'write' resets data's gradient buffer first
            prob._recorded = True
        return [res, prob]
    return res


categorical = multinomial


def shuffle(data, **kwargs):
    perm = torch.randperm(data.shape[0], device=data._data.device)
    return NDArray(data._data[perm])


def bernoulli(prob=None, logit=None, size=None, dtype=None, ctx=None, out=None):
    if prob is None:
        prob = torch.sigmoid(logit._data if isinstance(logit, NDArray) else torch.tensor(logit))
    else:
        prob = prob._data if isinstance(prob, NDArray) else torch.full(_shape(size), float(prob), device=_dev(ctx))
    t = torch.bernoulli(prob.float())
    return _out(t.to(torch_dtype(dtype)), out)


def uniform_like(data, low=0, high=1, **kwargs):
    return NDArray(torch.empty_like(data._data).uniform_(low, high))


def _like_op(opname, params):
    def f(data=None, *args, **kwargs):
        from .register import invoke_by_name
        kw = dict(zip(params, args))
        kw.update(kwargs)
        return invoke_by_name(opname, [data], kw)
    f.__name__ = opname[len('_random_'):]
    return f


gamma_like = _like_op('_random_gamma_like', ['alpha', 'beta'])
exponential_like = _like_op('_random_exponential_like', ['lam'])
poisson_like = _like_op('_random_poisson_like', ['lam'])
negative_binomial_like = _like_op('_random_negative_binomial_like', ['k', 'p'])
generalized_negative_binomial_like = _like_op('_random_generalized_negative_binomial_like', ['mu', 'alpha'])


def normal_like(data, loc=0, scale=1, **kwargs):
    return NDArray(torch.empty_like(data._data).normal_(loc, scale))
