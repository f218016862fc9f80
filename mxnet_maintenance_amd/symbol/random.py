"""Symbolic random sampling (mx.sym.random).  Parity: python/mxnet/symbol/random.py."""
from .symbol import _op_func, Symbol


def _dispatch(scalar_op, tensor_op, params):
    def f(*args, shape=None, dtype=None, name=None, **kwargs):
        vals = dict(zip(params, args))
        vals.update({k: v for k, v in kwargs.items() if k in params})
        if any(isinstance(v, Symbol) for v in vals.values()):
            extra = {'dtype': dtype} if dtype is not None else {}
            return _op_func(tensor_op)(*[vals[p] for p in params], shape=shape or (), name=name, **extra)
        kw = {k: v for k, v in vals.items()}
        kw['shape'] = shape or ()
        if dtype is not None:
            kw['dtype'] = dtype
        return _op_func(scalar_op)(name=name, **kw)
    return f


uniform = _dispatch('_random_uniform', '_sample_uniform', ['low', 'high'])
normal = _dispatch('_random_normal', '_sample_normal', ['loc', 'scale'])
gamma = _dispatch('_random_gamma', '_sample_gamma', ['alpha', 'beta'])
_exponential_lam = _dispatch('_random_exponential', '_sample_exponential', ['lam'])


def exponential(scale=1, shape=None, dtype=None, name=None, **kwargs):
    """Exponential samples with mean ``scale`` (rate 1 / scale), as mx.nd.random.exponential."""
    lam = kwargs.pop('lam', None)
    if lam is None:
        lam = (1.0 / scale) if not isinstance(scale, Symbol) else 1.0 / scale
    return _exponential_lam(lam, shape=shape, dtype=dtype, name=name)
poisson = _dispatch('_random_poisson', '_sample_poisson', ['lam'])
negative_binomial = _dispatch('_random_negative_binomial', '_sample_negative_binomial', ['k', 'p'])
generalized_negative_binomial = _dispatch('_random_generalized_negative_binomial',
                                          '_sample_generalized_negative_binomial', ['mu', 'alpha'])
randint = _dispatch('_random_randint', '_random_randint', ['low', 'high'])


def _like(opname, params):
    def f(data=None, *args, name=None, **kwargs):
        kw = dict(zip(params, args))
        kw.update({k: v for k, v in kwargs.items() if k in params})
        return _op_func(opname)(data, name=name, **kw)
    f.__name__ = opname[len('_random_'):]
    return f


uniform_like = _like('_random_uniform_like', ['low', 'high'])
normal_like = _like('_random_normal_like', ['loc', 'scale'])
gamma_like = _like('_random_gamma_like', ['alpha', 'beta'])
exponential_like = _like('_random_exponential_like', ['lam'])
poisson_like = _like('_random_poisson_like', ['lam'])
negative_binomial_like = _like('_random_negative_binomial_like', ['k', 'p'])
generalized_negative_binomial_like = _like('_random_generalized_negative_binomial_like', ['mu', 'alpha'])


def randn(*shape, loc=0, scale=1, dtype=None, name=None, **kwargs):
    """Normal samples of the given shape (positional dimensions, like numpy.random.randn)."""
    if 'shape' in kwargs:
        shape = kwargs.pop('shape')
    if isinstance(kwargs.get('data'), Symbol):
        # sample with the shape of a symbol (the reference forwards ``data`` to the sampler)
        out = _op_func('_random_normal_like')(kwargs['data'], loc=loc, scale=scale, name=name)
        return out if dtype is None else _op_func('Cast')(out, dtype=dtype)
    return normal(loc, scale, shape=tuple(shape) if shape else (), dtype=dtype, name=name)


def multinomial(data, shape=None, get_prob=False, dtype='int32', name=None):
    return _op_func('_sample_multinomial')(data, shape=shape or (), get_prob=get_prob, dtype=dtype, name=name)


def shuffle(data, name=None):
    return _op_func('_shuffle')(data, name=name)
