"""Weight initializers.

Parity: python/mxnet/initializer.py (InitDesc, Initializer with name-suffix
dispatch, register/create, Load, Mixed, Zero, One, Constant, Uniform, Normal,
Orthogonal, Xavier, MSRAPrelu, Bilinear, LSTMBias, FusedRNN).
Initialisation runs on the array's device (torch RNG on HIP for gpu arrays).
"""
import json
import logging
import re
import warnings

import numpy as np
import torch

from .base import string_types, MXNetError

__all__ = ['InitDesc', 'Initializer', 'register', 'create', 'Load', 'Mixed', 'Zero', 'One', 'Constant',
           'Uniform', 'Normal', 'Orthogonal', 'Xavier', 'MSRAPrelu', 'Bilinear', 'LSTMBias', 'FusedRNN']

_INIT_REGISTRY = {}


def register(klass):
    """Register an initializer class under its lower-case name."""
    _INIT_REGISTRY[klass.__name__.lower()] = klass
    return klass


def alias(*aliases):
    def reg(klass):
        for a in aliases:
            _INIT_REGISTRY[a.lower()] = klass
        return klass
    return reg


def create(init, **kwargs):
    if isinstance(init, Initializer):
        return init
    if isinstance(init, string_types):
        if init.startswith('['):
            name, kw = json.loads(init)
            return _INIT_REGISTRY[name.lower()](**kw)
        return _INIT_REGISTRY[init.lower()](**kwargs)
    raise ValueError('Cannot create initializer from %s' % str(init))


class InitDesc(str):
    """Parameter name with attributes (global_init and attrs such as __init__)."""

    def __new__(cls, name, attrs=None, global_init=None):
        ret = super().__new__(cls, name)
        ret.attrs = attrs or {}
        ret.global_init = global_init
        return ret


class Initializer:
    """Base initializer: dispatches on the parameter-name suffix."""

    def __init__(self, **kwargs):
        self._kwargs = kwargs
        self._verbose = False
        self._print_func = None

    def set_verbosity(self, verbose=False, print_func=None):
        self._verbose = verbose
        self._print_func = print_func or (lambda x: str(float((x.norm() / np.sqrt(x.size)).asscalar()))
                                          if hasattr(x, 'norm') else '')
        return self

    def _verbose_print(self, desc, init, arr):
        if self._verbose and self._print_func:
            logging.info('Initialized %s as %s: %s', desc, init, self._print_func(arr))

    def dumps(self):
        return json.dumps([self.__class__.__name__.lower(), self._kwargs])

    def __call__(self, desc, arr):
        if not isinstance(desc, InitDesc):
            self._legacy_init(desc, arr)
            return
        if desc.global_init is None:
            desc.global_init = self
        init = desc.attrs.get('__init__', '')
        if init:
            create(init)._init_weight(desc, arr)
            self._verbose_print(desc, init, arr)
            return
        if desc.endswith('weight'):
            self._init_weight(desc, arr)
            self._verbose_print(desc, 'weight', arr)
        elif desc.endswith('bias'):
            self._init_bias(desc, arr)
            self._verbose_print(desc, 'bias', arr)
        elif desc.endswith('gamma'):
            self._init_gamma(desc, arr)
        elif desc.endswith('beta'):
            self._init_beta(desc, arr)
        elif desc.endswith('min'):
            self._init_zero(desc, arr)
        elif desc.endswith('max'):
            self._init_one(desc, arr)
        elif desc.endswith('moving_mean') or desc.endswith('running_mean'):
            self._init_zero(desc, arr)
        elif desc.endswith('moving_var') or desc.endswith('running_var'):
            self._init_one(desc, arr)
        elif desc.endswith('moving_inv_var'):
            self._init_zero(desc, arr)
        elif desc.endswith('moving_avg'):
            self._init_zero(desc, arr)
        else:
            self._init_default(desc, arr)

    def _legacy_init(self, name, arr):
        warnings.warn('Calling initializer with init(str, NDArray) has been deprecated. '
                      'please use init(mx.init.InitDesc(...), NDArray) instead.', DeprecationWarning)
        self.__call__(InitDesc(name), arr)

    # --- helpers that write into an NDArray -----------------------------------
    @staticmethod
    def _set(arr, t):
        with torch.no_grad():
            arr._data.copy_(t.to(arr._data.dtype).reshape(arr._data.shape))

    def _init_bilinear(self, _, arr):
        shape = arr.shape
        weight = np.zeros(int(np.prod(shape)), dtype='float32')
        f = np.ceil(shape[3] / 2.)
        c = (2 * f - 1 - f % 2) / (2. * f)
        for i in range(int(np.prod(shape))):
            x = i % shape[3]
            y = (i // shape[3]) % shape[2]
            weight[i] = (1 - abs(x / f - c)) * (1 - abs(y / f - c))
        self._set(arr, torch.from_numpy(weight))

    def _init_loc_bias(self, _, arr):
        assert arr.shape[0] == 6
        self._set(arr, torch.tensor([1.0, 0, 0, 0, 1.0, 0]))

    def _init_zero(self, _, arr):
        with torch.no_grad():
            arr._data.zero_()

    def _init_one(self, _, arr):
        with torch.no_grad():
            arr._data.fill_(1.0)

    def _init_bias(self, _, arr):
        self._init_zero(_, arr)

    def _init_gamma(self, _, arr):
        self._init_one(_, arr)

    def _init_beta(self, _, arr):
        self._init_zero(_, arr)

    def _init_weight(self, name, arr):
        raise NotImplementedError('Must override it')

    def _init_default(self, name, _):
        raise ValueError('Unknown initialization pattern for %s. Default initialization is now limited to '
                         '"weight", "bias", "gamma" (1.0), and "beta" (0.0).' % name)

    def __eq__(self, other):
        return isinstance(other, Initializer) and self.dumps() == other.dumps()

    def __hash__(self):
        return hash(self.dumps())


class Load:
    """Initialize from a dict of arrays (or a .params file), falling back to ``default_init``."""

    def __init__(self, param, default_init=None, verbose=False):
        from . import ndarray as nd
        if isinstance(param, str):
            param = nd.load(param)
        assert isinstance(param, dict)
        self.param = {}
        for name, arr in param.items():
            if name.startswith('arg:') or name.startswith('aux:'):
                self.param[name[4:]] = arr
            else:
                self.param[name] = arr
        self.default_init = default_init
        self.verbose = verbose

    def __call__(self, name, arr):
        if name in self.param:
            assert arr.shape == self.param[name].shape, \
                'Parameter %s cannot be initialized from loading. Shape mismatch, target %s vs loaded %s' % (
                    name, str(arr.shape), self.param[name].shape)
            Initializer._set(arr, self.param[name]._data)
        else:
            assert self.default_init is not None, \
                'Cannot Initialize %s. Not found in loaded param and no default Initializer is provided.' % name
            self.default_init(name, arr)


class Mixed:
    """Pick an initializer by the first regex pattern that matches the name."""

    def __init__(self, patterns, initializers):
        assert len(patterns) == len(initializers)
        self.map = list(zip([re.compile(p) for p in patterns], initializers))

    def __call__(self, name, arr):
        for prog, init in self.map:
            if prog.match(name):
                init(name, arr)
                return
        raise ValueError('Parameter name %s did not match any pattern. Consider add a ".*" pattern at the '
                         'and with default Initializer.' % name)


@register
@alias('zeros')
class Zero(Initializer):
    def __init__(self):
        super().__init__()

    def _init_weight(self, _, arr):
        self._init_zero(_, arr)

    _init_default = _init_weight


@register
@alias('ones')
class One(Initializer):
    def __init__(self):
        super().__init__()

    def _init_weight(self, _, arr):
        self._init_one(_, arr)

    _init_default = _init_weight


@register
class Constant(Initializer):
    def __init__(self, value):
        super().__init__(value=value)
        self.value = value

    def _init_weight(self, _, arr):
        from .ndarray.ndarray import NDArray
        if isinstance(self.value, NDArray):
            self._set(arr, self.value._data)
        elif isinstance(self.value, (list, tuple, np.ndarray)):
            self._set(arr, torch.as_tensor(np.asarray(self.value, dtype=np.float32)))
        else:
            with torch.no_grad():
                arr._data.fill_(self.value)

    _init_default = _init_weight

    def dumps(self):
        val = self._kwargs['value']
        if not np.isscalar(val):
            self._kwargs['value'] = val.tolist() if isinstance(val, np.ndarray) else (
                val.asnumpy().tolist() if hasattr(val, 'asnumpy') else val)
        return json.dumps([self.__class__.__name__.lower(), self._kwargs])


@register
class Uniform(Initializer):
    def __init__(self, scale=0.07):
        super().__init__(scale=scale)
        self.scale = scale

    def _init_weight(self, _, arr):
        with torch.no_grad():
            arr._data.uniform_(-self.scale, self.scale)


@register
class Normal(Initializer):
    def __init__(self, sigma=0.01):
        super().__init__(sigma=sigma)
        self.sigma = sigma

    def _init_weight(self, _, arr):
        with torch.no_grad():
            arr._data.normal_(0, self.sigma)


@register
class Orthogonal(Initializer):
    def __init__(self, scale=1.414, rand_type='uniform'):
        super().__init__(scale=scale, rand_type=rand_type)
        self.scale = scale
        self.rand_type = rand_type

    def _init_weight(self, _, arr):
        nout = arr.shape[0]
        nin = int(np.prod(arr.shape[1:]))
        if self.rand_type == 'uniform':
            tmp = np.random.uniform(-1.0, 1.0, (nout, nin))
        else:
            tmp = np.random.normal(0.0, 1.0, (nout, nin))
        u, _, v = np.linalg.svd(tmp, full_matrices=False)
        res = u if u.shape == tmp.shape else v
        self._set(arr, torch.from_numpy((self.scale * res).astype(np.float32)))


@register
class Xavier(Initializer):
    """Xavier/Glorot initialisation (rnd_type uniform|gaussian, factor_type avg|in|out)."""

    def __init__(self, rnd_type='uniform', factor_type='avg', magnitude=3):
        super().__init__(rnd_type=rnd_type, factor_type=factor_type, magnitude=magnitude)
        self.rnd_type = rnd_type
        self.factor_type = factor_type
        self.magnitude = float(magnitude)

    def _init_weight(self, name, arr):
        shape = arr.shape
        hw_scale = 1.
        if len(shape) < 2:
            raise ValueError('Xavier initializer cannot be applied to vector {0}. It requires at least 2D.'
                             .format(name))
        if len(shape) > 2:
            hw_scale = np.prod(shape[2:])
        fan_in, fan_out = shape[1] * hw_scale, shape[0] * hw_scale
        factor = 1.
        if self.factor_type == 'avg':
            factor = (fan_in + fan_out) / 2.0
        elif self.factor_type == 'in':
            factor = fan_in
        elif self.factor_type == 'out':
            factor = fan_out
        else:
            raise ValueError('Incorrect factor type')
        scale = np.sqrt(self.magnitude / factor)
        with torch.no_grad():
            if self.rnd_type == 'uniform':
                arr._data.uniform_(-scale, scale)
            elif self.rnd_type == 'gaussian':
                arr._data.normal_(0, scale)
            else:
                raise ValueError('Unknown random type')


@register
class MSRAPrelu(Xavier):
    def __init__(self, factor_type='avg', slope=0.25):
        magnitude = 2. / (1 + slope ** 2)
        super().__init__('gaussian', factor_type, magnitude)
        self._kwargs = {'factor_type': factor_type, 'slope': slope}


@register
class Bilinear(Initializer):
    def __init__(self):
        super().__init__()

    def _init_weight(self, _, arr):
        self._init_bilinear(_, arr)


@register
class LSTMBias(Initializer):
    """Zero biases except the forget gate (set to ``forget_bias``)."""

    def __init__(self, forget_bias=1.0):
        super().__init__(forget_bias=forget_bias)
        self.forget_bias = forget_bias

    def _init_weight(self, name, arr):
        with torch.no_grad():
            arr._data.zero_()
            num_hidden = int(arr.shape[0] / 4)
            arr._data[num_hidden:2 * num_hidden] = self.forget_bias


@register
class FusedRNN(Initializer):
    """Initialise the flat parameter vector of a fused RNN layer piece by piece."""

    def __init__(self, init, num_hidden, num_layers, mode, bidirectional=False, forget_bias=1.0):
        if isinstance(init, string_types):
            init = create(init)
        super().__init__(init=init.dumps() if init is not None else None, num_hidden=num_hidden,
                         num_layers=num_layers, mode=mode, bidirectional=bidirectional,
                         forget_bias=forget_bias)
        self._init = init
        self._num_hidden = num_hidden
        self._num_layers = num_layers
        self._mode = mode
        self._bidirectional = bidirectional
        self._forget_bias = forget_bias

    def _init_weight(self, desc, arr):
        from .ops.nn import _GATES
        from .ndarray.ndarray import NDArray
        g = _GATES[self._mode]
        d = 2 if self._bidirectional else 1
        h = self._num_hidden
        total = arr.shape[0]
        # solve input size from total parameter count
        per_rest = 0
        for layer in range(1, self._num_layers):
            per_rest += d * (g * h * h * d + g * h * h + 2 * g * h)
        first = total - per_rest
        ni = (first // d - g * h * h - 2 * g * h) // (g * h)
        off = 0
        # FusedRNN(None, ...): the pieces take the global initializer (the reference's desc.global_init)
        sub = self._init if self._init is not None else (getattr(desc, 'global_init', None) or Uniform())
        with torch.no_grad():
            for layer in range(self._num_layers):
                nin = ni if layer == 0 else h * d
                for _ in range(d):
                    for n in (g * h * nin, g * h * h):
                        piece = NDArray(arr._data[off:off + n].view(g * h, -1))
                        sub._init_weight(InitDesc('weight'), piece)
                        off += n
            for layer in range(self._num_layers):
                for _ in range(d):
                    for _k in range(2):
                        b = arr._data[off:off + g * h]
                        b.zero_()
                        if self._mode == 'lstm':
                            b[h:2 * h] = self._forget_bias / 2.0
                        off += g * h
