"""Parameter initializers (mx.init).

Behavioural parity with python/mxnet/initializer.py: InitDesc (:35), Initializer with its
name-suffix dispatch (:60-200), register/alias/create (:210), Load (:250), Mixed (:300), Zero,
One, Constant, Uniform, Normal, Orthogonal, Xavier, MSRAPrelu, Bilinear, LSTMBias and FusedRNN
(:330-760).

Random draws run where the array lives (torch's generator on the HIP device for GPU
parameters), so initialising a large model never round-trips through the host; the few
deterministic patterns (bilinear upsampling kernels, orthogonal bases) are computed in numpy
and copied once.
"""
import json
import logging
import re
import warnings

import numpy as np
import torch

from .base import string_types

__all__ = ['InitDesc', 'Initializer', 'register', 'create', 'Load', 'Mixed', 'Zero', 'One', 'Constant',
           'Uniform', 'Normal', 'Orthogonal', 'Xavier', 'MSRAPrelu', 'Bilinear', 'LSTMBias', 'FusedRNN']

_REGISTRY = {}


def register(klass):
    """Class decorator: make ``klass`` creatable by its lower-case name (``mx.init.create``)."""
    _REGISTRY[klass.__name__.lower()] = klass
    return klass


def alias(*aliases):
    """Class decorator: extra registry names for an initializer."""
    def add(klass):
        _REGISTRY.update({name.lower(): klass for name in aliases})
        return klass
    return add


def create(init, **kwargs):
    """An initializer from an instance, a registered name, or a ``dumps()`` JSON string."""
    if isinstance(init, Initializer):
        return init
    if not isinstance(init, string_types):
        raise ValueError('Cannot create initializer from %s' % str(init))
    if init.startswith('['):
        name, params = json.loads(init)
        return _REGISTRY[name.lower()](**params)
    return _REGISTRY[init.lower()](**kwargs)


class InitDesc(str):
    """A parameter name carrying its symbol attributes (``attrs``, e.g. ``__init__``) and the
    initializer that the whole model was initialised with (``global_init``)."""

    def __new__(cls, name, attrs=None, global_init=None):
        desc = super().__new__(cls, name)
        desc.attrs = attrs or {}
        desc.global_init = global_init
        return desc


# ------------------------------------------------------------------------- array writers
def _write(arr, values):
    """Copy ``values`` (tensor / array-like, any dtype) into NDArray ``arr`` in place."""
    src = values if isinstance(values, torch.Tensor) else torch.as_tensor(np.asarray(values, dtype=np.float32))
    with torch.no_grad():
        arr._data.copy_(src.to(arr._data.dtype).reshape(arr._data.shape))


def _fill(arr, value):
    with torch.no_grad():
        arr._data.fill_(value)


def _uniform(arr, bound):
    with torch.no_grad():
        arr._data.uniform_(-bound, bound)


def _gaussian(arr, sigma):
    with torch.no_grad():
        arr._data.normal_(0, sigma)


def _bilinear_kernel(shape):
    """Bilinear-upsampling deconvolution weights: a separable tent over the last two axes."""
    kh, kw = shape[2], shape[3]
    f = np.ceil(kw / 2.0)
    centre = (2 * f - 1 - f % 2) / (2.0 * f)
    tent_x = 1 - np.abs(np.arange(kw) / f - centre)
    tent_y = 1 - np.abs(np.arange(kh) / f - centre)
    return np.broadcast_to(np.outer(tent_y, tent_x), shape).astype(np.float32)


# name suffix -> the default-pattern hook that initialises it (first match wins; order matters:
# 'moving_inv_var' must not fall into 'var', '...weight' is checked before everything else)
_SUFFIX_HOOKS = (
    ('weight', '_init_weight'), ('bias', '_init_bias'), ('gamma', '_init_gamma'), ('beta', '_init_beta'),
    ('min', '_init_zero'), ('max', '_init_one'),
    ('moving_mean', '_init_zero'), ('running_mean', '_init_zero'),
    ('moving_var', '_init_one'), ('running_var', '_init_one'),
    ('moving_inv_var', '_init_zero'), ('moving_avg', '_init_zero'),
)
_VERBOSE_SUFFIXES = ('weight', 'bias')


class Initializer:
    """Base class.  Calling ``init(InitDesc(name), arr)`` initialises ``arr`` by the parameter's
    ``__init__`` attribute if it has one, otherwise by its name suffix (weight -> ``_init_weight``,
    bias/beta -> 0, gamma -> 1, running statistics -> 0 / 1)."""

    def __init__(self, **kwargs):
        self._kwargs = kwargs
        self._verbose = False
        self._print_func = None

    def set_verbosity(self, verbose=False, print_func=None):
        """Log every initialised array through ``print_func(arr)`` (default: its RMS)."""
        def rms(x):
            return str(float((x.norm() / np.sqrt(x.size)).asscalar())) if hasattr(x, 'norm') else ''
        self._verbose = verbose
        self._print_func = print_func or rms
        return self

    def _verbose_print(self, desc, init, arr):
        if self._verbose and self._print_func:
            logging.info('Initialized %s as %s: %s', desc, init, self._print_func(arr))

    def dumps(self):
        """``[name, kwargs]`` JSON: ``create(init.dumps())`` rebuilds the initializer."""
        return json.dumps([type(self).__name__.lower(), self._kwargs])

    def __call__(self, desc, arr):
        if not isinstance(desc, InitDesc):
            warnings.warn('Calling initializer with init(str, NDArray) has been deprecated. '
                          'please use init(mx.init.InitDesc(...), NDArray) instead.', DeprecationWarning)
            desc = InitDesc(desc)
        if desc.global_init is None:
            desc.global_init = self
        explicit = desc.attrs.get('__init__', '')
        if explicit:
            create(explicit)._init_weight(desc, arr)
            self._verbose_print(desc, explicit, arr)
            return
        for suffix, hook in _SUFFIX_HOOKS:
            if desc.endswith(suffix):
                getattr(self, hook)(desc, arr)
                if suffix in _VERBOSE_SUFFIXES:
                    self._verbose_print(desc, suffix, arr)
                return
        self._init_default(desc, arr)

    def _legacy_init(self, name, arr):
        self(name, arr)

    # default patterns --------------------------------------------------------
    _set = staticmethod(_write)

    def _init_bilinear(self, _, arr):
        _write(arr, _bilinear_kernel(tuple(arr.shape)))

    def _init_loc_bias(self, _, arr):
        assert arr.shape[0] == 6
        _write(arr, [1.0, 0, 0, 0, 1.0, 0])          # identity affine transform

    def _init_zero(self, _, arr):
        _fill(arr, 0.0)

    def _init_one(self, _, arr):
        _fill(arr, 1.0)

    _init_bias = _init_zero
    _init_beta = _init_zero
    _init_gamma = _init_one

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
    """Initialise from saved arrays (a dict or a ``.params`` file; ``arg:``/``aux:`` prefixes are
    dropped), deferring unknown names to ``default_init``."""

    def __init__(self, param, default_init=None, verbose=False):
        if isinstance(param, str):
            from . import ndarray as nd
            param = nd.load(param)
        assert isinstance(param, dict)
        self.param = {(k[4:] if k[:4] in ('arg:', 'aux:') else k): v for k, v in param.items()}
        self.default_init = default_init
        self.verbose = verbose

    def __call__(self, name, arr):
        saved = self.param.get(name)
        if saved is None:
            assert self.default_init is not None, \
                'Cannot Initialize %s. Not found in loaded param and no default Initializer is provided.' % name
            self.default_init(name, arr)
            return
        assert arr.shape == saved.shape, \
            'Parameter %s cannot be initialized from loading. Shape mismatch, target %s vs loaded %s' % (
                name, str(arr.shape), saved.shape)
        _write(arr, saved._data)
        if self.verbose:
            logging.info('Initialized %s by loading', name)


class Mixed:
    """Route each parameter to the initializer of the first regex in ``patterns`` it matches."""

    def __init__(self, patterns, initializers):
        assert len(patterns) == len(initializers)
        self.map = [(re.compile(p), init) for p, init in zip(patterns, initializers)]

    def __call__(self, name, arr):
        for regex, init in self.map:
            if regex.match(name):
                init(name, arr)
                return
        raise ValueError('Parameter name %s did not match any pattern. Consider add a ".*" pattern at the '
                         'and with default Initializer.' % name)


@register
@alias('zeros')
class Zero(Initializer):
    """Everything (any name) to 0."""

    def __init__(self):
        super().__init__()

    def _init_weight(self, _, arr):
        _fill(arr, 0.0)

    _init_default = _init_weight


@register
@alias('ones')
class One(Initializer):
    """Everything (any name) to 1."""

    def __init__(self):
        super().__init__()

    def _init_weight(self, _, arr):
        _fill(arr, 1.0)

    _init_default = _init_weight


@register
class Constant(Initializer):
    """Everything to ``value`` (a scalar, or an array broadcast-copied into the parameter)."""

    def __init__(self, value):
        super().__init__(value=value)
        self.value = value

    def _init_weight(self, _, arr):
        val = self.value
        if np.isscalar(val):
            _fill(arr, val)
        else:
            _write(arr, val._data if hasattr(val, '_data') else val)

    _init_default = _init_weight

    def dumps(self):
        val = self._kwargs['value']
        if not np.isscalar(val):
            host = val.asnumpy() if hasattr(val, 'asnumpy') else np.asarray(val)
            self._kwargs['value'] = host.tolist()
        return super().dumps()


@register
class Uniform(Initializer):
    """Weights ~ U(-scale, scale)."""

    def __init__(self, scale=0.07):
        super().__init__(scale=scale)
        self.scale = scale

    def _init_weight(self, _, arr):
        _uniform(arr, self.scale)


@register
class Normal(Initializer):
    """Weights ~ N(0, sigma^2)."""

    def __init__(self, sigma=0.01):
        super().__init__(sigma=sigma)
        self.sigma = sigma

    def _init_weight(self, _, arr):
        _gaussian(arr, self.sigma)


@register
class Orthogonal(Initializer):
    """Weights = ``scale`` x an orthonormal basis (Saxe et al. 2013) from the SVD of a random
    (fan_out, fan_in) matrix."""

    def __init__(self, scale=1.414, rand_type='uniform'):
        super().__init__(scale=scale, rand_type=rand_type)
        self.scale = scale
        self.rand_type = rand_type

    def _init_weight(self, _, arr):
        rows, cols = arr.shape[0], int(np.prod(arr.shape[1:]))
        draw = np.random.uniform(-1.0, 1.0, (rows, cols)) if self.rand_type == 'uniform' \
            else np.random.normal(0.0, 1.0, (rows, cols))
        left, _sv, right = np.linalg.svd(draw, full_matrices=False)
        basis = left if left.shape == draw.shape else right
        _write(arr, (self.scale * basis).astype(np.float32))


_FAN_CHOICES = {'avg': lambda fin, fout: (fin + fout) / 2.0, 'in': lambda fin, fout: fin,
                'out': lambda fin, fout: fout}


@register
class Xavier(Initializer):
    """Glorot / Xavier: variance ``magnitude / fan`` with fan = mean (``avg``), ``in`` or ``out``
    of the receptive-field-scaled fan-in / fan-out; ``rnd_type`` uniform or gaussian."""

    def __init__(self, rnd_type='uniform', factor_type='avg', magnitude=3):
        super().__init__(rnd_type=rnd_type, factor_type=factor_type, magnitude=magnitude)
        self.rnd_type = rnd_type
        self.factor_type = factor_type
        self.magnitude = float(magnitude)

    def _init_weight(self, name, arr):
        shape = arr.shape
        if len(shape) < 2:
            raise ValueError('Xavier initializer cannot be applied to vector {0}. It requires at least 2D.'
                             .format(name))
        field = float(np.prod(shape[2:])) if len(shape) > 2 else 1.0
        if self.factor_type not in _FAN_CHOICES:
            raise ValueError('Incorrect factor type')
        fan = _FAN_CHOICES[self.factor_type](shape[1] * field, shape[0] * field)
        spread = np.sqrt(self.magnitude / fan)
        if self.rnd_type == 'uniform':
            _uniform(arr, spread)
        elif self.rnd_type == 'gaussian':
            _gaussian(arr, spread)
        else:
            raise ValueError('Unknown random type')


@register
class MSRAPrelu(Xavier):
    """He et al. 2015 initialisation for PReLU nets: gaussian Xavier with magnitude 2/(1+slope^2)."""

    def __init__(self, factor_type='avg', slope=0.25):
        super().__init__('gaussian', factor_type, 2.0 / (1 + slope ** 2))
        self._kwargs = {'factor_type': factor_type, 'slope': slope}


@register
class Bilinear(Initializer):
    """Bilinear-upsampling kernels for deconvolution weights."""

    def __init__(self):
        super().__init__()

    def _init_weight(self, _, arr):
        self._init_bilinear(_, arr)


@register
class LSTMBias(Initializer):
    """LSTM biases: 0 except the forget-gate block (gate order i, f, c, o) set to ``forget_bias``."""

    def __init__(self, forget_bias=1.0):
        super().__init__(forget_bias=forget_bias)
        self.forget_bias = forget_bias

    def _init_weight(self, name, arr):
        hidden = int(arr.shape[0] / 4)
        with torch.no_grad():
            arr._data.zero_()
            arr._data[hidden:2 * hidden] = self.forget_bias


@register
class FusedRNN(Initializer):
    """Initialise a fused RNN layer's flat parameter vector.

    The vector holds, per layer and direction, ``W_x`` (gates*H, in) and ``W_h`` (gates*H, H),
    followed by all biases (``b_x``, ``b_h`` per layer and direction).  Each weight block goes
    through ``init`` (or the model's global initializer), biases are zero with LSTM forget gates
    at ``forget_bias`` split across the two bias vectors.
    """

    def __init__(self, init, num_hidden, num_layers, mode, bidirectional=False, forget_bias=1.0):
        if isinstance(init, string_types):
            init = create(init)
        super().__init__(init=None if init is None else init.dumps(), num_hidden=num_hidden,
                         num_layers=num_layers, mode=mode, bidirectional=bidirectional, forget_bias=forget_bias)
        self._init = init
        self._num_hidden = num_hidden
        self._num_layers = num_layers
        self._mode = mode
        self._bidirectional = bidirectional
        self._forget_bias = forget_bias

    def _blocks(self, total):
        """(offset, rows, cols) of every weight block, then (offset, length) of every bias."""
        from .ops.nn import _GATES
        gates, hid, dirs = _GATES[self._mode], self._num_hidden, 2 if self._bidirectional else 1
        rows = gates * hid
        deep = (self._num_layers - 1) * dirs * (rows * hid * dirs + rows * hid + 2 * rows)
        in0 = ((total - deep) // dirs - rows * hid - 2 * rows) // rows   # solve the input width
        weights, pos = [], 0
        for layer in range(self._num_layers):
            width = in0 if layer == 0 else hid * dirs
            for _ in range(dirs):
                for cols in (width, hid):
                    weights.append((pos, rows, cols))
                    pos += rows * cols
        biases = [(pos + k * rows, rows) for k in range(2 * dirs * self._num_layers)]
        return weights, biases

    def _init_weight(self, desc, arr):
        from .ndarray.ndarray import NDArray
        weights, biases = self._blocks(arr.shape[0])
        # FusedRNN(None, ...): blocks take the model's global initializer (reference desc.global_init)
        inner = self._init if self._init is not None else (getattr(desc, 'global_init', None) or Uniform())
        flat = arr._data
        with torch.no_grad():
            for pos, rows, cols in weights:
                inner._init_weight(InitDesc('weight'), NDArray(flat[pos:pos + rows * cols].view(rows, cols)))
            hid = self._num_hidden
            for pos, length in biases:
                flat[pos:pos + length].zero_()
                if self._mode == 'lstm':
                    flat[pos + hid:pos + 2 * hid] = self._forget_bias / 2.0
