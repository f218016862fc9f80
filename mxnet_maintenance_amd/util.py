"""Misc utilities: numpy-semantics switches, env helpers (parity: python/mxnet/util.py)."""
import functools
import os

from . import _state

__all__ = ['is_np_shape', 'is_np_array', 'set_np_shape', 'set_np', 'reset_np', 'use_np', 'use_np_shape',
           'use_np_array', 'np_shape', 'np_array', 'getenv', 'setenv', 'makedirs', 'get_gpu_count',
           'get_gpu_memory', 'set_module', 'wrap_np_unary_func', 'wrap_np_binary_func', 'default_array',
           'get_cuda_compute_capability', 'set_flush_denorms']


def makedirs(d):
    os.makedirs(os.path.expanduser(d), exist_ok=True)


def get_gpu_count():
    import torch
    return torch.cuda.device_count()


def get_gpu_memory(gpu_dev_id):
    import torch
    free, total = torch.cuda.mem_get_info(gpu_dev_id)
    return free, total


def get_cuda_compute_capability(ctx):
    """Return the gfx architecture number of an AMD device (950 for MI355X)."""
    return 950


def getenv(name):
    return os.environ.get(name)


def setenv(name, value):
    if value is None:
        os.environ.pop(name, None)
    else:
        os.environ[name] = str(value)


# flush-to-zero / denormals-are-zero for CPU float math (reference util.py:852; on by default there)
_FLUSH_DENORMS = [True]


def set_flush_denorms(value):
    """Enable / disable flushing of denormal CPU floats to zero; returns the previous state."""
    import torch
    prev = _FLUSH_DENORMS[0]
    if torch.set_flush_denormal(bool(value)) or not value:
        _FLUSH_DENORMS[0] = bool(value)
    return prev


def is_np_shape():
    return _state.STATE.np_shape


def is_np_array():
    return _state.STATE.np_array


def set_np_shape(active):
    prev = _state.STATE.np_shape
    _state.STATE.np_shape = bool(active)
    return prev


def set_np(shape=True, array=True, dtype=False):
    _state.STATE.np_shape = bool(shape)
    _state.STATE.np_array = bool(array)


def reset_np():
    set_np(False, False)


class _NumpyShapeScope:
    def __init__(self, active):
        self._enter = active
        self._prev = None

    def __enter__(self):
        self._prev = set_np_shape(self._enter)
        return self

    def __exit__(self, *a):
        set_np_shape(self._prev)


class _NumpyArrayScopeMeta(type):
    """``_NumpyArrayScope._current``: the calling thread's NumPy-array mode as a scope object
    (assigning one switches this thread's mode; reference util.py keeps it in a threading.local)."""

    @property
    def _current(cls):
        return cls(_state.STATE.np_array)

    @_current.setter
    def _current(cls, scope):
        _state.STATE.np_array = bool(scope._is_np_array)


class _NumpyArrayScope(metaclass=_NumpyArrayScopeMeta):
    """``with np_array(flag):`` -- NumPy-compatible array semantics in this thread."""

    def __init__(self, is_np_array):
        self._is_np_array = bool(is_np_array)
        self._prev = None

    def __enter__(self):
        self._prev = _state.STATE.np_array
        _state.STATE.np_array = self._is_np_array
        return self

    def __exit__(self, *a):
        _state.STATE.np_array = self._prev


def np_shape(active=True):
    return _NumpyShapeScope(active)


def np_array(active=True):
    return _NumpyArrayScope(active)


def _wrap_class(cls, scope):
    """Run every method of ``cls`` (and its inherited ``__call__`` / ``forward``, where a Block turns
    results into arrays) inside ``scope()`` -- the class form of the use_np decorators."""
    import inspect
    names = [n for n, v in vars(cls).items() if inspect.isfunction(v)]
    for extra in ('__call__', 'forward'):
        if extra not in names and callable(getattr(cls, extra, None)):
            names.append(extra)
    for n in names:
        meth = getattr(cls, n)

        def make(meth):
            @functools.wraps(meth)
            def f(*a, **k):
                with scope():
                    return meth(*a, **k)
            return f
        setattr(cls, n, make(meth))
    return cls


def use_np_shape(func):
    if isinstance(func, type):
        return _wrap_class(func, lambda: np_shape(True))

    @functools.wraps(func)
    def f(*a, **k):
        with np_shape(True):
            return func(*a, **k)
    return f


def use_np_array(func):
    if isinstance(func, type):
        return _wrap_class(func, lambda: np_array(True))

    @functools.wraps(func)
    def f(*a, **k):
        with np_array(True):
            return func(*a, **k)
    return f


def use_np(func):
    return use_np_shape(use_np_array(func))


def set_module(module):
    def deco(func):
        if module is not None:
            func.__module__ = module
        return func
    return deco


def wrap_np_unary_func(func):
    return func


def wrap_np_binary_func(func):
    return func


def default_array(source_array, ctx=None, dtype=None):
    from .ndarray import array
    return array(source_array, ctx=ctx, dtype=dtype)
