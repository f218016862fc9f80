"""``mx.sym.np`` / ``F.np`` for Symbols: the mx.np functions in graph-building mode.

Parity: python/mxnet/symbol/numpy/_symbol.py.  The functions are the same
objects as ``mx.np.*``; calling them through this namespace forces graph
construction even for input-less ops (``F.np.zeros``)."""
import functools
import types

from . import multiarray as _ma


class _SymNamespace(types.ModuleType):
    def __init__(self, name, mod):
        super().__init__(name)
        self._mod = mod

    def __getattr__(self, item):
        obj = getattr(self._mod, item)
        if isinstance(obj, types.ModuleType):
            ns = _SymNamespace(self.__name__ + '.' + item, obj)
            setattr(self, item, ns)
            return ns
        if not callable(obj) or isinstance(obj, type):
            return obj

        @functools.wraps(obj)
        def f(*args, **kwargs):
            prev = _ma._FORCE_SYM[0]
            _ma._FORCE_SYM[0] = True
            try:
                return obj(*args, **kwargs)
            finally:
                _ma._FORCE_SYM[0] = prev
        setattr(self, item, f)
        return f


def make():
    from .. import numpy as np_mod
    return _SymNamespace('mxnet.symbol.numpy', np_mod)
