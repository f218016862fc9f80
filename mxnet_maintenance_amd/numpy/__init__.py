"""``mx.np``: NumPy-compatible array interface (parity: python/mxnet/numpy/*).

``mx.np.ndarray`` shares storage, autograd and device placement with the
legacy ``mx.nd.NDArray``; its functions are registered ``_npi_*`` operators
(usable imperatively and in hybridized graphs), with host-NumPy fallbacks for
the long tail (as the reference does in fallback.py).
"""
from . import multiarray
from .multiarray import *  # noqa: F401,F403
from .multiarray import ndarray, _np_out
from . import linalg, random
from . import io
from .io import genfromtxt  # noqa: F401
from . import _internal
from . import fallback as _fallback
from . import fallback
from . import fallback_linalg

_fallback.install(globals())
_fallback.install(linalg.__dict__, _fallback._LINALG, __import__('numpy').linalg)


def save(file, arr):
    """Save an ndarray (or a dict/list of them) in MXNet's ``.params`` container."""
    from ..numpy_extension import save as _s
    _s(file, arr)


def load(file):
    from ..numpy_extension import load as _l
    return _l(file)


def set_module(name):
    def deco(f):
        f.__module__ = name
        return f
    return deco


def __getattr__(name):
    if name == '_Symbol':       # mx.sym.np._Symbol: the Symbol class np-mode graphs are built from
        from ..symbol.symbol import Symbol
        return Symbol
    raise AttributeError("module 'mxnet.numpy' has no attribute '%s'" % name)
