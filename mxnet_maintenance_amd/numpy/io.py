"""Text I/O for mx.np arrays (reference: python/mxnet/numpy/io.py:28)."""
import numpy as onp

from ..context import current_context
from .multiarray import array

__all__ = ['genfromtxt']


def genfromtxt(*args, **kwargs):
    """``numpy.genfromtxt`` parsed on the host, returned as an mx.np array on ``ctx`` (keyword,
    default: the current context)."""
    ctx = kwargs.pop('ctx', None) or current_context()
    host = onp.genfromtxt(*args, **kwargs)
    return array(host, dtype=host.dtype, ctx=ctx)
