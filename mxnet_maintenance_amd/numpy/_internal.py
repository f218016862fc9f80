"""``mx.np._internal``: the NumPy-interface backend operators by their short names.

Parity: python/mxnet/ndarray/numpy/_internal.py -- ``_internal.<name>`` invokes the registered
operator ``_npi_<name>`` (or ``_np_<name>``) imperatively, or builds a graph node for Symbols.
"""
from ..ops import registry as _registry
from .multiarray import _call


def boolean_mask_assign_scalar(data, mask, value, start_axis=0, out=None):
    """``data[mask] = value`` with ``mask`` spanning the axes from ``start_axis``; written into
    ``out`` when given (the reference's in-place form ``out=data``)."""
    return _call('_npi_boolean_mask_assign_scalar', data, mask, value=float(value), start_axis=start_axis, out=out)


def boolean_mask_assign_tensor(data, mask, value, start_axis=0, out=None):
    """``data[mask] = value`` for an array ``value`` broadcast over the selected positions."""
    return _call('_npi_boolean_mask_assign_tensor', data, mask, value, start_axis=start_axis, out=out)


def __getattr__(name):
    for op in ('_npi_' + name, '_np_' + name):
        if _registry.has(op):
            def f(*args, _op=op, **kwargs):
                return _call(_op, *args, **kwargs)
            f.__name__ = name
            return f
    raise AttributeError("module 'mx.np._internal' has no attribute '%s'" % name)
