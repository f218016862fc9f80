"""Python signatures for the NumPy-compatible operators.

Parity: python/mxnet/numpy_op_signature.py (``_get_builtin_op``: operator name -> the Python function
behind it).  Operator names follow the reference's convention: ``_np_<name>`` lives in ``mx.np``,
``_np_<sub>_<name>`` in ``mx.np.<sub>`` (linalg, random, fft), ``_npx_<name>`` in ``mx.npx``.  The
functions here are ordinary Python functions, so ``inspect.signature`` already works on them; this
module only provides the name resolution.
"""
import inspect

__all__ = ['_get_builtin_op']

_NP_SUBMODULES = ('linalg', 'random', 'fft')


def _get_builtin_op(op_name):
    from . import numpy as mx_np
    from . import numpy_extension as mx_npx
    if op_name.startswith('_npx_'):
        root, rest, subs = mx_npx, op_name[len('_npx_'):], ()
    elif op_name.startswith('_np_'):
        root, rest, subs = mx_np, op_name[len('_np_'):], _NP_SUBMODULES
    else:
        return None
    module = root
    for sub in subs:
        if rest.startswith(sub + '_'):
            module = getattr(root, sub, None)
            if module is None:
                raise ValueError('Cannot find submodule {} in module {}'.format(sub, root.__name__))
            rest = rest[len(sub) + 1:]
            break
    op = getattr(module, rest, None)
    if op is None:
        raise ValueError('Cannot find operator {} in module {}'.format(rest, module.__name__))
    from . import _numpy_op_doc
    doc = getattr(_numpy_op_doc, op_name, None)
    if doc is not None and getattr(op, '__signature__', None) is None:
        try:
            op.__signature__ = inspect.signature(doc)
        except (AttributeError, TypeError):
            pass
    return op


def _signature(op_name):
    """``inspect.Signature`` of an operator's Python function (None when it has none)."""
    op = _get_builtin_op(op_name)
    try:
        return inspect.signature(op)
    except (TypeError, ValueError):
        return None
