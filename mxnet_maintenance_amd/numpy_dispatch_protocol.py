"""NumPy dispatch protocols for mx.np arrays (NEP-18 ``__array_function__``, NEP-13 ``__array_ufunc__``).

Parity: python/mxnet/numpy_dispatch_protocol.py (the operator lists :80-300 and the registration
:143 / :280).  Importing the package registers every official NumPy function below whose mx.np
counterpart exists, so ``numpy.sum(mx.np.array(...))`` runs mx.np.sum on the array's device and
returns an mx.np array; unregistered functions fall back to a host round trip (refused while
autograd records).  ``with_array_function_protocol`` / ``with_array_ufunc_protocol`` are the
test decorators of the reference.
"""
import functools

import numpy as _onp

from . import numpy as _mx_np
from .numpy.multiarray import _NUMPY_ARRAY_FUNCTION_DICT, _NUMPY_ARRAY_UFUNC_DICT

__all__ = ['with_array_function_protocol', 'with_array_ufunc_protocol', 'registered_functions']

# functions with an mx.np implementation dispatched through __array_function__
_NUMPY_ARRAY_FUNCTION_LIST = '''
all any sometrue argmin argmax around round round_ argsort sort append broadcast_arrays broadcast_to clip
concatenate copy cumsum diag diagonal diagflat dot expand_dims fix flip flipud fliplr inner insert max amax
mean min amin nonzero ones_like atleast_1d atleast_2d atleast_3d prod product ravel repeat reshape roll
split array_split hsplit vsplit dsplit squeeze stack std sum swapaxes take tensordot tile transpose unique
unravel_index diag_indices_from delete var vdot vstack column_stack hstack dstack zeros_like linalg.norm
linalg.cholesky linalg.inv linalg.solve linalg.tensorinv linalg.tensorsolve linalg.pinv linalg.eigvals
linalg.eig linalg.eigvalsh linalg.eigh shape trace tril meshgrid outer einsum polyval shares_memory
may_share_memory quantile percentile diff ediff1d resize where full_like bincount empty_like nan_to_num
isnan isfinite isposinf isneginf isinf pad
'''.split()

# ufuncs dispatched through __array_ufunc__
_NUMPY_ARRAY_UFUNC_LIST = '''
abs fabs add arctan2 copysign degrees hypot lcm subtract multiply true_divide negative power mod matmul
absolute rint sign exp log log2 log10 expm1 sqrt square cbrt reciprocal invert bitwise_not remainder sin
cos tan sinh cosh tanh arcsin arccos arctan arcsinh arccosh arctanh maximum minimum ceil trunc floor
bitwise_and bitwise_xor bitwise_or logical_not equal not_equal less less_equal greater greater_equal
'''.split()

_MISSING = []


def _lookup(root, dotted):
    obj = root
    for part in dotted.split('.'):
        obj = getattr(obj, part, None)
        if obj is None:
            return None
    return obj


def _register():
    if len(set(_NUMPY_ARRAY_FUNCTION_LIST)) != len(_NUMPY_ARRAY_FUNCTION_LIST) or len(set(_NUMPY_ARRAY_UFUNC_LIST)) != len(_NUMPY_ARRAY_UFUNC_LIST):
        raise ValueError('duplicate operator name in the dispatch lists')
    for name in _NUMPY_ARRAY_FUNCTION_LIST:
        official, ours = _lookup(_onp, name), _lookup(_mx_np, name)
        if official is None or ours is None:
            _MISSING.append(name)
            continue
        _NUMPY_ARRAY_FUNCTION_DICT[official] = ours
    for name in _NUMPY_ARRAY_UFUNC_LIST:
        ours = getattr(_mx_np, name, None)
        if ours is None:
            _MISSING.append(name)
            continue
        _NUMPY_ARRAY_UFUNC_DICT[name] = ours


def registered_functions():
    """Names of the NumPy functions / ufuncs that dispatch to mx.np (the rest run on the host)."""
    return sorted(getattr(f, '__name__', str(f)) for f in _NUMPY_ARRAY_FUNCTION_DICT) + sorted(
        _NUMPY_ARRAY_UFUNC_DICT)


def _protocol_runner(label):
    def decorate(func):
        @functools.wraps(func)
        def run(*args, **kwargs):
            try:
                func(*args, **kwargs)
            except Exception as err:  # pylint: disable=broad-except
                raise RuntimeError('Running function {} with NumPy array {} protocol failed with exception {}'
                                   .format(func.__name__, label, err))
        return run
    return decorate


with_array_function_protocol = _protocol_runner('function')
with_array_ufunc_protocol = _protocol_runner('ufunc')

_register()
