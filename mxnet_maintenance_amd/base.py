"""Basic types, dtype tables and errors.

Parity: python/mxnet/base.py (MXNetError, numeric_types, string_types,
_DTYPE_NP_TO_MX / _DTYPE_MX_TO_NP type-flag tables used by the .params format).
"""
import numbers

import numpy as np
import torch


def data_dir_default():
    """Default directory for downloaded data and models: ``%APPDATA%/mxnet`` on Windows,
    ``~/.mxnet`` elsewhere (reference python/mxnet/base.py:57)."""
    import os
    import platform
    if platform.system() == 'Windows':
        return os.path.join(os.environ.get('APPDATA'), 'mxnet')
    return os.path.join(os.path.expanduser('~'), '.mxnet')


def data_dir():
    """``$MXNET_HOME`` if set, else :func:`data_dir_default`."""
    import os
    return os.getenv('MXNET_HOME', data_dir_default())

__all__ = ['MXNetError', 'numeric_types', 'integer_types', 'string_types', 'py_str', 'mx_real_t', '_as_list',
           'np_dtype', 'torch_dtype', 'dtype_to_flag', 'flag_to_dtype']


class MXNetError(RuntimeError):
    """Error raised by the framework (mirrors mxnet.base.MXNetError)."""


class MXNetIndexError(MXNetError, IndexError):
    """An out-of-bounds index inside an operator: an MXNetError that is also an IndexError (the
    reference maps dmlc's IndexError-typed errors to Python's IndexError)."""


class AsyncOpError(MXNetError):
    """Failure inside an operator's *execution* (not its argument / shape checks).  As with the
    reference's threaded engine, the imperative layer does not raise it at the call: the outputs are
    marked failed and the error surfaces at the next synchronisation point that touches them
    (``wait_to_read`` / ``asnumpy`` / ``mx.nd.waitall``)."""


class MXNetValueError(MXNetError, ValueError):
    """An MXNetError that is also a ValueError (the reference maps C++ errors whose message starts
    with ``ValueError:`` to this Python type)."""


class AsyncValueError(AsyncOpError, ValueError):
    """A deferred operator failure rethrown as a ValueError (invalid parameter values)."""


class NotImplementedForSymbol(MXNetError):
    def __init__(self, function, alias, *args):
        super().__init__()
        self.function = function.__name__ if callable(function) else str(function)
        self.alias = alias
        self.args = [str(type(a)) for a in args]

    def __str__(self):
        msg = 'Function {}'.format(self.function)
        if self.alias:
            msg += ' (namely operator "{}")'.format(self.alias)
        if self.args:
            msg += ' with arguments ({})'.format(', '.join(self.args))
        msg += ' is not implemented for Symbol and only available in NDArray.'
        return msg


numeric_types = (float, int, np.generic, numbers.Number)
integer_types = (int, np.integer)
string_types = (str,)
py_str = lambda x: x.decode('utf-8') if isinstance(x, bytes) else x     # noqa: E731  (bytes from C -> str)
mx_real_t = np.float32                                                  # default real type
mx_uint = np.uint32
mx_int = np.int32


def _as_list(obj):
    """``obj`` if it is a list, else ``[obj]``."""
    return obj if isinstance(obj, list) else [obj]


def check_call(ret):
    """C-API status check of the reference; here native calls raise directly, so only non-zero
    integers are reported."""
    if isinstance(ret, int) and ret != 0:
        raise MXNetError('native call failed with status %d' % ret)

# MXNet type flags (include/mxnet/base.h / mshadow type_flag). These values are
# part of the on-disk .params format, so they must match the reference exactly.
_FLAG_TO_NP = {
    0: np.float32, 1: np.float64, 2: np.float16, 3: np.uint8, 4: np.int32,
    5: np.int8, 6: np.int64, 7: np.bool_, 8: np.int16, 9: np.uint16,
    10: np.uint32, 11: np.uint64,
}
_NP_TO_FLAG = {np.dtype(v): k for k, v in _FLAG_TO_NP.items()}
# bfloat16 has no numpy dtype; MXNet uses flag 12 for it.
BFLOAT16_FLAG = 12

_NP_TO_TORCH = {
    np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64,
    np.dtype(np.float16): torch.float16, np.dtype(np.uint8): torch.uint8,
    np.dtype(np.int32): torch.int32, np.dtype(np.int8): torch.int8,
    np.dtype(np.int64): torch.int64, np.dtype(np.bool_): torch.bool,
    np.dtype(np.int16): torch.int16, np.dtype(np.uint16): torch.uint16,
    np.dtype(np.uint32): torch.uint32, np.dtype(np.uint64): torch.uint64,
}
_TORCH_TO_NP = {v: k.type for k, v in _NP_TO_TORCH.items()}


class _BF16Marker:
    """Stand-in numpy-side type object for bfloat16 (numpy has none)."""
    __name__ = 'bfloat16'
    name = 'bfloat16'

    def __repr__(self):
        return "<class 'bfloat16'>"


bfloat16 = _BF16Marker()


def torch_dtype(dtype):
    """Convert any dtype spec (str, numpy type, torch dtype, None) to a torch dtype."""
    if dtype is None:
        return torch.float32
    if isinstance(dtype, torch.dtype):
        return dtype
    if dtype is bfloat16 or (isinstance(dtype, str) and dtype in ('bfloat16', 'bf16')):
        return torch.bfloat16
    if isinstance(dtype, str) and dtype == 'float16':
        return torch.float16
    return _NP_TO_TORCH[np.dtype(dtype)]


def np_dtype(dtype):
    """Numpy dtype *type* (e.g. ``np.float32``) used as NDArray.dtype."""
    if isinstance(dtype, torch.dtype):
        if dtype == torch.bfloat16:
            return bfloat16
        return _TORCH_TO_NP[dtype]
    if dtype is bfloat16 or dtype == 'bfloat16':
        return bfloat16
    return np.dtype(dtype).type


def dtype_to_flag(dtype):
    td = torch_dtype(dtype)
    if td == torch.bfloat16:
        return BFLOAT16_FLAG
    return _NP_TO_FLAG[np.dtype(_TORCH_TO_NP[td])]


def flag_to_dtype(flag):
    if flag == BFLOAT16_FLAG:
        return torch.bfloat16
    return torch_dtype(_FLAG_TO_NP[flag])


def dtype_name(dtype):
    td = torch_dtype(dtype)
    if td == torch.bfloat16:
        return 'bfloat16'
    return np.dtype(_TORCH_TO_NP[td]).name


def check_call(ret):
    """Compatibility helper: raise MXNetError on non-zero return codes."""
    if ret != 0:
        raise MXNetError('native call failed with code {}'.format(ret))


class _NullType:
    """Placeholder for arguments that were not passed (mirrors base._Null)."""

    def __repr__(self):
        return '_Null'

    def __bool__(self):
        return False


_Null = _NullType()


# ----------------------------------------------------------------------------------------------
# C-API shim: the reference's tests drive a few graph-partitioning entry points through ctypes
# (``check_call(_LIB.MXBuildSubgraphByOpNames(sym.handle, c_str(b), mx_uint(n), c_str_array(names),
# ctypes.byref(out)))`` then ``Symbol(out)``).  ``_LIB`` implements those functions in Python over
# symbol/subgraph.py; handles are ctypes.c_void_p values naming objects in a handle table.
# ----------------------------------------------------------------------------------------------
import ctypes as _ctypes

SymbolHandle = _ctypes.c_void_p
NDArrayHandle = _ctypes.c_void_p
ExecutorHandle = _ctypes.c_void_p
_HANDLES = {}


def c_str(string):
    return _ctypes.c_char_p(string.encode('utf-8'))


def c_str_array(strings):
    arr = (_ctypes.c_char_p * len(strings))()
    arr[:] = [s.encode('utf-8') for s in strings]
    return arr


def c_array(ctype, values):
    return (ctype * len(values))(*values)


def _new_handle(obj):
    key = id(obj)
    _HANDLES[key] = obj
    return key


def _handle_object(h):
    v = h.value if isinstance(h, _ctypes.c_void_p) else h
    if v not in _HANDLES:
        raise MXNetError('invalid handle')
    return _HANDLES[v]


def _cstr(v):
    if isinstance(v, _ctypes.c_char_p):
        v = v.value
    return v.decode('utf-8') if isinstance(v, bytes) else str(v)


def _names(n, arr):
    return [_cstr(arr[i]) for i in range(int(n))]


class _CAPI:
    """The subset of the reference's libmxnet C API its Python tests call through ctypes."""

    @staticmethod
    def MXBuildSubgraphByOpNames(sym, backend, n, names, out):  # noqa: N802
        from .symbol import subgraph
        part = subgraph.partition(sym, _names(n, names))
        target = out._obj if hasattr(out, '_obj') else out
        target.value = _new_handle(part)
        return 0

    @staticmethod
    def MXSetSubgraphPropertyOpNames(backend, n, names):  # noqa: N802
        from .symbol import subgraph
        subgraph.set_backend_op_names(_cstr(backend), _names(n, names))
        return 0

    MXSetSubgraphPropertyOpNamesV2 = MXSetSubgraphPropertyOpNames

    @staticmethod
    def MXRemoveSubgraphPropertyOpNames(backend):  # noqa: N802
        from .symbol import subgraph
        subgraph.remove_backend(_cstr(backend))
        return 0

    MXRemoveSubgraphPropertyOpNamesV2 = MXRemoveSubgraphPropertyOpNames

    @staticmethod
    def MXNotifyShutdown():  # noqa: N802
        return 0

    @staticmethod
    def MXNDArrayFromDLPack(dlpack, out):  # noqa: N802
        """Wrap a ``DLManagedTensor*`` (the pointer inside a 'dltensor' capsule) as an NDArray; the
        new array owns the tensor (its deleter runs when the array is freed)."""
        import torch.utils.dlpack as _tdl
        ptr = dlpack.value if isinstance(dlpack, _ctypes.c_void_p) else dlpack
        new_capsule = _ctypes.pythonapi.PyCapsule_New
        new_capsule.restype = _ctypes.py_object
        new_capsule.argtypes = [_ctypes.c_void_p, _ctypes.c_char_p, _ctypes.c_void_p]
        capsule = new_capsule(ptr, _DLTENSOR_NAME, None)
        from .ndarray.ndarray import NDArray
        arr = NDArray(_tdl.from_dlpack(capsule))
        target = out._obj if hasattr(out, '_obj') else out
        target.value = _new_handle(arr)
        return 0


_DLTENSOR_NAME = b'dltensor'     # capsule names must outlive the capsules


_LIB = _CAPI()
