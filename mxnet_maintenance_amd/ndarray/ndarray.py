"""NDArray: the imperative tensor type.

Parity: python/mxnet/ndarray/ndarray.py (NDArray class, array/empty/zeros/
ones/full/arange/concatenate/moveaxis/imdecode, operator overloads, basic and
advanced indexing, fluent methods) and src/ndarray/ndarray.cc.

An NDArray owns a ``torch.Tensor`` (HBM on an MI355X, host memory on cpu).
Device work is ordered by the HIP stream, so ``wait_to_read`` is a stream
synchronisation; host-side asynchrony (IO, kvstore) goes through the native
dependency engine (engine.py).
"""
import ctypes

import numpy as np
import torch

from .. import _state
from .. import engine as _engine
from ..base import (MXNetError, numeric_types, integer_types, torch_dtype, np_dtype,
                    dtype_name)
from ..context import Context, current_context, context_from_torch

def _shares_storage(a, b):
    try:
        return a.untyped_storage().data_ptr() == b.untyped_storage().data_ptr()
    except RuntimeError:
        return False


# storage type ids of the reference C API (include/mxnet/ndarray.h NDArrayStorageType)
_STORAGE_TYPE_UNDEFINED = -1
_STORAGE_TYPE_DEFAULT = 0
_STORAGE_TYPE_ROW_SPARSE = 1
_STORAGE_TYPE_CSR = 2
_STORAGE_TYPE_STR_TO_ID = {'undefined': _STORAGE_TYPE_UNDEFINED, 'default': _STORAGE_TYPE_DEFAULT,
                           'row_sparse': _STORAGE_TYPE_ROW_SPARSE, 'csr': _STORAGE_TYPE_CSR}
_STORAGE_TYPE_ID_TO_STR = {v: k for k, v in _STORAGE_TYPE_STR_TO_ID.items()}
py_slice = slice       # the reference keeps the builtin under this name (``slice`` is an op there)

__all__ = ['NDArray', 'CachedOp', 'array', 'empty', 'zeros', 'ones', 'full', 'arange', 'linspace',
           'concatenate', 'moveaxis', 'waitall', 'from_numpy', 'from_dlpack', 'to_dlpack_for_read',
           'to_dlpack_for_write', 'eye', 'maximum', 'minimum', 'add', 'subtract', 'multiply',
           'divide', 'modulo', 'power', 'equal', 'not_equal', 'greater', 'greater_equal',
           'lesser', 'lesser_equal', 'logical_and', 'logical_or', 'logical_xor', 'true_divide',
           'negative', 'onehot_encode', 'histogram', 'split_v2', 'zeros_like', 'ones_like']

_GRAD_REQ = ('null', 'write', 'add')


def _wrap(t):
    return NDArray(t)



def _engine_copy(src, dev):
    """Host -> GPU copies of plain (non-recorded, big enough) tensors go through the dependency
    engine's copy streams (engine.host_to_device) instead of a copy on the compute stream."""
    if not torch.cuda.is_available() or _state.STATE.recording:
        return False
    from .. import engine
    return type(src) is torch.Tensor and engine.async_copy_ok(src, torch.device(dev))


def _async_upload(src, context):
    from .. import engine
    dst, var = engine.host_to_device(src, context.torch_device, name='as_in_context')
    out = NDArray(dst)
    out._engine_var = var
    return out

class NDArray:
    """An n-dimensional array on a :class:`Context`."""
    __slots__ = ('_data', '_grad', '_grad_req', '_stype', '__weakref__', '_fresh_grad', '_arena', '_host_ctx',
                 '_exc', '_recorded', '_idt', '_hist', '_engine_var', '_symbol')
    __array_priority__ = 1000.0

    def __init__(self, data=None, ctx=None, dtype=None, stype='default', writable=True, handle=None):
        if handle is not None:
            data = handle
        if isinstance(data, ctypes.c_void_p):
            # a handle from the C-API shim (monitor callbacks, partitioning): the array it names
            from ..base import _handle_object
            data = _handle_object(data)
        if isinstance(data, NDArray):
            data = data._data
        if not isinstance(data, torch.Tensor):
            data = torch.as_tensor(np.asarray(data))
        if dtype is not None:
            data = data.to(torch_dtype(dtype))
        if ctx is not None:
            data = data.to(ctx.torch_device)
        self._data = data
        self._grad = None
        self._grad_req = None
        self._stype = stype
        self._fresh_grad = False
        self._arena = None

    # ------------------------------------------------------------------ props
    @property
    def data(self):
        return self._data

    @property
    def shape(self):
        return tuple(self._data.shape)

    @property
    def size(self):
        return self._data.numel()

    @property
    def ndim(self):
        return self._data.dim()

    @property
    def dtype(self):
        return np_dtype(getattr(self, '_idt', None) or self._data.dtype)

    @property
    def stype(self):
        return self._stype

    @property
    def context(self):
        t = self._data
        if t.device.type == 'cpu' and getattr(self, '_host_ctx', None) is not None:
            return self._host_ctx       # cpu_pinned requested on a host without a GPU runtime to pin with
        if t.device.type == 'cpu' and t.is_pinned():
            from ..context import cpu_pinned
            return cpu_pinned(0)
        return context_from_torch(t.device)

    ctx = context

    @property
    def device(self):
        return self.context

    @property
    def handle(self):
        return self._data

    @property
    def writable(self):
        return True

    @property
    def grad(self):
        return self._grad

    @property
    def T(self):
        if self.ndim < 2:
            return self.copy()
        return self.transpose()

    @property
    def _fresh_grad_(self):
        return self._fresh_grad

    def __len__(self):
        if self.ndim == 0:
            raise TypeError('len() of unsized object')
        return self.shape[0]

    def __repr__(self):
        shape_info = 'x'.join(str(x) for x in self.shape)
        return '\n%s\n<%s %s @%s>' % (str(self.asnumpy()), self.__class__.__name__, shape_info, self.context)

    def __str__(self):
        return self.__repr__()

    def __hash__(self):
        return id(self)

    def __bool__(self):
        n = self.size
        if n == 0:
            return False            # reference: an empty NDArray is falsy
        if n == 1:
            return bool(self._data.reshape(-1)[0].item())
        raise ValueError('The truth value of an NDArray with multiple elements is ambiguous.')

    __nonzero__ = __bool__

    def __float__(self):
        return float(self.asscalar())

    def __int__(self):
        return int(self.asscalar())

    def __index__(self):
        return int(self.asscalar())

    def __iter__(self):
        if self.ndim == 1:
            for i in range(self.shape[0]):
                yield self[i]
        else:
            box = getattr(self, '_exc', None)
            for i in range(self.shape[0]):
                v = NDArray(self._data[i])
                if box is not None:
                    v._exc = box
                yield v

    def __array__(self, dtype=None, copy=None):
        a = self.asnumpy()
        return a.astype(dtype) if dtype is not None else a

    def __getstate__(self):
        return {'data': self.asnumpy(), 'ctx': self.context}

    def __setstate__(self, state):
        if 'handle' in state:
            # the reference's pickled state: one array in the raw-bytes save format
            # (MXNDArraySaveRawBytes); a GPU context in it loads on the CPU when no GPU is present
            from .utils import _Reader, _read_array
            self._data = _read_array(_Reader(bytes(state['handle'])))._data
        else:
            self._data = torch.from_numpy(np.ascontiguousarray(state['data']))
        self._grad = None
        self._grad_req = None
        self._stype = 'default'
        self._fresh_grad = False
        self._arena = None

    def __reduce__(self):
        return (_rebuild, (self.asnumpy(),))

    # ---------------------------------------------------------------- sync/io
    def _rethrow(self):
        """Raise the deferred failure of the operator that produced this array (once)."""
        box = getattr(self, '_exc', None)
        if box is not None and box[0] is not None:
            from .. import engine
            engine.rethrow(box)

    def wait_to_read(self):
        _engine.join_workers()
        var = getattr(self, '_engine_var', None)
        if var is not None:
            # an array written by an engine op (e.g. an async host -> device copy): its variable
            from .. import engine
            engine.wait_for_var(var)
        if self._data.is_cuda:
            torch.cuda.current_stream(self._data.device).synchronize()
        self._rethrow()

    wait_to_write = wait_to_read

    def asnumpy(self):
        _engine.join_workers()
        self._rethrow()
        t = self._data.detach()
        idt = getattr(self, '_idt', None)
        if idt is not None:
            t = t.to(idt)       # an integer variable carried in float64 for autograd
        if t.dtype == torch.bfloat16:
            t = t.float()
        return t.cpu().numpy().copy() if t.device.type == 'cpu' else t.cpu().numpy()

    def asscalar(self):
        if self.size != 1:
            raise ValueError('The current array is not a scalar')
        return self.asnumpy().reshape(-1)[0]

    def item(self):
        return self.asscalar()

    def tolist(self):
        return self.asnumpy().tolist()

    def astype(self, dtype, copy=True):
        td = torch_dtype(dtype)
        if not copy and td == self._data.dtype:
            return self
        return _invoke_unary(lambda t: t.to(td) if t.dtype != td else t.clone(), self)

    def copy(self):
        if self._stype != 'default' and type(self) is NDArray:
            # a dense array tagged with a sparse storage type (a sparse Parameter's replica): its copy
            # is a real sparse array of that type
            from . import sparse
            cls = sparse.RowSparseNDArray if self._stype == 'row_sparse' else sparse.CSRNDArray
            return _tag_host_ctx(cls(self._data.detach().clone()), getattr(self, '_host_ctx', None))
        return _invoke_unary(lambda t: t.clone(), self)

    def __copy__(self):
        return self.copy()

    def __deepcopy__(self, memo):
        return NDArray(self._data.detach().clone())

    def copyto(self, other):
        _engine.join_workers()
        if isinstance(other, NDArray):
            if other is self:
                return other
            src = self._data.detach() if not _state.STATE.recording else self._data
            if other.shape != self.shape:
                raise MXNetError('copyto: shape mismatch %s vs %s' % (self.shape, other.shape))
            if _engine_copy(src, other._data.device) and other._data.is_contiguous() \
                    and other._data.dtype == src.dtype:
                from .. import engine
                _, other._engine_var = engine.host_to_device(src, other._data.device, out=other._data,
                                                             var=getattr(other, '_engine_var', None), name='copyto')
            else:
                with torch.no_grad():
                    other._data.copy_(src)
            _share_failure(self, other)
            return other
        if isinstance(other, Context):
            if _engine_copy(self._data, other.torch_device):
                return _share_failure(self, _async_upload(self._data, other))
            return _share_failure(self, _tag_host_ctx(NDArray(self._data.to(other.torch_device, copy=True)), other))
        raise TypeError('copyto does not support type ' + str(type(other)))

    def as_in_context(self, context):
        if self.context == context:
            return self
        _engine.join_workers()
        if context.device_typeid == 3:
            t = self._data.detach().cpu()
            if torch.cuda.is_available():
                return NDArray(t.pin_memory())
            out = NDArray(t.clone() if t.data_ptr() == self._data.data_ptr() else t)
            out._host_ctx = context
            return out
        if _engine_copy(self._data, context.torch_device):
            return _share_failure(self, _async_upload(self._data, context))
        return _tag_host_ctx(_invoke_unary(lambda t: t.to(context.torch_device), self), context)

    as_in_ctx = as_in_context

    def to_device(self, device):
        return self.as_in_context(device)

    def detach(self):
        return NDArray(self._data.detach())

    def tostype(self, stype):
        from . import sparse
        return sparse.cast_storage(self, stype)

    def asnd(self):
        return self

    def as_np_ndarray(self):
        """Zero-copy ``mx.np.ndarray`` view sharing data, gradient buffer and grad_req."""
        from ..numpy import ndarray as np_ndarray
        r = np_ndarray.__new__(np_ndarray)
        for k in ('_data', '_grad', '_grad_req', '_stype', '_fresh_grad', '_arena'):
            setattr(r, k, getattr(self, k))
        return r

    def as_nd_ndarray(self):
        return self

    def to_dlpack_for_read(self):
        return torch.utils.dlpack.to_dlpack(self._data)

    to_dlpack_for_write = to_dlpack_for_read

    # ------------------------------------------------------------- autograd
    def attach_grad(self, grad_req='write', stype=None):
        """Allocate a gradient buffer and mark this array as a leaf variable."""
        if grad_req not in _GRAD_REQ:
            raise ValueError('grad_req must be one of %s' % (_GRAD_REQ,))
        t = self._data.detach()
        if grad_req == 'null':
            self._data = t
            self._grad = None
            self._grad_req = None
            return
        if not t.is_floating_point():
            # integer (and bool) variables differentiate as in the reference: the values are carried
            # in float64 (exact for the integers tests use) with the integer dtype kept in _idt;
            # operators on them compute the integer result and take the gradient path from the
            # float copy (register.invoke), and the gradient reports the integer dtype too
            idt = getattr(self, '_idt', None) or t.dtype
            t = t.to(torch.float64).requires_grad_(True)
            self._data = t
            self._idt = idt
            self._grad = NDArray(torch.zeros_like(t))
            self._grad._idt = idt
            if self.__class__ is not NDArray:
                self._grad.__class__ = self.__class__
            t.grad = self._grad._data       # autograd accumulates straight into the buffer
            self._grad_req = grad_req
            return
        t.requires_grad_(True)
        self._data = t
        g = torch.zeros_like(t)
        gstype = stype or self._stype
        if gstype != 'default':
            # sparse gradient buffer (reference: attach_grad(stype=...)); its dense view is the tensor
            # autograd accumulates into, the compressed form is derived on access
            from . import sparse
            self._grad = {'row_sparse': sparse.RowSparseNDArray, 'csr': sparse.CSRNDArray}[gstype](g)
            g = self._grad._data
        else:
            self._grad = NDArray(g)
            if self.__class__ is not NDArray and self._stype == 'default':
                self._grad.__class__ = self.__class__
        t.grad = g
        self._grad_req = grad_req

    def _set_grad_buffer(self, gbuf, grad_req='write'):
        """Bind an external (e.g. bucketed flat) gradient buffer to this leaf."""
        t = self._data.detach().requires_grad_(True)
        self._data = t
        t.grad = gbuf
        if self._grad is None:
            self._grad = NDArray(gbuf)
        else:
            self._grad._data = gbuf
        self._grad_req = grad_req

    def backward(self, out_grad=None, retain_graph=False, train_mode=True):
        from .. import autograd
        autograd.backward([self], None if out_grad is None else [out_grad],
                          retain_graph=retain_graph, train_mode=train_mode)

    # ------------------------------------------------------------ indexing
    def __getitem__(self, key):
        key = _convert_key(key)
        t = self._data
        if isinstance(key, int) and t.dim() >= 1:
            n = t.shape[0]
            if not -n <= key < n:
                raise IndexError('index %d is out of bounds for axis 0 with size %d' % (key, n))
        r = _index_fn(t, key)
        if r.dim() == 0 and not _state.STATE.np_shape:
            r = r.reshape(1)
        out = NDArray(r)
        idt = getattr(self, '_idt', None)
        if idt is not None:
            out._idt = idt                  # an integer variable's float64 carrier: the result is integer too
        if _state.STATE.recording and self._grad_req is not None:
            _state.STATE.tape_leaves[id(self)] = self
        box = getattr(self, '_exc', None)
        if box is not None:
            out._exc = box
        return out

    def __setitem__(self, key, value):
        _engine.join_workers()
        key = _convert_key(key)
        if isinstance(value, NDArray):
            _share_failure(value, self)          # writing a failed result fails the target too
            v = value._data
        elif torch.is_tensor(value):
            v = value
        elif isinstance(value, np.generic):
            v = value.item()
        elif isinstance(value, numeric_types):
            v = value
        else:
            v = torch.as_tensor(np.asarray(value), dtype=self._data.dtype)
        t = self._data
        if _state.STATE.recording and torch.is_tensor(v) and v.requires_grad and not t.requires_grad:
            # a recorded write of a differentiable value into an untracked array: the array joins the
            # graph (its untouched elements are constants); an integer array cannot carry gradients
            if not t.is_floating_point():
                raise MXNetError('Inplace operations (+=, -=, x[:]=, etc) are not supported when recording with '
                                 'autograd: the %s target cannot carry the value\'s gradient' % t.dtype)
            if t._base is not None:
                # replacing a view's storage would silently detach it from its parent array
                raise MXNetError('Inplace operations (+=, -=, x[:]=, etc) are not supported when recording with '
                                 'autograd: the target is a view of another array')
            new = t.detach().clone()
            new[key] = v.to(new.device, new.dtype)
            self._data = new
            return
        if _state.STATE.recording and t.requires_grad and not t.is_leaf:
            new = t.clone()
            new[key] = v.to(new.device, new.dtype) if torch.is_tensor(v) else v
            self._data = new
            return
        whole = (isinstance(key, slice) and key == slice(None)) or key is Ellipsis or key == ()
        if t.dim() == 0 and whole:
            # x[:] = v on a 0-d array (NumPy semantics: assign the scalar)
            with torch.no_grad():
                t.copy_(v.to(t.device, t.dtype).reshape(()) if torch.is_tensor(v) else torch.as_tensor(v, dtype=t.dtype))
            return
        key, flips = _positive_step_key(t, key)
        if flips is None:
            # key is now a tensor of flat positions
            if not torch.is_tensor(v):
                v = torch.as_tensor(v, dtype=t.dtype)
            v = v.to(t.device, t.dtype)
            while v.dim() > key.dim() and v.shape[0] == 1:
                v = v[0]
            with torch.no_grad():
                vals = v.expand(key.shape).reshape(-1)
                if t.is_contiguous():
                    t.view(-1)[key.reshape(-1)] = vals
                else:
                    # strided / transposed target: scatter through the unravelled indices
                    idx = torch.unravel_index(key.reshape(-1), t.shape)
                    t[idx] = vals
            return
        if flips:
            # negative-step slices: write the mirrored positive-step slice with the value flipped
            if not torch.is_tensor(v):
                v = torch.as_tensor(v, dtype=t.dtype)
            v = v.to(t.device, t.dtype)
            tshape = t[key].shape
            while v.dim() > len(tshape) and v.shape[0] == 1:
                v = v[0]
            v = v.expand(tshape).flip(flips)
        with torch.no_grad():
            if torch.is_tensor(v):
                v = v.to(t.device, t.dtype)
                tgt = t[key] if not (isinstance(key, slice) and key == slice(None)) else t
                if tgt.dim() and v.dim() > tgt.dim():
                    # extra leading unit axes broadcast away (value (1, 1, 1, 9) into a (16, 9, 9) slot)
                    while v.dim() > tgt.dim() and v.shape[0] == 1:
                        v = v[0]
                    if v.dim() > tgt.dim():
                        v = v.reshape(tgt.shape)
            t[key] = v

    def slice(self, *args, **kwargs):
        return _op('slice', self, *args, **kwargs)

    def _at(self, idx):
        return NDArray(self._data[idx])

    def _slice(self, start, stop):
        return NDArray(self._data[start:stop])

    # ----------------------------------------------------------- reshaping
    def reshape(self, *shape, **kwargs):
        if len(shape) == 1 and isinstance(shape[0], (list, tuple)):
            shape = tuple(shape[0])
        if not shape:
            shape = kwargs.get('shape', ())
        reverse = kwargs.get('reverse', False)
        from ..ops.tensor import infer_reshape
        new = infer_reshape(self.shape, shape, reverse)
        n = 1
        for d in new:
            n *= d
        if n != self.size:
            raise ValueError('cannot reshape array of size %d into shape %s' % (self.size, tuple(new)))
        return _invoke_unary(lambda t: t.reshape(new), self)

    def reshape_like(self, *args, **kwargs):
        return _op('reshape_like', self, *args, **kwargs)

    def zeros_like(self, *args, **kwargs):
        return _op('zeros_like', self, *args, **kwargs)

    def ones_like(self, *args, **kwargs):
        return _op('ones_like', self, *args, **kwargs)

    def broadcast_to(self, shape):
        return _op('broadcast_to', self, shape=shape)

    def broadcast_like(self, other):
        return _op('broadcast_like', self, other)

    @staticmethod
    def _basic_indexing_slice_is_contiguous(slc_key, shape):
        """Whether ``x[slc_key]`` (one slice per axis) of a C-contiguous ``x`` is contiguous: after
        dropping length-1 axes, each remaining axis must step by exactly the product of the
        lengths of the axes after it."""
        lens, steps = [], []
        stride = 1
        for slc, n in reversed(list(zip(slc_key, shape))):
            start, stop, step = slc.indices(n)
            length = len(range(start, stop, step))
            if length == 0:
                return True
            lens.append(length)
            steps.append(stride * step)
            stride *= n
        expect = 1
        for length, st in zip(lens, steps):      # innermost first
            if length == 1:
                continue
            if st != expect:
                return False
            expect *= length
        return True

    # shape-only views: ``inplace=True`` shares storage with self, otherwise the result is a copy
    def _maybe_copy(self, out, inplace):
        if inplace or not _shares_storage(out._data, self._data):
            return out
        return _invoke_unary(lambda t: t.clone(), out)

    def flatten(self, inplace=False):
        return self._maybe_copy(_op('Flatten', self), inplace)

    def expand_dims(self, axis, inplace=False):
        return self._maybe_copy(_op('expand_dims', self, axis=axis), inplace)

    def squeeze(self, axis=None, inplace=False):
        return self._maybe_copy(_op('squeeze', self, axis=axis), inplace)

    def transpose(self, *axes, **kwargs):
        if len(axes) == 1 and isinstance(axes[0], (list, tuple)):
            axes = tuple(axes[0])
        if not axes:
            axes = kwargs.get('axes', ())
        return _op('transpose', self, axes=axes)

    def diag(self, k=0, **kwargs):
        return _op('diag', self, k=k, **kwargs)

    def split(self, *args, **kwargs):
        return _op('split', self, *args, **kwargs)

    def split_v2(self, *args, **kwargs):
        return split_v2(self, *args, **kwargs)

    # ----------------------------------------------------------- arithmetic
    def __add__(self, other):
        return _ufunc(self, other, 'broadcast_add', '_plus_scalar')

    def __iadd__(self, other):
        return _inplace(self, other, torch.Tensor.add_, 'broadcast_add', '_plus_scalar')

    def __radd__(self, other):
        return self.__add__(other)

    def __sub__(self, other):
        return _ufunc(self, other, 'broadcast_sub', '_minus_scalar')

    def __isub__(self, other):
        return _inplace(self, other, torch.Tensor.sub_, 'broadcast_sub', '_minus_scalar')

    def __rsub__(self, other):
        return _ufunc(self, other, 'broadcast_sub', '_rminus_scalar', reverse=True)

    def __mul__(self, other):
        return _ufunc(self, other, 'broadcast_mul', '_mul_scalar')

    def __imul__(self, other):
        return _inplace(self, other, torch.Tensor.mul_, 'broadcast_mul', '_mul_scalar')

    def __rmul__(self, other):
        return self.__mul__(other)

    def __truediv__(self, other):
        return _ufunc(self, other, 'broadcast_div', '_div_scalar')

    __div__ = __truediv__

    def __itruediv__(self, other):
        return _inplace(self, other, torch.Tensor.div_, 'broadcast_div', '_div_scalar')

    __idiv__ = __itruediv__

    def __rtruediv__(self, other):
        return _ufunc(self, other, 'broadcast_div', '_rdiv_scalar', reverse=True)

    __rdiv__ = __rtruediv__

    def __mod__(self, other):
        return _ufunc(self, other, 'broadcast_mod', '_mod_scalar')

    def __rmod__(self, other):
        return _ufunc(self, other, 'broadcast_mod', '_rmod_scalar', reverse=True)

    def __imod__(self, other):
        r = self.__mod__(other)
        self._assign(r)
        return self

    def __pow__(self, other):
        return _ufunc(self, other, 'broadcast_power', '_power_scalar')

    def __rpow__(self, other):
        return _ufunc(self, other, 'broadcast_power', '_rpower_scalar', reverse=True)

    def __neg__(self):
        return _op('negative', self)

    def __pos__(self):
        return self

    def __abs__(self):
        return _op('abs', self)

    def __eq__(self, other):
        if other is None:
            return False
        return _ufunc(self, other, 'broadcast_equal', '_equal_scalar')

    def __ne__(self, other):
        if other is None:
            return True
        return _ufunc(self, other, 'broadcast_not_equal', '_not_equal_scalar')

    def __gt__(self, other):
        return _ufunc(self, other, 'broadcast_greater', '_greater_scalar')

    def __ge__(self, other):
        return _ufunc(self, other, 'broadcast_greater_equal', '_greater_equal_scalar')

    def __lt__(self, other):
        return _ufunc(self, other, 'broadcast_lesser', '_lesser_scalar')

    def __le__(self, other):
        return _ufunc(self, other, 'broadcast_lesser_equal', '_lesser_equal_scalar')

    def __matmul__(self, other):
        return _op('dot', self, other)

    def _assign(self, r):
        if _state.STATE.recording and (self._data.requires_grad or r._data.requires_grad) and not self._data.is_leaf:
            self._data = r._data
        else:
            _engine.join_workers()
            with torch.no_grad():
                self._data.copy_(r._data)

    def __getattr__(self, name):
        # fluent methods: a.sum(axis=1) -> nd.sum(a, axis=1)
        if name.startswith('__'):
            raise AttributeError(name)
        from ..ops import registry
        if name in _FLUENT and registry.has(_FLUENT[name]):
            opname = _FLUENT[name]
            return lambda *args, **kwargs: _op(opname, self, *args, **kwargs)
        raise AttributeError("'NDArray' object has no attribute '%s'" % name)


# fluent method name -> operator name
_FLUENT = {n: n for n in [
    'sum', 'mean', 'max', 'min', 'prod', 'nansum', 'nanprod', 'norm', 'argmax', 'argmin',
    'argmax_channel', 'pick', 'clip', 'abs', 'sign', 'sqrt', 'rsqrt', 'cbrt', 'rcbrt', 'square',
    'exp', 'expm1', 'log', 'log10', 'log2', 'log1p', 'sin', 'cos', 'tan', 'arcsin', 'arccos',
    'arctan', 'sinh', 'cosh', 'tanh', 'arcsinh', 'arccosh', 'arctanh', 'degrees', 'radians',
    'relu', 'sigmoid', 'softmax', 'log_softmax', 'softmin', 'round', 'rint', 'fix', 'floor',
    'ceil', 'trunc', 'reciprocal', 'tile', 'repeat', 'pad', 'flip', 'sort', 'argsort', 'topk',
    'take', 'one_hot', 'slice_axis', 'slice_like', 'swapaxes', 'depth_to_space', 'space_to_depth',
    'shape_array', 'size_array', 'nanprod', 'gamma', 'gammaln', 'erf', 'erfinv', 'ones_like',
    'log_sigmoid', 'mish', 'where', 'dot', 'batch_dot']}
_FLUENT['broadcast_axes'] = 'broadcast_axes'
_FLUENT['sum_axis'] = 'sum'
_FLUENT['max_axis'] = 'max'
_FLUENT['min_axis'] = 'min'


def _rebuild(arr):
    return NDArray(torch.from_numpy(np.ascontiguousarray(arr)))


# ---------------------------------------------------------------------------
# indexing helpers
# ---------------------------------------------------------------------------

def _convert_key(key):
    if isinstance(key, NDArray):
        t = key._data
        return t.to(torch.int64) if t.is_floating_point() else t
    if isinstance(key, np.ndarray):
        return torch.as_tensor(key.astype(np.int64) if key.dtype.kind == 'f' else key)
    if isinstance(key, list):
        if key and all(isinstance(k, (bool, np.bool_)) for k in key):
            return torch.as_tensor(np.asarray(key, dtype=np.bool_))       # a boolean mask
        return torch.as_tensor(np.asarray(key, dtype=np.int64))
    if isinstance(key, tuple):
        return tuple(_convert_key(k) if isinstance(k, (NDArray, np.ndarray, list)) else
                     (int(k) if isinstance(k, np.integer) else k) for k in key)
    if isinstance(key, np.integer):
        return int(key)
    return key


def _index_fn(t, key):
    if isinstance(key, tuple):
        key = tuple(k.to(t.device) if torch.is_tensor(k) else k for k in key)
        neg = any(isinstance(k, slice) and k.step is not None and k.step < 0 for k in key)
        if neg and not any(k is Ellipsis for k in key):
            # torch has no negative-step slicing: apply those axes with index_select
            # first (keeps the rank), then the rest of the key.
            ax = 0
            newkey = []
            for k in key:
                if k is None:
                    newkey.append(k)
                    continue
                if isinstance(k, slice) and k.step is not None and k.step < 0:
                    b, e, s = k.indices(t.shape[ax])
                    t = t.index_select(ax, torch.tensor(list(range(b, e, s)), dtype=torch.long, device=t.device))
                    newkey.append(slice(None))
                else:
                    newkey.append(k)
                ax += 1
            key = tuple(newkey)
    elif torch.is_tensor(key):
        key = key.to(t.device)
    elif isinstance(key, slice) and key.step is not None and key.step < 0:
        from ..ops.tensor import _neg_step_slice
        return _neg_step_slice(t, [key])
    return t[key]


# ---------------------------------------------------------------------------
# op invocation helpers
# ---------------------------------------------------------------------------

def _op(name, *args, **kwargs):
    from .register import invoke_by_name
    return invoke_by_name(name, args, kwargs)


def _invoke_unary(fn, arr):
    from .register import invoke_fn
    return invoke_fn(fn, [arr])


def _ufunc(lhs, rhs, bop, sop, reverse=False):
    if isinstance(rhs, NDArray):
        if reverse:
            return _op(bop, rhs, lhs)
        return _op(bop, lhs, rhs)
    if isinstance(rhs, numeric_types):
        return _op(sop, lhs, scalar=float(rhs) if not isinstance(rhs, bool) else float(rhs))
    if isinstance(rhs, np.ndarray):
        other = array(rhs, ctx=lhs.context, dtype=lhs.dtype)
        return _ufunc(lhs, other, bop, sop, reverse)
    return NotImplemented


def _inplace(self, other, torch_fn, bop, sop):
    if _state.STATE.recording and (self._data.requires_grad or
                                   (isinstance(other, NDArray) and other._data.requires_grad)):
        r = _ufunc(self, other, bop, sop)
        self._data = r._data
        return self
    o = other._data if isinstance(other, NDArray) else other
    _engine.join_workers()       # a direct write on the caller's stream (worker streams done first)
    with torch.no_grad():
        if torch.is_tensor(o) and o.shape != self._data.shape:
            torch_fn(self._data, o.expand_as(self._data) if o.dim() <= self._data.dim() else o)
        else:
            torch_fn(self._data, o)
    return self


# ---------------------------------------------------------------------------
# creation functions
# ---------------------------------------------------------------------------

def _ctx(ctx):
    return ctx if ctx is not None else current_context()


def _share_failure(src, dst):
    """``dst`` was computed from ``src``: it carries ``src``'s pending operator failure."""
    box = getattr(src, '_exc', None)
    if box is not None and box[0] is not None:
        dst._exc = box
    return dst


def _positive_step_key(t, key):
    """A basic index with negative-step slices -> (the same elements as positive-step slices, the
    result axes whose order those reverse).  torch has no negative-step views; assignment through
    one writes the mirrored slice with a flipped value."""
    items = key if isinstance(key, tuple) else (key,)
    if not any(isinstance(k, slice) and k.step is not None and k.step < 0 for k in items):
        return key, []
    if any(torch.is_tensor(k) or isinstance(k, (list, np.ndarray)) for k in items):
        # with advanced indices: the flat positions NumPy's indexing selects (one host pass)
        nkey = tuple(k.cpu().numpy() if torch.is_tensor(k) else k for k in items)
        flat = np.arange(t.numel()).reshape(tuple(t.shape))[nkey]
        return torch.from_numpy(np.ascontiguousarray(flat)).to(t.device), None
    if any(k is Ellipsis for k in items):
        i = [j for j, k in enumerate(items) if k is Ellipsis][0]
        used = sum(1 for k in items if k is not None and k is not Ellipsis)
        items = items[:i] + (slice(None),) * (t.dim() - used) + items[i + 1:]
    out, flips = [], []
    ax = oax = 0
    for k in items:
        if k is None:
            out.append(k)
            oax += 1
            continue
        if isinstance(k, slice) and k.step is not None and k.step < 0:
            b, e, s = k.indices(t.shape[ax])
            n = len(range(b, e, s))
            if n == 0:
                out.append(slice(0, 0))
            else:
                last = b + (n - 1) * s
                out.append(slice(last, b + 1, -s))
                flips.append(oax)
            oax += 1
        else:
            out.append(k)
            if isinstance(k, slice):
                oax += 1
        ax += 1
    return tuple(out), flips


def _tag_host_ctx(arr, ctx):
    """Label a host array with a virtual CPU context (``cpu(k)``, k > 0): every CPU context is the same
    host memory here, but an array created or placed on ``cpu(k)`` reports that context, as in the
    reference, which keeps one storage pool per CPU device id.  ``cpu_shared`` arrays live in shared
    memory (the storage worker processes hand to each other) and report that context."""
    if isinstance(ctx, str):
        ctx = Context(ctx)
    if not isinstance(ctx, Context) or arr._data.device.type != 'cpu':
        return arr
    if ctx.device_typeid == 5:
        arr._data.share_memory_()
        arr._host_ctx = ctx
    elif ctx.device_typeid == 1 and ctx.device_id != 0:
        arr._host_ctx = ctx
    return arr


def array(source_array, ctx=None, dtype=None):
    """Create an NDArray from any array-like (float32 by default, like MXNet)."""
    ctx = _ctx(ctx)
    if getattr(source_array, 'stype', 'default') != 'default' or (
            hasattr(source_array, 'tocsr') and not isinstance(source_array, (NDArray, torch.Tensor))):
        from . import sparse      # sparse NDArray / scipy matrix sources stay sparse
        return sparse.array(source_array, ctx=ctx, dtype=dtype)
    if isinstance(source_array, NDArray):
        dt = torch_dtype(dtype) if dtype is not None else source_array._data.dtype
        return NDArray(source_array._data.detach().to(device=ctx.torch_device, dtype=dt, copy=True))
    if isinstance(source_array, torch.Tensor):
        dt = torch_dtype(dtype) if dtype is not None else source_array.dtype
        return NDArray(source_array.detach().to(device=ctx.torch_device, dtype=dt, copy=True))
    if isinstance(source_array, np.ndarray):
        # MXNet: only NDArray sources keep their dtype; everything else defaults to float32
        dt = dtype if dtype is not None else np.float32
    else:
        dt = dtype if dtype is not None else np.float32
        source_array = np.asarray(source_array, dtype=None if dtype is None else None)
    td = torch_dtype(dt)
    if td == torch.bfloat16:
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(source_array, dtype=np.float32))).to(td)
    else:
        npd = np.dtype(np_dtype(td)) if td != torch.bfloat16 else np.float32
        t = torch.from_numpy(np.array(source_array, dtype=npd, copy=True))
    if ctx.device_typeid == 3:
        if torch.cuda.is_available():
            t = t.pin_memory()
        else:
            out = NDArray(t)
            out._host_ctx = ctx
            return out
    return _tag_host_ctx(NDArray(t.to(ctx.torch_device) if ctx.device_typeid == 2 else t), ctx)


def from_numpy(ndarray, zero_copy=True):
    """NDArray over a numpy array.  With ``zero_copy`` the memory is shared and the numpy array
    becomes read-only (as in the reference, which takes ownership of the buffer)."""
    if not zero_copy:
        return NDArray(torch.from_numpy(np.array(ndarray, copy=True)))
    if not ndarray.flags['C_CONTIGUOUS']:
        raise ValueError('from_numpy with zero_copy=True needs a C-contiguous array; use zero_copy=False')
    src = ndarray
    t = torch.from_numpy(src)
    ndarray.flags.writeable = False
    return NDArray(t)


def from_dlpack(dlpack):
    return NDArray(torch.utils.dlpack.from_dlpack(dlpack))


def to_dlpack_for_read(data):
    return data.to_dlpack_for_read()


def to_dlpack_for_write(data):
    return data.to_dlpack_for_write()


def _into(out, result):
    """Honour an ``out=`` argument of the creation functions."""
    if out is None:
        return result
    out[:] = result
    return out


def empty(shape, ctx=None, dtype=None, stype=None):
    if isinstance(shape, (int, np.integer)):
        shape = (int(shape),)
    else:
        shape = tuple(int(d) for d in shape)
    if stype not in (None, 'default'):
        from . import sparse
        return sparse.empty(stype, shape, ctx=ctx, dtype=dtype)
    return _tag_host_ctx(NDArray(torch.empty(shape, dtype=torch_dtype(dtype), device=_ctx(ctx).torch_device)), ctx)


def _created(opname, make):
    """Creation functions are operators of the reference (_zeros, _ones, _full): profiled as such."""
    from .. import profiler as _prof
    if not _prof.active_imperative:
        return make()
    with _prof.op_span(_prof.current_scope() + opname):
        r = make()
    if _prof.active_memory:
        _prof.memory_alloc(r)
    return r


def _check_creation_shape(shape, what):
    """Legacy (non NumPy-shape) semantics: a 0 dim means "unknown" and () is no shape, so creating
    such an array is an error (reference: InitNDArray shape checks); under np_shape both are real."""
    from ..util import is_np_shape
    if not is_np_shape() and (len(shape) == 0 or any(int(d) == 0 for d in shape)):
        raise MXNetError('%s: shape %s has unknown (0) dimensions; use mx.np_shape() for scalar or '
                         'zero-size arrays' % (what, tuple(shape)))


def zeros(shape, ctx=None, dtype=None, stype=None, out=None, **kwargs):
    if isinstance(shape, int):
        shape = (shape,)
    if stype in (None, 'default'):
        _check_creation_shape(tuple(shape), 'zeros')
    if stype not in (None, 'default'):
        from . import sparse
        return sparse.zeros(stype, shape, ctx=ctx, dtype=dtype)
    return _into(out, _created('_zeros', lambda: _tag_host_ctx(NDArray(torch.zeros(
        shape, dtype=torch_dtype(dtype), device=_ctx(ctx).torch_device)), ctx)))


def ones(shape, ctx=None, dtype=None, out=None, **kwargs):
    if isinstance(shape, int):
        shape = (shape,)
    _check_creation_shape(tuple(shape), 'ones')
    return _into(out, _created('_ones', lambda: _tag_host_ctx(NDArray(torch.ones(
        shape, dtype=torch_dtype(dtype), device=_ctx(ctx).torch_device)), ctx)))


def full(shape, val, ctx=None, dtype=np.float32, out=None):
    if isinstance(shape, int):
        shape = (shape,)
    r = _tag_host_ctx(NDArray(torch.full(shape, val, dtype=torch_dtype(dtype), device=_ctx(ctx).torch_device)), ctx)
    if out is not None:
        out[:] = r
        return out
    return r


def eye(N, M=0, k=0, ctx=None, dtype=None):
    return _op('_eye', N=N, M=M, k=k, ctx=_ctx(ctx), dtype=dtype_name(dtype or np.float32))


def arange(start, stop=None, step=1.0, repeat=1, infer_range=None, ctx=None, dtype=np.float32):
    if stop is None:
        start, stop = 0, start
    return _op('_arange', start=start, stop=stop, step=step, repeat=repeat, ctx=_ctx(ctx),
               dtype=dtype_name(dtype))


def linspace(start, stop, num, endpoint=True, ctx=None, dtype=np.float32):
    return _op('_linspace', start=start, stop=stop, num=num, endpoint=endpoint, ctx=_ctx(ctx),
               dtype=dtype_name(dtype))


def zeros_like(data, **kwargs):
    return _op('zeros_like', data)


def ones_like(data, **kwargs):
    return _op('ones_like', data)


def concatenate(arrays, axis=0, always_copy=True):
    return _op('Concat', *arrays, dim=axis, num_args=len(arrays))


def moveaxis(tensor, source, destination):
    """Move axes ``source`` to positions ``destination`` (ints or sequences of ints)."""
    def norm(a):
        axes = tuple(a) if isinstance(a, (list, tuple, range)) else (a,)
        for ax in axes:
            if not -tensor.ndim <= ax < tensor.ndim:
                raise ValueError('moveaxis: axis %d is out of bounds for an array of dimension %d' % (ax, tensor.ndim))
        return tuple(a) if isinstance(a, (list, tuple, range)) else a
    src, dst = norm(source), norm(destination)
    s_list = src if isinstance(src, tuple) else (src,)
    d_list = dst if isinstance(dst, tuple) else (dst,)
    if len(s_list) != len(d_list):
        raise ValueError('moveaxis: source and destination must have the same number of elements')
    for lst, what in ((s_list, 'source'), (d_list, 'destination')):
        if len({a % tensor.ndim for a in lst}) != len(lst):
            raise ValueError('moveaxis: repeated axis in %s' % what)
    return NDArray(torch.movedim(tensor._data, src, dst).contiguous())


def waitall():
    """Block until all pending device work and engine work has completed; then raise the oldest
    deferred operator failure, if any (every pending failure is cleared)."""
    _engine.join_workers()
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()
    from .. import engine
    engine.wait_all()
    engine.rethrow_all()


def onehot_encode(indices, out):
    r = _op('one_hot', indices, depth=out.shape[1], dtype=dtype_name(out.dtype))
    out[:] = r
    return out


def split_v2(ary, indices_or_sections, axis=0, squeeze_axis=False):
    if isinstance(indices_or_sections, int):
        return _op('_split_v2', ary, axis=axis, squeeze_axis=squeeze_axis, sections=indices_or_sections)
    return _op('_split_v2', ary, axis=axis, squeeze_axis=squeeze_axis,
               indices=(0,) + tuple(indices_or_sections))


def histogram(a, bins=10, range=None):
    if isinstance(bins, NDArray):
        return _op('_histogram', a, bins)
    return _op('_histogram', a, bin_cnt=bins, range=range)


def _binary_helper(lhs, rhs, bop, sop, rsop=None):
    if isinstance(lhs, NDArray):
        return _ufunc(lhs, rhs, bop, sop)
    if isinstance(rhs, NDArray):
        if rsop is None:
            return _ufunc(rhs, lhs, bop, sop)
        return _ufunc(rhs, lhs, bop, rsop, reverse=True)
    # two python scalars: the plain scalar result (reference _ufunc_helper's lfn_scalar)
    import operator
    fn = {'broadcast_add': operator.add, 'broadcast_sub': operator.sub, 'broadcast_mul': operator.mul,
          'broadcast_div': operator.truediv, 'broadcast_mod': operator.mod, 'broadcast_power': operator.pow,
          'broadcast_maximum': max, 'broadcast_minimum': min, 'broadcast_hypot': lambda a, b: (a * a + b * b) ** 0.5,
          'broadcast_equal': lambda a, b: float(a == b), 'broadcast_not_equal': lambda a, b: float(a != b),
          'broadcast_greater': lambda a, b: float(a > b), 'broadcast_greater_equal': lambda a, b: float(a >= b),
          'broadcast_lesser': lambda a, b: float(a < b), 'broadcast_lesser_equal': lambda a, b: float(a <= b)}.get(bop)
    if fn is None:
        raise TypeError('%s: at least one operand must be an NDArray' % bop)
    return fn(lhs, rhs)


def add(lhs, rhs):
    return _binary_helper(lhs, rhs, 'broadcast_add', '_plus_scalar')


def subtract(lhs, rhs):
    return _binary_helper(lhs, rhs, 'broadcast_sub', '_minus_scalar', '_rminus_scalar')


def multiply(lhs, rhs):
    return _binary_helper(lhs, rhs, 'broadcast_mul', '_mul_scalar')


def divide(lhs, rhs):
    return _binary_helper(lhs, rhs, 'broadcast_div', '_div_scalar', '_rdiv_scalar')


true_divide = divide


def modulo(lhs, rhs):
    return _binary_helper(lhs, rhs, 'broadcast_mod', '_mod_scalar', '_rmod_scalar')


def power(base, exp):
    return _binary_helper(base, exp, 'broadcast_power', '_power_scalar', '_rpower_scalar')


def maximum(lhs, rhs):
    return _binary_helper(lhs, rhs, 'broadcast_maximum', '_maximum_scalar')


def minimum(lhs, rhs):
    return _binary_helper(lhs, rhs, 'broadcast_minimum', '_minimum_scalar')


def equal(lhs, rhs):
    return _binary_helper(lhs, rhs, 'broadcast_equal', '_equal_scalar')


def not_equal(lhs, rhs):
    return _binary_helper(lhs, rhs, 'broadcast_not_equal', '_not_equal_scalar')


def greater(lhs, rhs):
    return _binary_helper(lhs, rhs, 'broadcast_greater', '_greater_scalar', '_lesser_scalar')


def greater_equal(lhs, rhs):
    return _binary_helper(lhs, rhs, 'broadcast_greater_equal', '_greater_equal_scalar', '_lesser_equal_scalar')


def lesser(lhs, rhs):
    return _binary_helper(lhs, rhs, 'broadcast_lesser', '_lesser_scalar', '_greater_scalar')


def lesser_equal(lhs, rhs):
    return _binary_helper(lhs, rhs, 'broadcast_lesser_equal', '_lesser_equal_scalar', '_greater_equal_scalar')


def logical_and(lhs, rhs):
    return _binary_helper(lhs, rhs, 'broadcast_logical_and', '_logical_and_scalar')


def logical_or(lhs, rhs):
    return _binary_helper(lhs, rhs, 'broadcast_logical_or', '_logical_or_scalar')


def logical_xor(lhs, rhs):
    return _binary_helper(lhs, rhs, 'broadcast_logical_xor', '_logical_xor_scalar')


def negative(arr):
    return _op('negative', arr)


class CachedOp:
    """Imperative handle on a Symbol graph (reference ``mx.nd.CachedOp``, src/imperative/cached_op.cc).

    ``op(*inputs, out=None)`` feeds the NDArrays in ``sym.list_inputs()`` order
    through the graph's slot program; under ``autograd.record()`` the run is
    taped like any imperative op, so gradients reach the inputs.
    """

    def __init__(self, sym, flags=()):
        from ..executor import GraphProgram
        self._sym = sym
        self._flags = dict(flags)
        self._prog = GraphProgram(sym)
        self._names = sym.list_inputs()

    def __call__(self, *args, **kwargs):
        from .register import _run, _note_leaves
        out = kwargs.pop('out', None)
        if len(args) != len(self._names):
            raise MXNetError('CachedOp expects %d inputs (%s), got %d' % (len(self._names), self._names, len(args)))
        _note_leaves(list(args))
        names = self._names
        outs = _run(lambda *ts: self._prog.run(dict(zip(names, ts))), [a._data for a in args], {})
        res = [NDArray(o) for o in outs]
        if out is not None:
            outs_l = out if isinstance(out, (list, tuple)) else [out]
            for dst, src in zip(outs_l, res):
                dst[:] = src
            return out
        return res[0] if len(res) == 1 else res
