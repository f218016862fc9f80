"""Sparse NDArrays with compressed storage (row_sparse / csr).

Parity: python/mxnet/ndarray/sparse.py (CSRNDArray, RowSparseNDArray,
csr_matrix, row_sparse_array, cast_storage, retain, dot, add/subtract/
multiply/divide, zeros/empty/array) and the storage semantics of
include/mxnet/ndarray.h (kCSRStorage: data + indptr + indices;
kRowSparseStorage: data + row indices).

Storage model.  The compressed components are the array's state:

* ``CSRNDArray``: ``data`` (nnz,), ``indices`` (nnz,) column ids and
  ``indptr`` (rows + 1,), int64;
* ``RowSparseNDArray``: ``data`` (k, *shape[1:]) and ``indices`` (k,) sorted
  row ids.

Sparse-aware operations work on them directly and never build the dense
array: ``dot(csr, dense)`` / ``dot(csr.T, dense)`` (gfx950 kernels in
src/kernels/sparse_kernels.hip; torch sparse ops on the CPU), ``retain``,
row-sparse ``+ - *`` scalar/elementwise, CSR row slicing, kvstore
``row_sparse_pull`` (gathers only the requested rows), lazy optimizer updates
over the rows present in a row-sparse gradient, ``.params`` save/load, scipy
conversion.  Every other operator receives a dense view: reading ``_data``
materialises (and caches) the dense array; since the caller may write
through it, the compressed form is then re-derived from the dense one the
next time it is needed.
"""
import numpy as np
import torch

from ..base import torch_dtype, MXNetError
from ..context import current_context, context_from_torch, Context
from .ndarray import NDArray

__all__ = ['BaseSparseNDArray', 'CSRNDArray', 'RowSparseNDArray', 'csr_matrix', 'row_sparse_array', 'cast_storage',
           'zeros', 'empty', 'array', 'retain', 'dot', 'add', 'subtract', 'multiply', 'divide',
           'elemwise_add', 'elemwise_sub', 'elemwise_mul', 'elemwise_div']

_I64 = torch.int64


def _t(a, dtype=None, device=None):
    """Tensor from NDArray / numpy / list (no copy when already a tensor of that dtype/device)."""
    if isinstance(a, NDArray):
        t = a._data.detach()
    elif isinstance(a, torch.Tensor):
        t = a.detach()
    else:
        t = torch.as_tensor(np.asarray(a))
    if dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    if device is not None and t.device != device:
        t = t.to(device)
    return t


# ------------------------------------------------------------------ dense <-> compressed
def _csr_from_dense(d):
    d = d.detach()
    if d.dim() != 2:
        raise ValueError('csr storage needs a 2-D array, got shape %s' % (tuple(d.shape),))
    mask = d != 0
    counts = mask.sum(1)
    indptr = torch.zeros(d.shape[0] + 1, dtype=_I64, device=d.device)
    torch.cumsum(counts, 0, out=indptr[1:])
    nz = mask.nonzero()                      # row-major: sorted by row, then column
    return d[mask].clone(), nz[:, 1].to(_I64).contiguous(), indptr


def _csr_to_dense(vals, indices, indptr, shape):
    out = torch.zeros(shape, dtype=vals.dtype, device=vals.device)
    if vals.numel():
        counts = indptr[1:] - indptr[:-1]
        rows = torch.repeat_interleave(torch.arange(shape[0], device=vals.device), counts)
        out.index_put_((rows, indices), vals, accumulate=True)
    return out


def _rsp_from_dense(d):
    d = d.detach()
    if d.dim() == 0:
        raise MXNetError('row_sparse storage needs at least 1 dimension')
    idx = (d.reshape(d.shape[0], -1) != 0).any(1).nonzero().reshape(-1).to(_I64)
    return d.index_select(0, idx).clone(), idx


def _rsp_to_dense(vals, indices, shape):
    out = torch.zeros(shape, dtype=vals.dtype, device=vals.device)
    if indices.numel():
        out.index_copy_(0, indices, vals.reshape((-1,) + tuple(shape[1:])))
    return out


class BaseSparseNDArray(NDArray):
    """Common machinery: compressed state + lazily materialised dense view."""
    __slots__ = ('_vals', '_aux', '_shp', '_dense', '_stale')

    _STYPE = None

    def __init__(self, dense=None, ctx=None, dtype=None, stype=None):
        # NDArray-compatible constructor from a dense tensor / array; sparse-native code uses _make
        self._vals = None
        self._aux = ()
        self._shp = ()
        self._dense = None
        self._stale = False
        NDArray.__init__(self, torch.zeros(0) if dense is None else dense, ctx=ctx, dtype=dtype,
                         stype=self._STYPE)

    @classmethod
    def _make(cls, vals, aux, shape):
        r = cls.__new__(cls)
        r._vals = vals
        r._aux = tuple(aux)
        r._shp = tuple(int(s) for s in shape)
        r._dense = None
        r._stale = False
        r._grad = None
        r._grad_req = None
        r._stype = cls._STYPE
        r._fresh_grad = False
        r._arena = None
        return r

    # ---- the dense view every generic operator sees
    @property
    def _data(self):
        if self._dense is None or self._dense.shape != torch.Size(self._shp):
            self._dense = self._densify()
        self._stale = True          # the caller may write through it
        return self._dense

    @_data.setter
    def _data(self, value):
        if not isinstance(value, torch.Tensor):
            value = torch.as_tensor(np.asarray(value))
        self._dense = value
        self._shp = tuple(value.shape)
        self._stale = True

    def _sync(self):
        """Re-derive the compressed form after the dense view may have changed."""
        if self._stale and self._dense is not None:
            self._compress(self._dense)
        self._stale = False

    # ---- metadata without densifying
    @property
    def shape(self):
        return self._shp

    @property
    def size(self):
        n = 1
        for s in self._shp:
            n *= s
        return n

    @property
    def ndim(self):
        return len(self._shp)

    @property
    def dtype(self):
        from ..base import np_dtype
        self._sync()
        return np_dtype(self._vals.dtype)

    @property
    def context(self):
        self._sync()
        hc = getattr(self, '_host_ctx', None)
        if hc is not None and self._vals.device.type == 'cpu':
            return hc           # cpu(k), k > 0: same host memory, reported context (see _tag_host_ctx)
        return context_from_torch(self._vals.device)

    ctx = context

    @property
    def device(self):
        return self.context

    def _values(self):
        self._sync()
        return self._vals

    def _aux_arrays(self):
        self._sync()
        return list(self._aux)

    def todense(self):
        self._sync()
        return NDArray(self._densify())

    def tostype(self, stype):
        return cast_storage(self, stype)

    def asnumpy(self):
        self._sync()
        return NDArray(self._densify()).asnumpy()

    def _keep_ctx(self, r):
        hc = getattr(self, '_host_ctx', None)
        if hc is not None:
            r._host_ctx = hc
        return r

    def copy(self):
        self._sync()
        return self._keep_ctx(type(self)._make(self._vals.clone(), [a.clone() for a in self._aux], self._shp))

    def __deepcopy__(self, memo):
        return self.copy()

    def detach(self):
        self._sync()
        return type(self)._make(self._vals.detach(), list(self._aux), self._shp)

    def astype(self, dtype, copy=True):
        self._sync()
        td = torch_dtype(dtype)
        if not copy and td == self._vals.dtype:
            return self
        return self._keep_ctx(type(self)._make(self._vals.to(td), [a.clone() for a in self._aux], self._shp))

    def as_in_context(self, context):
        self._sync()
        if self.context == context:
            return self
        dev = context.torch_device
        r = type(self)._make(self._vals.to(dev), [a.to(dev) for a in self._aux], self._shp)
        if context.device_typeid == 1 and context.device_id != 0:
            r._host_ctx = context
        return r

    as_in_ctx = as_in_context

    def copyto(self, other):
        self._sync()
        if isinstance(other, Context):
            return self.as_in_context(other).copy() if other == self.context else self.as_in_context(other)
        if isinstance(other, BaseSparseNDArray):
            if other.shape != self.shape:
                raise MXNetError('copyto: shape mismatch %s vs %s' % (self.shape, other.shape))
            if other._STYPE == self._STYPE:
                dev = other.context.torch_device
                other._vals = self._vals.to(dev, other._vals.dtype if other._vals is not None else None)
                other._aux = tuple(a.to(dev) for a in self._aux)
                other._dense = None
                other._stale = False
                return other
            other._data = self._densify().to(other.context.torch_device)
            return other
        return NDArray.copyto(NDArray(self._densify()), other)

    def check_format(self, full_check=True):
        self._sync()
        self._check(full_check)

    @property
    def data(self):
        self._sync()
        return NDArray(self._vals)

    def __repr__(self):
        return '\n<%s %s @%s>' % (self.__class__.__name__, 'x'.join(str(s) for s in self._shp), self.context)

    # elementwise arithmetic keeps the storage type where the result stays sparse
    def __add__(self, other):
        return add(self, other)

    def __sub__(self, other):
        return subtract(self, other)

    def __mul__(self, other):
        return multiply(self, other)

    def __truediv__(self, other):
        return divide(self, other)

    def __neg__(self):
        return multiply(self, -1.0)

    # comparisons / arithmetic with a scalar: the result stays sparse when the op maps 0 to 0
    # (reference: FInferStorageType of the *_scalar operators), dense otherwise
    def _scalar_op(self, scalar, fn):
        from .. import _state
        if not isinstance(scalar, (int, float, np.number)) or _state.STATE.recording:
            return None
        self._sync()
        dt = self._vals.dtype
        zero = fn(torch.zeros((), dtype=dt), scalar)
        if float(zero) == 0.0:
            return type(self)._make(fn(self._vals, scalar).to(dt), [a.clone() for a in self._aux], self._shp)
        return NDArray(fn(self._densify(), scalar).to(dt))

    def _cmp(self, other, fn, name):
        r = self._scalar_op(other, fn)
        if r is not None:
            return r
        return getattr(NDArray, name)(NDArray(self._data), NDArray(other._data) if isinstance(other, NDArray)
                                      else other)

    @property
    def _num_aux(self):
        return len(self._aux) if self._aux else (2 if self._STYPE == 'csr' else 1)

    def __reduce__(self):
        self._sync()
        return (_rebuild_sparse, (self._STYPE, _np_of(self._vals), [_np_of(a) for a in self._aux], self._shp))

    def __getstate__(self):
        return None

    def __eq__(self, other):
        return self._cmp(other, torch.eq, '__eq__')

    def __ne__(self, other):
        return self._cmp(other, torch.ne, '__ne__')

    def __gt__(self, other):
        return self._cmp(other, torch.gt, '__gt__')

    def __ge__(self, other):
        return self._cmp(other, torch.ge, '__ge__')

    def __lt__(self, other):
        return self._cmp(other, torch.lt, '__lt__')

    def __le__(self, other):
        return self._cmp(other, torch.le, '__le__')

    __hash__ = NDArray.__hash__

    def __iadd__(self, other):
        return self._assign(add(self, other))

    def __isub__(self, other):
        return self._assign(subtract(self, other))

    def __imul__(self, other):
        return self._assign(multiply(self, other))

    def __itruediv__(self, other):
        return self._assign(divide(self, other))

    def _assign(self, r):
        if isinstance(r, type(self)):
            r._sync()
            self._vals, self._aux, self._shp = r._vals, r._aux, r._shp
            self._dense, self._stale = None, False
        else:
            self._data = r._data
        return self


class CSRNDArray(BaseSparseNDArray):
    """Compressed sparse row matrix: ``data`` (nnz,), ``indices`` (nnz,) columns, ``indptr`` (rows + 1,)."""
    __slots__ = ()
    _STYPE = 'csr'

    def _densify(self):
        return _csr_to_dense(self._vals, self._aux[1], self._aux[0], self._shp)

    def _compress(self, d):
        self._vals, idx, ptr = _csr_from_dense(d)
        self._aux = (ptr, idx)
        self._shp = tuple(d.shape)

    def _check(self, full):
        ptr, idx = self._aux
        if ptr.numel() != self._shp[0] + 1 or idx.numel() != self._vals.numel():
            raise MXNetError('csr: inconsistent aux array lengths')
        if full and ptr.numel():
            if int(ptr[0]) != 0 or bool((ptr[1:] < ptr[:-1]).any()) or int(ptr[-1]) != idx.numel():
                raise MXNetError('csr: indptr must start at 0, be non-decreasing and end at nnz')
            if idx.numel() and (bool((idx < 0).any()) or bool((idx >= self._shp[1]).any())):
                raise MXNetError('csr: column index out of range')
            if idx.numel() > 1:
                # column indices strictly increasing inside every row
                counts = ptr[1:] - ptr[:-1]
                rows = torch.repeat_interleave(torch.arange(self._shp[0], device=idx.device), counts)
                same_row = rows[1:] == rows[:-1]
                if bool(((idx[1:] <= idx[:-1]) & same_row).any()):
                    raise MXNetError('csr: column indices must be sorted and unique within each row')

    @property
    def indices(self):
        self._sync()
        return NDArray(self._aux[1])

    @property
    def indptr(self):
        self._sync()
        return NDArray(self._aux[0])

    def __getitem__(self, key):
        self._sync()
        if isinstance(key, int):
            key = slice(key, key + 1)
        if isinstance(key, slice) and key.step in (None, 1):
            start, stop, _ = key.indices(self._shp[0])
            stop = max(start, stop)
            ptr, idx = self._aux
            lo, hi = int(ptr[start]), int(ptr[stop])
            return CSRNDArray._make(self._vals[lo:hi].clone(), [ptr[start:stop + 1] - lo, idx[lo:hi].clone()],
                                    (stop - start, self._shp[1]))
        r = NDArray.__getitem__(NDArray(self._densify()), key)
        return r

    def asscipy(self):
        import scipy.sparse as sp
        self._sync()
        ptr, idx = self._aux
        v = self._vals.float() if self._vals.dtype == torch.bfloat16 else self._vals
        return sp.csr_matrix((v.cpu().numpy(), idx.cpu().numpy(), ptr.cpu().numpy()), shape=self._shp)


class RowSparseNDArray(BaseSparseNDArray):
    """Mostly-zero rows: ``data`` holds the stored rows, ``indices`` their (sorted) row ids."""
    __slots__ = ()
    _STYPE = 'row_sparse'

    def _densify(self):
        return _rsp_to_dense(self._vals, self._aux[0], self._shp)

    def _compress(self, d):
        self._vals, idx = _rsp_from_dense(d)
        self._aux = (idx,)
        self._shp = tuple(d.shape)

    def _check(self, full):
        idx, = self._aux
        if idx.numel() != (self._vals.shape[0] if self._vals.dim() else 0):
            raise MXNetError('row_sparse: data rows and indices differ in length')
        if full and idx.numel():
            if bool((idx[1:] <= idx[:-1]).any()):
                raise MXNetError('row_sparse: indices must be strictly increasing')
            if int(idx.min()) < 0 or int(idx.max()) >= self._shp[0]:
                raise MXNetError('row_sparse: row index out of range')

    @property
    def indices(self):
        self._sync()
        return NDArray(self._aux[0])

    def retain(self, indices):
        return retain(self, indices)

    def __getitem__(self, key):
        if isinstance(key, slice) and key == slice(None):
            return self
        # a view of the current dense image (earlier writes through it included); writes into the
        # view (``out=x[i]``) land in this array, whose rows are re-derived at the next sync
        return NDArray.__getitem__(NDArray(self._data), key)


def _np_of(t):
    t = t.detach().cpu()
    return (t.float() if t.dtype == torch.bfloat16 else t).numpy()


def _rebuild_sparse(stype, vals, aux, shape):
    cls = CSRNDArray if stype == 'csr' else RowSparseNDArray
    return cls._make(torch.from_numpy(np.array(vals)), [torch.from_numpy(np.array(a)) for a in aux], shape)


# ------------------------------------------------------------------ constructors
def _tagged(fn):
    """Constructors report a requested ``cpu(k)`` context (k > 0) on their result."""
    import functools

    @functools.wraps(fn)
    def f(*args, **kwargs):
        r = fn(*args, **kwargs)
        ctx = kwargs.get('ctx')
        if ctx is None:
            names = fn.__code__.co_varnames[:fn.__code__.co_argcount]
            if 'ctx' in names and len(args) > names.index('ctx'):
                ctx = args[names.index('ctx')]
        if isinstance(ctx, str):
            ctx = Context(ctx)
        if (isinstance(r, BaseSparseNDArray) and isinstance(ctx, Context) and ctx.device_typeid == 1
                and ctx.device_id != 0):
            r._host_ctx = ctx
        return r
    return f


def _dev(ctx):
    return (ctx or current_context()).torch_device


def _default_dtype(t, dtype, src=None):
    """The dtype a sparse constructor gives its values: ``dtype``, else the source's own dtype when
    it is an NDArray / numpy array / scipy matrix, else float32 (reference: sparse.py
    _prepare_default_dtype)."""
    if dtype is not None:
        return torch_dtype(dtype)
    if src is not None:
        if isinstance(src, (NDArray, np.ndarray)) or hasattr(src, 'tocsr'):
            return t.dtype
        return torch.float32
    return t.dtype if t.is_floating_point() else torch.float32


@_tagged
def csr_matrix(arg1, shape=None, ctx=None, dtype=None):
    """CSRNDArray from ``(data, indices, indptr)``, ``(M, N)`` (empty), a dense array or a scipy matrix."""
    dev = _dev(ctx)
    if isinstance(arg1, tuple) and len(arg1) == 3:
        data = _t(arg1[0], device=dev)
        data = data.to(_default_dtype(data, dtype, arg1[0]))
        indices = _t(arg1[1], _I64, dev)
        indptr = _t(arg1[2], _I64, dev)
        if shape is None:
            if not indices.numel():
                raise ValueError('csr_matrix: cannot infer the number of columns without indices; pass shape')
            shape = (indptr.numel() - 1, int(indices.max()) + 1)
        r = CSRNDArray._make(data.reshape(-1).clone(), [indptr.clone(), indices.clone()], shape)
        r._check(False)
        return r
    if isinstance(arg1, tuple) and len(arg1) == 2 and all(isinstance(s, (int, np.integer)) for s in arg1):
        if shape is not None and tuple(shape) != tuple(arg1):
            raise ValueError('csr_matrix: shape %s does not match %s' % (shape, arg1))
        return zeros('csr', arg1, ctx=ctx, dtype=dtype)
    if isinstance(arg1, tuple) and len(arg1) == 2:
        # scipy-style (data, (row, col)) COO definition
        data, (row, col) = arg1
        d = _t(data, device=dev)
        d = d.to(_default_dtype(d, dtype, data))
        dense = torch.zeros(shape, dtype=d.dtype, device=dev)
        dense.index_put_((_t(row, _I64, dev), _t(col, _I64, dev)), d, accumulate=True)
        return cast_storage(NDArray(dense), 'csr')
    if shape is not None and hasattr(arg1, 'shape') and tuple(arg1.shape) != tuple(shape):
        raise ValueError('csr_matrix: shape %s does not match the source array %s' % (shape, tuple(arg1.shape)))
    if isinstance(arg1, CSRNDArray):
        r = arg1.astype(dtype) if dtype is not None else arg1.copy()
        return r.as_in_context(ctx) if ctx is not None else r
    if hasattr(arg1, 'tocsr') and not isinstance(arg1, NDArray):
        m = arg1.tocsr(copy=True)
        m.sum_duplicates()          # canonical form: duplicates summed, column indices sorted per row
        m.sort_indices()
        dt = torch_dtype(dtype) if dtype is not None else torch_dtype(m.dtype if m.dtype.kind == 'f' else np.float32)
        return CSRNDArray._make(torch.as_tensor(m.data).to(dev, dt), [torch.as_tensor(m.indptr).to(dev, _I64),
                                                                      torch.as_tensor(m.indices).to(dev, _I64)],
                                m.shape)
    d = _t(arg1, device=dev)
    d = d.to(_default_dtype(d, dtype, arg1))
    return cast_storage(NDArray(d), 'csr')


@_tagged
def row_sparse_array(arg1, shape=None, ctx=None, dtype=None):
    """RowSparseNDArray from ``(data, indices)``, a shape tuple (empty) or a dense array."""
    dev = _dev(ctx)
    if isinstance(arg1, tuple) and len(arg1) == 2 and not isinstance(arg1[0], (int, np.integer)):
        data = _t(arg1[0], device=dev)
        data = data.to(_default_dtype(data, dtype, arg1[0]))
        indices = _t(arg1[1], _I64, dev).reshape(-1)
        if shape is None:
            shape = (int(indices.max()) + 1 if indices.numel() else 0,) + tuple(data.shape[1:])
        data = data.reshape((indices.numel(),) + tuple(shape[1:]))
        # kept as given: unsorted / negative / out-of-range indices are an invalid format that
        # check_format reports (reference: RowSparseNDArray format checks)
        return RowSparseNDArray._make(data.clone(), [indices.clone()], shape)
    if isinstance(arg1, tuple):
        if shape is not None and tuple(shape) != tuple(arg1):
            raise ValueError('row_sparse_array: shape %s does not match %s' % (shape, arg1))
        return zeros('row_sparse', arg1, ctx=ctx, dtype=dtype)
    if shape is not None and hasattr(arg1, 'shape') and tuple(arg1.shape) != tuple(shape):
        raise ValueError('row_sparse_array: shape %s does not match the source array %s'
                         % (shape, tuple(arg1.shape)))
    if isinstance(arg1, RowSparseNDArray):
        r = arg1.astype(dtype) if dtype is not None else arg1.copy()
        return r.as_in_context(ctx) if ctx is not None else r
    d = _t(arg1, device=dev)
    d = d.to(_default_dtype(d, dtype, arg1))
    return cast_storage(NDArray(d), 'row_sparse')


@_tagged
def zeros(stype, shape, ctx=None, dtype=None, **kwargs):
    if stype not in ('csr', 'row_sparse', 'default'):
        raise ValueError('unknown storage type %s' % stype)
    dev = _dev(ctx)
    dt = torch_dtype(dtype) if dtype is not None else torch.float32
    shape = (shape,) if isinstance(shape, int) else tuple(shape)
    if stype == 'csr':
        return CSRNDArray._make(torch.zeros(0, dtype=dt, device=dev),
                                [torch.zeros(shape[0] + 1, dtype=_I64, device=dev),
                                 torch.zeros(0, dtype=_I64, device=dev)], shape)
    if stype == 'row_sparse':
        return RowSparseNDArray._make(torch.zeros((0,) + shape[1:], dtype=dt, device=dev),
                                      [torch.zeros(0, dtype=_I64, device=dev)], shape)
    return NDArray(torch.zeros(shape, dtype=dt, device=dev))


def empty(stype, shape, ctx=None, dtype=None):
    return zeros(stype, shape, ctx, dtype)


@_tagged
def array(source_array, ctx=None, dtype=None):
    """Sparse array from a sparse NDArray or a scipy sparse matrix (copies)."""
    if isinstance(source_array, CSRNDArray):
        r = source_array.astype(dtype) if dtype is not None else source_array.copy()
        return r.as_in_context(ctx) if ctx is not None else r
    if isinstance(source_array, RowSparseNDArray):
        r = source_array.astype(dtype) if dtype is not None else source_array.copy()
        return r.as_in_context(ctx) if ctx is not None else r
    if hasattr(source_array, 'tocsr'):
        return csr_matrix(source_array, ctx=ctx, dtype=dtype)
    raise MXNetError('sparse.array expects a sparse source, got %s' % type(source_array))


def cast_storage(data, stype):
    """Convert between 'default', 'csr' and 'row_sparse' storage."""
    cur = getattr(data, 'stype', 'default')
    if cur == stype:
        return data.copy()
    if isinstance(data, BaseSparseNDArray):
        data._sync()
        dense = data._densify()
    else:
        dense = data._data.detach()
    if stype == 'default':
        return NDArray(dense.clone() if not isinstance(data, BaseSparseNDArray) else dense)
    if stype == 'csr':
        v, idx, ptr = _csr_from_dense(dense)
        return CSRNDArray._make(v, [ptr, idx], dense.shape)
    if stype == 'row_sparse':
        v, idx = _rsp_from_dense(dense)
        return RowSparseNDArray._make(v, [idx], dense.shape)
    raise MXNetError('unknown storage type %s' % stype)


def retain(data, indices=None, **kwargs):
    """Keep only the rows of a row_sparse array whose ids are in ``indices`` (compressed in, compressed out)."""
    if kwargs:
        raise MXNetError('retain: unknown argument(s) %s' % sorted(kwargs))
    if not isinstance(data, RowSparseNDArray) or indices is None:
        raise MXNetError('retain expects a row_sparse array and the row indices to keep')
    data._sync()
    idx, = data._aux
    want = _t(indices, _I64, idx.device).reshape(-1)
    keep = torch.isin(idx, want)
    return RowSparseNDArray._make(data._vals[keep].clone(), [idx[keep].clone()], data.shape)


# ------------------------------------------------------------------ dot
def _kernels():
    from ..ops import kernels as K
    return K if (K.available() and K.enabled()) else None


def _csr_dot_dense(a, rhs, transpose_a):
    """csr . dense -> dense  |  csr^T . dense -> row_sparse (rows = the columns a stores)."""
    a._sync()
    ptr, idx = a._aux
    vals = a._vals
    M, K = a.shape
    rhs = rhs.contiguous()
    if rhs.dim() == 1:
        out = _csr_dot_dense(a, rhs.reshape(-1, 1), transpose_a)
        if isinstance(out, RowSparseNDArray):
            return RowSparseNDArray._make(out._vals.reshape(-1), list(out._aux), (out.shape[0],))
        return NDArray(out._data.reshape(-1))
    N = rhs.shape[1]
    dt = torch.promote_types(vals.dtype, rhs.dtype)
    vals = vals.to(dt)
    rhs = rhs.to(dt)
    lib = _kernels()
    use_hip = lib is not None and vals.is_cuda and dt in (torch.float32, torch.float16, torch.bfloat16)
    if not transpose_a:
        if rhs.shape[0] != K:
            raise MXNetError('dot(csr, dense): shape mismatch %s x %s' % (a.shape, tuple(rhs.shape)))
        out = torch.empty((M, N), dtype=dt, device=vals.device)
        if use_hip:
            from ..ops.kernel_fns import _DT, _stream
            lib.lib().csr_dot_dense(_DT[dt], ptr.data_ptr(), idx.data_ptr(), vals.contiguous().data_ptr(),
                                    rhs.data_ptr(), out.data_ptr(), M, K, N, _stream())
        else:
            import warnings
            with warnings.catch_warnings():
                warnings.simplefilter('ignore')       # "sparse CSR support is in beta"
                sp = torch.sparse_csr_tensor(ptr, idx, vals, size=(M, K))
                out = torch.sparse.mm(sp, rhs) if vals.numel() else out.zero_()
        return NDArray(out)
    if rhs.shape[0] != M:
        raise MXNetError('dot(csr.T, dense): shape mismatch %s^T x %s' % (a.shape, tuple(rhs.shape)))
    rows = torch.unique(idx)                              # sorted output row ids
    if use_hip:
        from ..ops.kernel_fns import _DT, _stream
        slot = torch.full((K,), -1, dtype=_I64, device=vals.device)
        slot[rows] = torch.arange(rows.numel(), device=vals.device)
        acc = torch.zeros((rows.numel(), N), dtype=torch.float32, device=vals.device)
        lib.lib().csrT_dot_dense(_DT[dt], ptr.data_ptr(), idx.data_ptr(), vals.contiguous().data_ptr(),
                                 rhs.data_ptr(), slot.data_ptr(), acc.data_ptr(), M, K, N, _stream())
        return RowSparseNDArray._make(acc.to(dt), [rows], (K, N))
    counts = ptr[1:] - ptr[:-1]
    src_rows = torch.repeat_interleave(torch.arange(M, device=vals.device), counts)
    pos = torch.searchsorted(rows, idx)
    acc = torch.zeros((rows.numel(), N), dtype=torch.float32, device=vals.device)
    acc.index_add_(0, pos, vals.float().unsqueeze(1) * rhs.float().index_select(0, src_rows))
    return RowSparseNDArray._make(acc.to(dt), [rows], (K, N))


def dot(lhs, rhs, transpose_a=False, transpose_b=False, forward_stype=None):
    """Sparse-aware dot: csr . dense (and csr^T . dense -> row_sparse) on compressed storage."""
    from .ndarray import _op
    from .. import _state
    if _state.STATE.recording:
        r = _op('dot', NDArray(lhs._data), NDArray(rhs._data), transpose_a=transpose_a, transpose_b=transpose_b)
    elif isinstance(lhs, CSRNDArray) and not isinstance(rhs, BaseSparseNDArray) and not transpose_b:
        r = _csr_dot_dense(lhs, rhs._data.detach(), transpose_a)
    elif isinstance(lhs, CSRNDArray) and isinstance(rhs, RowSparseNDArray) and not transpose_b:
        r = _csr_dot_dense(lhs, rhs._densify(), transpose_a)
    else:
        r = _op('dot', NDArray(lhs._data), NDArray(rhs._data), transpose_a=transpose_a, transpose_b=transpose_b)
    if forward_stype is not None and getattr(r, 'stype', 'default') != forward_stype:
        r = cast_storage(r, forward_stype)
    return r


# ------------------------------------------------------------------ elementwise
def _rsp_union(a, b, fn):
    a._sync()
    b._sync()
    ia, ib = a._aux[0], b._aux[0]
    rows = torch.unique(torch.cat([ia, ib]))
    tail = tuple(a.shape[1:])
    dt = torch.promote_types(a._vals.dtype, b._vals.dtype)
    va = torch.zeros((rows.numel(),) + tail, dtype=dt, device=rows.device)
    vb = torch.zeros_like(va)
    va.index_copy_(0, torch.searchsorted(rows, ia), a._vals.to(dt))
    vb.index_copy_(0, torch.searchsorted(rows, ib), b._vals.to(dt))
    return RowSparseNDArray._make(fn(va, vb), [rows], a.shape)


def _elem(op, torch_fn, zero_preserving_scalar):
    def f(lhs, rhs):
        from .ndarray import _op
        from .. import _state
        if _state.STATE.recording:
            # autograd: the dense views carry the graph (compressed values are not differentiable leaves)
            lt = lhs._data if isinstance(lhs, NDArray) else torch.as_tensor(lhs)
            rt = rhs._data if isinstance(rhs, NDArray) else rhs
            if isinstance(rt, torch.Tensor):
                return _op(op, NDArray(lt), NDArray(rt))
            return NDArray(torch_fn(lt, rt))
        if isinstance(lhs, RowSparseNDArray) and isinstance(rhs, RowSparseNDArray) and lhs.shape == rhs.shape \
                and op in ('broadcast_add', 'broadcast_sub'):
            return _rsp_union(lhs, rhs, torch_fn)
        if isinstance(lhs, RowSparseNDArray) and isinstance(rhs, RowSparseNDArray) and lhs.shape == rhs.shape \
                and op == 'broadcast_mul':
            lhs._sync()
            rhs._sync()
            keep = torch.isin(lhs._aux[0], rhs._aux[0])
            rows = lhs._aux[0][keep]
            vb = rhs._vals.index_select(0, torch.searchsorted(rhs._aux[0], rows))
            return RowSparseNDArray._make(lhs._vals[keep] * vb, [rows], lhs.shape)
        if isinstance(lhs, BaseSparseNDArray) and isinstance(rhs, (int, float)) and zero_preserving_scalar:
            lhs._sync()
            return type(lhs)._make(torch_fn(lhs._vals, rhs), [a.clone() for a in lhs._aux], lhs.shape)
        if isinstance(lhs, CSRNDArray) and isinstance(rhs, CSRNDArray) and lhs.shape == rhs.shape:
            r = _op(op, NDArray(lhs._densify()), NDArray(rhs._densify()))
            return cast_storage(r, 'csr')
        lt = lhs._data if isinstance(lhs, NDArray) else lhs
        rt = rhs._data if isinstance(rhs, NDArray) else rhs
        if not isinstance(lt, torch.Tensor) or not isinstance(rt, torch.Tensor):
            return NDArray(torch_fn(lt, rt) if isinstance(lt, torch.Tensor) else torch_fn(torch.as_tensor(lt), rt))
        return _op(op, NDArray(lt), NDArray(rt))
    f.__name__ = op
    return f


add = _elem('broadcast_add', torch.add, False)
subtract = _elem('broadcast_sub', torch.sub, False)
multiply = _elem('broadcast_mul', torch.mul, True)
divide = _elem('broadcast_div', torch.div, True)
elemwise_add, elemwise_sub, elemwise_mul, elemwise_div = add, subtract, multiply, divide


def __getattr__(name):
    # every other operator is available in this namespace with dense semantics (reference: the
    # generated mx.nd.sparse.<op> functions accept sparse inputs through storage fallback)
    from .. import ndarray as nd
    if name.startswith('__'):
        raise AttributeError(name)
    try:
        return getattr(nd, name)
    except AttributeError:
        raise AttributeError("module 'sparse' has no attribute %r" % name) from None
