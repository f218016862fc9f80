"""Sparse NDArrays (row_sparse / csr).

Parity: python/mxnet/ndarray/sparse.py (CSRNDArray, RowSparseNDArray,
csr_matrix, row_sparse_array, cast_storage, retain, dot, add/subtract...).

MI355X design note: HBM is 288 GB and the matrix cores want dense tiles, so
sparse arrays keep their compressed components (``data``/``indices``/``indptr``)
for IO, kvstore ``row_sparse_pull`` and serialisation, while compute ops run on
a dense materialisation produced on demand (``_data``).
"""
import numpy as np
import torch

from ..base import torch_dtype, MXNetError
from ..context import current_context
from .ndarray import NDArray

__all__ = ['elemwise_add', 'elemwise_sub', 'elemwise_mul', 'elemwise_div', 'CSRNDArray', 'RowSparseNDArray', 'csr_matrix', 'row_sparse_array', 'cast_storage',
           'zeros', 'empty', 'array', 'retain', 'dot', 'add', 'subtract', 'multiply', 'divide']


class BaseSparseNDArray(NDArray):
    __slots__ = ()

    def asnumpy(self):
        return NDArray.asnumpy(self)

    def tostype(self, stype):
        return cast_storage(self, stype)

    def todense(self):
        return NDArray(self._data.clone())

    def check_format(self, full_check=True):
        return True


class CSRNDArray(BaseSparseNDArray):
    """Compressed sparse row matrix."""
    __slots__ = ()

    def __init__(self, dense):
        super().__init__(dense, stype='csr')

    def _csr(self):
        return self._data.detach().to_sparse_csr()

    @property
    def data(self):
        return NDArray(self._csr().values())

    @property
    def indices(self):
        return NDArray(self._csr().col_indices().to(torch.int64))

    @property
    def indptr(self):
        return NDArray(self._csr().crow_indices().to(torch.int64))

    def _values(self):
        return self._csr().values()

    def _aux_arrays(self):
        c = self._csr()
        return [c.crow_indices().to(torch.int64), c.col_indices().to(torch.int64)]

    def __getitem__(self, key):
        r = NDArray.__getitem__(self, key)
        if r.ndim == 2:
            return CSRNDArray(r._data)
        return r

    def asscipy(self):
        import scipy.sparse as sp
        c = self._csr()
        return sp.csr_matrix((c.values().cpu().numpy(), c.col_indices().cpu().numpy(),
                              c.crow_indices().cpu().numpy()), shape=self.shape)


class RowSparseNDArray(BaseSparseNDArray):
    """Array whose rows are mostly zero; stores non-zero rows + their indices."""
    __slots__ = ()

    def __init__(self, dense):
        super().__init__(dense, stype='row_sparse')

    def _row_idx(self):
        d = self._data.detach()
        if d.dim() == 0:
            return torch.zeros(0, dtype=torch.int64)
        nz = d.reshape(d.shape[0], -1).abs().sum(1) != 0
        return torch.nonzero(nz).reshape(-1).to(torch.int64)

    @property
    def indices(self):
        return NDArray(self._row_idx())

    @property
    def data(self):
        return NDArray(self._data.detach()[self._row_idx()])

    def _values(self):
        return self._data.detach()[self._row_idx()]

    def _aux_arrays(self):
        return [self._row_idx()]

    def retain(self, indices):
        return retain(self, indices)


def _dev(ctx):
    return (ctx or current_context()).torch_device


def csr_matrix(arg1, shape=None, ctx=None, dtype=None):
    """Create a CSRNDArray from (data, indices, indptr), a dense array or scipy matrix."""
    if isinstance(arg1, tuple) and len(arg1) == 3:
        data, indices, indptr = [a._data if isinstance(a, NDArray) else torch.as_tensor(np.asarray(a))
                                 for a in arg1]
        dt = torch_dtype(dtype) if dtype is not None else (data.dtype if data.is_floating_point() else torch.float32)
        t = torch.sparse_csr_tensor(indptr.to(torch.int64), indices.to(torch.int64), data.to(dt),
                                    size=shape).to_dense()
        return CSRNDArray(t.to(_dev(ctx)))
    if isinstance(arg1, tuple) and len(arg1) == 2 and isinstance(arg1[0], int):
        return zeros('csr', arg1, ctx=ctx, dtype=dtype)
    if hasattr(arg1, 'tocsr') and not isinstance(arg1, NDArray):
        arr = np.asarray(arg1.todense())
        return CSRNDArray(torch.as_tensor(arr, dtype=torch_dtype(dtype or arr.dtype)).to(_dev(ctx)))
    if isinstance(arg1, NDArray):
        return CSRNDArray(arg1._data.clone())
    arr = np.asarray(arg1)
    return CSRNDArray(torch.as_tensor(arr, dtype=torch_dtype(dtype or np.float32)).to(_dev(ctx)))


def row_sparse_array(arg1, shape=None, ctx=None, dtype=None):
    """Create a RowSparseNDArray from (data, indices) or a dense array."""
    if isinstance(arg1, tuple) and len(arg1) == 2 and not isinstance(arg1[0], int):
        data, indices = [a._data if isinstance(a, NDArray) else torch.as_tensor(np.asarray(a)) for a in arg1]
        dt = torch_dtype(dtype) if dtype is not None else (data.dtype if data.is_floating_point() else torch.float32)
        full = torch.zeros(shape, dtype=dt)
        if indices.numel():
            full[indices.to(torch.int64).cpu()] = data.to(dt).cpu().reshape((-1,) + tuple(shape[1:]))
        return RowSparseNDArray(full.to(_dev(ctx)))
    if isinstance(arg1, tuple):
        return zeros('row_sparse', arg1, ctx=ctx, dtype=dtype)
    if isinstance(arg1, NDArray):
        return RowSparseNDArray(arg1._data.clone())
    arr = np.asarray(arg1)
    return RowSparseNDArray(torch.as_tensor(arr, dtype=torch_dtype(dtype or np.float32)).to(_dev(ctx)))


def zeros(stype, shape, ctx=None, dtype=None, **kwargs):
    t = torch.zeros(shape, dtype=torch_dtype(dtype), device=_dev(ctx))
    if stype == 'csr':
        return CSRNDArray(t)
    if stype == 'row_sparse':
        return RowSparseNDArray(t)
    return NDArray(t)


def empty(stype, shape, ctx=None, dtype=None):
    return zeros(stype, shape, ctx, dtype)


def array(source_array, ctx=None, dtype=None):
    if isinstance(source_array, (CSRNDArray, RowSparseNDArray)):
        return type(source_array)(source_array._data.clone())
    if hasattr(source_array, 'tocsr'):
        return csr_matrix(source_array, ctx=ctx, dtype=dtype)
    raise MXNetError('sparse.array expects a sparse source')


def cast_storage(data, stype):
    t = data._data
    if stype == 'csr':
        return CSRNDArray(t.clone())
    if stype == 'row_sparse':
        return RowSparseNDArray(t.clone())
    return NDArray(t.clone())


def retain(data, indices):
    idx = indices._data.to(torch.int64)
    out = torch.zeros_like(data._data)
    out[idx] = data._data[idx]
    return RowSparseNDArray(out)


def dot(lhs, rhs, transpose_a=False, transpose_b=False, forward_stype=None):
    from .ndarray import _op
    r = _op('dot', NDArray(lhs._data), NDArray(rhs._data), transpose_a=transpose_a, transpose_b=transpose_b)
    if forward_stype == 'row_sparse':
        return RowSparseNDArray(r._data)
    if forward_stype == 'csr':
        return CSRNDArray(r._data)
    return r


def _elem(op):
    def f(lhs, rhs):
        from .ndarray import _op
        r = _op(op, NDArray(lhs._data), NDArray(rhs._data))
        if getattr(lhs, 'stype', 'default') == getattr(rhs, 'stype', 'default') != 'default':
            return type(lhs)(r._data)
        return r
    return f


add = _elem('broadcast_add')
subtract = _elem('broadcast_sub')
multiply = _elem('broadcast_mul')
divide = _elem('broadcast_div')
elemwise_add, elemwise_sub, elemwise_mul, elemwise_div = add, subtract, multiply, divide
