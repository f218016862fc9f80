"""Contrib data iterators: a Gluon ``DataLoader`` exposed as a Module-API ``DataIter``.

Parity: reference python/mxnet/contrib/io.py:24 (``DataLoaderIter``).  The
loader yields ``(data, label)`` pairs; the iterator reports the shapes of the
first batch as ``provide_data`` / ``provide_label`` and pads a short final
batch (``last_batch='keep'``) up to ``batch_size`` so executors bound to the
full shape can consume it, reporting the padding through ``getpad``.
"""
from ..io import DataIter, DataDesc
from .. import ndarray as nd

__all__ = ['DataLoaderIter']


def _pad_to(arr, rows, dtype):
    arr = arr.astype(dtype)
    if arr.shape[0] == rows:
        return arr
    out = nd.zeros((rows,) + tuple(arr.shape[1:]), dtype=dtype, ctx=arr.context)
    out[:arr.shape[0]] = arr
    return out


class DataLoaderIter(DataIter):
    """``DataIter`` over a ``gluon.data.DataLoader`` (``data_name`` / ``label_name`` name the two
    fields of each batch, ``dtype`` is the dtype they are cast to)."""

    def __init__(self, loader, data_name='data', label_name='softmax_label', dtype='float32'):
        super().__init__()
        self._loader = loader
        first_data, first_label = next(iter(loader))
        self.batch_size = first_data.shape[0]
        self.dtype = dtype
        self.provide_data = [DataDesc(data_name, first_data.shape, dtype)]
        self.provide_label = [DataDesc(label_name, first_label.shape, dtype)]
        self._it = None
        self._cur = None
        self.reset()

    def reset(self):
        self._it = iter(self._loader)
        self._cur = None

    def iter_next(self):
        self._cur = next(self._it, None)
        return self._cur is not None

    def getpad(self):
        return self.batch_size - self._cur[0].shape[0]

    def getdata(self):
        return [_pad_to(self._cur[0], self.batch_size, self.dtype)]

    def getlabel(self):
        return [_pad_to(self._cur[1], self.batch_size, self.dtype)]

    def getindex(self):
        return None
