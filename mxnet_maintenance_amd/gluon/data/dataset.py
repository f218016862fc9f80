"""Datasets (API parity: python/mxnet/gluon/data/dataset.py).

Design: every derived dataset is a *view* of a base dataset.

* ``_IndexView(base, index)`` re-indexes ``base`` through an integer array
  (``filter``, ``shard``, ``take``, ``sample`` all produce one); views of views
  compose their index arrays, so a shard of a filtered dataset is still one
  array lookup away from the storage.
* ``_MapView(base, fn, first_only)`` applies a transform on access
  (``transform`` / ``transform_first``); ``lazy=False`` materialises it.

Samples that are tuples are passed to transforms unpacked (``fn(*sample)``),
like the reference.
"""
import os

import numpy as np

from ... import recordio
from ... import ndarray as nd

__all__ = ['Dataset', 'SimpleDataset', 'ArrayDataset', 'RecordFileDataset']


class Dataset:
    """Random-access collection: implement ``__getitem__`` and ``__len__``."""

    def __getitem__(self, idx):
        raise NotImplementedError('%s does not implement __getitem__' % type(self).__name__)

    def __len__(self):
        raise NotImplementedError('%s does not implement __len__' % type(self).__name__)

    # ------------------------------------------------------------ views
    def _view(self, index):
        return _IndexView(self, np.asarray(index, dtype=np.int64))

    def filter(self, fn):
        """Keep the samples for which ``fn(sample)`` is true (evaluated once, eagerly)."""
        return self._view([i for i in range(len(self)) if fn(self[i])])

    def shard(self, num_shards, index):
        """The ``index``-th of ``num_shards`` contiguous parts; the first ``len % num_shards``
        parts are one sample longer."""
        if num_shards <= 0:
            raise AssertionError('num_shards must be > 0')
        if not 0 <= index < num_shards:
            raise AssertionError('shard index %d out of range [0, %d)' % (index, num_shards))
        sizes = np.full(num_shards, len(self) // num_shards)
        sizes[:len(self) % num_shards] += 1
        start = int(sizes[:index].sum())
        return self._view(np.arange(start, start + int(sizes[index])))

    def take(self, count):
        """The first ``count`` samples (all of them if ``count`` is None or too large)."""
        n = len(self) if count is None else min(count, len(self))
        return self._view(np.arange(n))

    def sample(self, sampler):
        """Re-index through the indices a ``Sampler`` yields (drawn once)."""
        from .sampler import Sampler
        if not isinstance(sampler, Sampler):
            raise TypeError('sample() expects a gluon.data.Sampler, got %s' % type(sampler))
        return _IndexView(self, np.fromiter(iter(sampler), dtype=np.int64), length=len(sampler))

    def transform(self, fn, lazy=True):
        view = _MapView(self, fn, first_only=False)
        return view if lazy else SimpleDataset([view[i] for i in range(len(view))])

    def transform_first(self, fn, lazy=True):
        view = _MapView(self, fn, first_only=True)
        return view if lazy else SimpleDataset([view[i] for i in range(len(view))])


class SimpleDataset(Dataset):
    """Any indexable sequence (list, numpy array, NDArray) as a dataset."""

    def __init__(self, data):
        self._data = data

    def __len__(self):
        return len(self._data)

    def __getitem__(self, idx):
        return self._data[idx]


class _IndexView(Dataset):
    def __init__(self, base, index, length=None):
        if isinstance(base, _IndexView):          # compose instead of nesting
            index = base._index[index]
            base = base._base
        self._base = base
        self._index = index
        self._length = len(index) if length is None else length

    def __len__(self):
        return self._length

    def __getitem__(self, idx):
        return self._base[int(self._index[idx])]


class _MapView(Dataset):
    def __init__(self, base, fn, first_only):
        self._base = base
        self._fn = fn
        self._first_only = first_only

    def __len__(self):
        return len(self._base)

    def __getitem__(self, idx):
        item = self._base[idx]
        if not isinstance(item, tuple):
            return self._fn(item)
        if self._first_only:
            return (self._fn(item[0]),) + item[1:]
        return self._fn(*item)


class ArrayDataset(Dataset):
    """Column-zip of equal-length arrays / datasets: sample i is ``(a[i], b[i], ...)``
    (a bare ``a[i]`` when only one column is given).  1-D NDArrays are kept as host
    numpy columns so per-sample access is not a device round trip."""

    def __init__(self, *args):
        if not args:
            raise AssertionError('ArrayDataset needs at least one array')
        n = len(args[0])
        self._columns = []
        for pos, col in enumerate(args):
            if len(col) != n:
                raise AssertionError('all arrays must have the same length: array 0 has %d, array %d has %d'
                                     % (n, pos, len(col)))
            if isinstance(col, nd.NDArray) and col.ndim == 1:
                col = col.asnumpy()
            self._columns.append(col)
        self._length = n

    # reference attribute name
    @property
    def _data(self):
        return self._columns

    def __len__(self):
        return self._length

    def __getitem__(self, idx):
        if len(self._columns) == 1:
            return self._columns[0][idx]
        return tuple(col[idx] for col in self._columns)


class RecordFileDataset(Dataset):
    """Raw byte records of an indexed RecordIO file (``x.rec`` with its ``x.idx``).

    Picklable for worker processes: the reader handle is reopened after unpickling.
    """

    def __init__(self, filename):
        self.filename = filename
        stem, _ = os.path.splitext(filename)
        self.idx_file = stem + '.idx'
        self._open()

    def _open(self):
        self._reader = recordio.MXIndexedRecordIO(self.idx_file, self.filename, 'r')
        self._keys = list(self._reader.keys)

    def __len__(self):
        return len(self._keys)

    def __getitem__(self, idx):
        return self._reader.read_idx(self._keys[idx])

    def __getstate__(self):
        state = dict(self.__dict__)
        state.pop('_reader', None)
        return state

    def __setstate__(self, state):
        self.__dict__.update(state)
        self._open()


class _DownloadedDataset(Dataset):
    """Base of the vision datasets: ``_get_data`` fills ``_data`` / ``_label`` from files under
    ``root`` (there is no network here, so the files must already exist)."""

    def __init__(self, root, transform):
        super().__init__()
        self._root = os.path.expanduser(root)
        self._transform = transform
        self._data = None
        self._label = None
        os.makedirs(self._root, exist_ok=True)
        self._get_data()

    def __len__(self):
        return len(self._label)

    def __getitem__(self, idx):
        sample = (self._data[idx], self._label[idx])
        return self._transform(*sample) if self._transform is not None else sample

    def _get_data(self):
        raise NotImplementedError('%s must load its files in _get_data()' % type(self).__name__)
