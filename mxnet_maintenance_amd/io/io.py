"""Data iterators (mx.io).

Parity: python/mxnet/io/io.py (DataDesc, DataBatch, DataIter, ResizeIter,
PrefetchingIter, NDArrayIter, MXDataIter) and the C++ iterators of src/io
(CSVIter, MNISTIter, ImageRecordIter, ImageDetRecordIter, LibSVMIter) which
here are implemented over the native RecordIO reader with a decode thread pool.
"""
import csv
import gzip
import os
import queue
import struct
import threading
from collections import namedtuple, OrderedDict

import numpy as np

from ..base import MXNetError
from ..context import cpu
from .. import ndarray as nd
from ..ndarray.ndarray import NDArray
from .image_record import ImageRecordPipeline, DetRecordPipeline

__all__ = ['DataDesc', 'DataBatch', 'DataIter', 'ResizeIter', 'PrefetchingIter', 'NDArrayIter', 'MXDataIter',
           'CSVIter', 'MNISTIter', 'ImageRecordIter', 'ImageRecordUInt8Iter', 'ImageRecordInt8Iter', 'LibSVMIter',
           'ImageDetRecordIter']


class DataDesc(namedtuple('DataDesc', ['name', 'shape'])):
    """Named data description: name, shape, dtype and layout."""

    def __new__(cls, name, shape, dtype=np.float32, layout='NCHW'):
        ret = super().__new__(cls, name, shape)
        ret.dtype = dtype
        ret.layout = layout
        return ret

    def __repr__(self):
        return 'DataDesc[%s,%s,%s,%s]' % (self.name, self.shape, self.dtype, self.layout)

    @staticmethod
    def get_batch_axis(layout):
        if layout is None:
            return 0
        return layout.find('N')

    @staticmethod
    def get_list(shapes, types):
        if types is not None:
            type_dict = dict(types)
            return [DataDesc(x[0], x[1], type_dict[x[0]]) for x in shapes]
        return [DataDesc(x[0], x[1]) for x in shapes]


class DataBatch:
    """A batch of data and labels (plus pad / index / bucket key)."""

    def __init__(self, data, label=None, pad=None, index=None, bucket_key=None, provide_data=None,
                 provide_label=None):
        if data is not None:
            assert isinstance(data, (list, tuple)), 'Data must be list of NDArrays'
        if label is not None:
            assert isinstance(label, (list, tuple)), 'Label must be list of NDArrays'
        self.data = data
        self.label = label
        self.pad = pad
        self.index = index
        self.bucket_key = bucket_key
        self.provide_data = provide_data
        self.provide_label = provide_label

    def __str__(self):
        data_shapes = [d.shape for d in self.data]
        label_shapes = [l.shape for l in self.label] if self.label else None
        return '{}: data shapes: {} label shapes: {}'.format(self.__class__.__name__, data_shapes, label_shapes)


class DataIter:
    """Base iterator: ``reset``, ``next``, ``iter_next``, ``getdata/getlabel/getpad/getindex``."""

    def __init__(self, batch_size=0):
        self.batch_size = batch_size

    def __iter__(self):
        return self

    def reset(self):
        pass

    def next(self):
        if self.iter_next():
            return DataBatch(data=self.getdata(), label=self.getlabel(), pad=self.getpad(), index=self.getindex())
        raise StopIteration

    def __next__(self):
        return self.next()

    def iter_next(self):
        pass

    def getdata(self):
        pass

    def getlabel(self):
        pass

    def getindex(self):
        return None

    def getpad(self):
        pass


class ResizeIter(DataIter):
    """Resize an iterator to ``size`` batches per epoch (resetting the inner one as needed)."""

    def __init__(self, data_iter, size, reset_internal=True):
        super().__init__()
        self.data_iter = data_iter
        self.size = size
        self.reset_internal = reset_internal
        self.cur = 0
        self.current_batch = None
        self.provide_data = data_iter.provide_data
        self.provide_label = data_iter.provide_label
        self.batch_size = data_iter.batch_size
        if hasattr(data_iter, 'default_bucket_key'):
            self.default_bucket_key = data_iter.default_bucket_key

    def reset(self):
        self.cur = 0
        if self.reset_internal:
            self.data_iter.reset()

    def iter_next(self):
        if self.cur == self.size:
            return False
        try:
            self.current_batch = self.data_iter.next()
        except StopIteration:
            self.data_iter.reset()
            self.current_batch = self.data_iter.next()
        self.cur += 1
        return True

    def getdata(self):
        return self.current_batch.data

    def getlabel(self):
        return self.current_batch.label

    def getindex(self):
        return self.current_batch.index

    def getpad(self):
        return self.current_batch.pad


class PrefetchingIter(DataIter):
    """Prefetch batches of one or more iterators on background threads."""

    def __init__(self, iters, rename_data=None, rename_label=None):
        super().__init__()
        if not isinstance(iters, list):
            iters = [iters]
        self.n_iter = len(iters)
        assert self.n_iter > 0
        self.iters = iters
        self.rename_data = rename_data
        self.rename_label = rename_label
        self.batch_size = self.provide_data[0][1][0]
        self.data_ready = [threading.Event() for _ in range(self.n_iter)]
        self.data_taken = [threading.Event() for _ in range(self.n_iter)]
        for e in self.data_taken:
            e.set()
        self.started = True
        self.current_batch = [None for _ in range(self.n_iter)]
        self.next_batch = [None for _ in range(self.n_iter)]

        def prefetch_func(self, i):
            while True:
                self.data_taken[i].wait()
                if not self.started:
                    break
                try:
                    self.next_batch[i] = self.iters[i].next()
                except StopIteration:
                    self.next_batch[i] = None
                self.data_taken[i].clear()
                self.data_ready[i].set()
        self.prefetch_threads = [threading.Thread(target=prefetch_func, args=[self, i], daemon=True)
                                 for i in range(self.n_iter)]
        for thread in self.prefetch_threads:
            thread.start()

    def __del__(self):
        self.started = False
        for e in self.data_taken:
            e.set()

    @property
    def provide_data(self):
        if self.rename_data is None:
            return sum([i.provide_data for i in self.iters], [])
        return sum([[DataDesc(r[x.name], x.shape, x.dtype) if isinstance(x, DataDesc) else DataDesc(*x)
                     for x in i.provide_data] for r, i in zip(self.rename_data, self.iters)], [])

    @property
    def provide_label(self):
        if self.rename_label is None:
            return sum([i.provide_label for i in self.iters], [])
        return sum([[DataDesc(r[x.name], x.shape, x.dtype) if isinstance(x, DataDesc) else DataDesc(*x)
                     for x in i.provide_label] for r, i in zip(self.rename_label, self.iters)], [])

    def reset(self):
        for e in self.data_ready:
            e.wait()
        for i in self.iters:
            i.reset()
        for e in self.data_ready:
            e.clear()
        for e in self.data_taken:
            e.set()

    def iter_next(self):
        for e in self.data_ready:
            e.wait()
        if self.next_batch[0] is None:
            for i in self.next_batch:
                assert i is None, 'Number of entry mismatches between iterators'
            return False
        for batch in self.next_batch:
            assert batch.pad == self.next_batch[0].pad, 'Number of entry mismatches between iterators'
        self.current_batch = DataBatch(sum([batch.data for batch in self.next_batch], []),
                                       sum([batch.label for batch in self.next_batch], []),
                                       self.next_batch[0].pad, self.next_batch[0].index,
                                       provide_data=self.provide_data, provide_label=self.provide_label)
        for e in self.data_ready:
            e.clear()
        for e in self.data_taken:
            e.set()
        return True

    def next(self):
        if self.iter_next():
            return self.current_batch
        raise StopIteration

    def getdata(self):
        return self.current_batch.data

    def getlabel(self):
        return self.current_batch.label

    def getindex(self):
        return self.current_batch.index

    def getpad(self):
        return self.current_batch.pad


def _init_data(data, allow_empty, default_name):
    assert (data is not None) or allow_empty
    if data is None:
        data = []
    if isinstance(data, (np.ndarray, NDArray)):
        data = [data]
    if isinstance(data, list):
        if not allow_empty:
            assert len(data) > 0
        if len(data) == 1:
            data = OrderedDict([(default_name, data[0])])
        else:
            data = OrderedDict([('_%d_%s' % (i, default_name), d) for i, d in enumerate(data)])
    if not isinstance(data, dict):
        raise TypeError('Input must be NDArray, numpy.ndarray, a list of them or dict with them as values')
    for k, v in data.items():
        if not isinstance(v, NDArray):
            try:
                data[k] = nd.array(v)
            except Exception:
                raise TypeError(("Invalid type '%s' for %s, should be NDArray, numpy.ndarray or "
                                 "scipy.sparse.csr.csr_matrix") % (type(v), k))
    return list(sorted(data.items())) if isinstance(data, dict) and not isinstance(data, OrderedDict) else \
        list(data.items())


def _scipy_csr_to_nd(data):
    """scipy.sparse CSR inputs (alone, in a list or dict) become CSRNDArrays."""
    def conv(v):
        if hasattr(v, 'tocsr') and not isinstance(v, nd.NDArray):
            return nd.sparse.csr_matrix(v)
        return v
    if isinstance(data, dict):
        return {k: conv(v) for k, v in data.items()}
    if isinstance(data, (list, tuple)):
        return [conv(v) for v in data]
    return conv(data)


class NDArrayIter(DataIter):
    """Iterate over in-memory NDArrays/numpy arrays (shuffle, pad/discard/roll_over last batch)."""

    def __init__(self, data, label=None, batch_size=1, shuffle=False, last_batch_handle='pad', data_name='data',
                 label_name='softmax_label'):
        super().__init__(batch_size)
        data = _scipy_csr_to_nd(data)
        self.data = _init_data(data, allow_empty=False, default_name=data_name)
        self.label = _init_data(label, allow_empty=True, default_name=label_name)
        if last_batch_handle != 'discard' and any(getattr(v, 'stype', 'default') == 'csr' for _, v in self.data):
            raise NotImplementedError("`NDArrayIter` only supports ``CSRNDArray`` with `last_batch_handle` set to "
                                      "`discard`.")
        self.idx = np.arange(self.data[0][1].shape[0])
        self.shuffle = shuffle
        self.last_batch_handle = last_batch_handle
        self.batch_size = batch_size
        self.cursor = -self.batch_size
        self.num_data = self.idx.shape[0]
        self._cache_data = None
        self._cache_label = None
        self.reset()

    @property
    def provide_data(self):
        return [DataDesc(k, tuple([self.batch_size] + list(v.shape[1:])), v.dtype) for k, v in self.data]

    @property
    def provide_label(self):
        return [DataDesc(k, tuple([self.batch_size] + list(v.shape[1:])), v.dtype) for k, v in self.label]

    def hard_reset(self):
        if self.shuffle:
            self._shuffle_data()
        self.cursor = -self.batch_size
        self._cache_data = None
        self._cache_label = None

    def reset(self):
        if self.shuffle:
            self._shuffle_data()
        if self.last_batch_handle == 'roll_over' and \
                self.num_data - self.batch_size < self.cursor < self.num_data:
            # the cached partial batch is completed from the head of the next epoch
            self.cursor = self.cursor - self.num_data - self.batch_size
        else:
            self.cursor = -self.batch_size

    def iter_next(self):
        self.cursor += self.batch_size
        return self.cursor < self.num_data

    def next(self):
        if not self.iter_next():
            raise StopIteration
        data = self._batchify(self.data)
        label = self._batchify(self.label)
        if data[0].shape[0] != self.batch_size:
            self._cache_data = data
            self._cache_label = label
            raise StopIteration
        return DataBatch(data=data, label=label, pad=self.getpad(), index=None)

    def _getdata(self, data_source, start=None, end=None):
        assert start is not None or end is not None, 'should at least specify start or end'
        start = start if start is not None else 0
        if end is None:
            end = data_source[0][1].shape[0] if data_source else 0
        s = slice(start, end)
        return [x[1][self.idx[s]] if self.shuffle else x[1][s] for x in data_source]

    def _concat(self, first_data, second_data):
        if not first_data or not second_data:
            return first_data if first_data else second_data
        assert len(first_data) == len(second_data), 'data source should contain the same size'
        return [nd.concat(first_data[i], second_data[i], dim=0) for i in range(len(first_data))]

    def _batchify(self, data_source):
        assert self.cursor < self.num_data, 'DataIter needs reset.'
        if self.last_batch_handle == 'roll_over' and -self.batch_size < self.cursor < 0:
            assert self._cache_data is not None or self._cache_label is not None, \
                'next epoch should have cached data'
            cache_data = self._cache_data if self._cache_data is not None else self._cache_label
            second_data = self._getdata(data_source, end=self.cursor + self.batch_size)
            if self._cache_data is not None:
                self._cache_data = None
            else:
                self._cache_label = None
            return self._concat(cache_data, second_data)
        if self.last_batch_handle == 'pad' and self.cursor + self.batch_size > self.num_data:
            # wrap around (several times when the batch is larger than the data set)
            pos = np.arange(self.cursor, self.cursor + self.batch_size) % self.num_data
            if self.shuffle:
                pos = self.idx[pos]
            return [x[1][pos] for x in data_source]
        end_idx = self.cursor + self.batch_size if self.cursor + self.batch_size < self.num_data else self.num_data
        return self._getdata(data_source, self.cursor, end_idx)

    def getdata(self):
        return self._batchify(self.data)

    def getlabel(self):
        return self._batchify(self.label)

    def getpad(self):
        if self.last_batch_handle == 'pad' and self.cursor + self.batch_size > self.num_data:
            return self.cursor + self.batch_size - self.num_data
        if self.last_batch_handle == 'roll_over' and -self.batch_size < self.cursor < 0:
            return -self.cursor
        return 0

    def _shuffle_data(self):
        np.random.shuffle(self.idx)


class MXDataIter(DataIter):
    """Wrapper giving native-style iterators the DataIter interface (parity shim)."""

    def __init__(self, it, data_name='data', label_name='softmax_label', **_):
        super().__init__()
        self._it = it
        self.batch_size = it.batch_size
        self.provide_data = it.provide_data
        self.provide_label = it.provide_label

    def reset(self):
        self._it.reset()

    def next(self):
        return self._it.next()


# ---------------------------------------------------------------------------
# file-backed iterators (src/io/iter_csv.cc, iter_mnist.cc, iter_libsvm.cc)
# ---------------------------------------------------------------------------

class CSVIter(NDArrayIter):
    """Read ``data_csv`` (and optionally ``label_csv``) and iterate in batches."""

    def __init__(self, data_csv, data_shape, label_csv=None, label_shape=(1,), batch_size=1, round_batch=True,
                 dtype='float32', **kwargs):
        ldt = np.dtype(dtype) if np.dtype(dtype).kind in 'iu' else np.float32
        data = np.loadtxt(data_csv, delimiter=',', dtype=ldt, ndmin=2).reshape((-1,) + tuple(data_shape))
        if label_csv is not None:
            label = np.loadtxt(label_csv, delimiter=',', dtype=np.float32, ndmin=2).reshape(
                (-1,) + tuple(label_shape))
        else:
            label = np.zeros((data.shape[0],) + tuple(label_shape), dtype=np.float32)
        if tuple(label_shape) == (1,):
            label = label.reshape(-1)
        super().__init__(nd.array(data, dtype=dtype), nd.array(label), batch_size=batch_size, shuffle=False,
                         last_batch_handle='pad' if round_batch else 'discard')

    # like the reference's native CSVIter: getdata()/getlabel() give the current batch's arrays
    def getdata(self):
        return self._batchify(self.data)[0]

    def getlabel(self):
        return self._batchify(self.label)[0]


def _read_idx(path):
    opener = gzip.open if path.endswith('.gz') else open
    with opener(path, 'rb') as f:
        magic = struct.unpack('>I', f.read(4))[0]
        ndim = magic & 0xff
        dims = struct.unpack('>' + 'I' * ndim, f.read(4 * ndim))
        return np.frombuffer(f.read(), dtype=np.uint8).reshape(dims)


class MNISTIter(NDArrayIter):
    """MNIST idx-format reader (image/label files; optionally flattened)."""

    def __init__(self, image, label, batch_size=128, shuffle=True, flat=False, silent=False, seed=0,
                 num_parts=1, part_index=0, **kwargs):
        img = _read_idx(image).astype(np.float32) / 255.0
        lab = _read_idx(label).astype(np.float32)
        n = img.shape[0] // num_parts
        img = img[part_index * n:(part_index + 1) * n]
        lab = lab[part_index * n:(part_index + 1) * n]
        img = img.reshape(img.shape[0], -1) if flat else img.reshape(img.shape[0], 1, 28, 28)
        if shuffle:
            rs = np.random.RandomState(seed)
            perm = rs.permutation(img.shape[0])
            img, lab = img[perm], lab[perm]
        super().__init__(img, lab, batch_size=batch_size, shuffle=False, last_batch_handle='discard')

    # native iterator accessors: the current batch's single data / label array
    def getdata(self):
        return self._batchify(self.data)[0]

    def getlabel(self):
        return self._batchify(self.label)[0]


def _read_libsvm(path, ncol):
    """(dense rows [n, ncol], leading labels) of a LibSVM text file; malformed ids raise MXNetError."""
    from ..base import MXNetError
    rows, labels = [], []
    with open(path) as f:
        for ln, line in enumerate(f, 1):
            parts = line.strip().split()
            if not parts:
                continue
            labels.append(float(parts[0]))
            row = np.zeros(ncol, dtype=np.float32)
            for p in parts[1:]:
                k, v = p.split(':')
                k = int(k)
                if k < 0 or k >= ncol:
                    raise MXNetError('%s:%d: feature index %d out of range [0, %d)' % (path, ln, k, ncol))
                row[k] = float(v)
            rows.append(row)
    return np.stack(rows) if rows else np.zeros((0, ncol), np.float32), labels


class LibSVMIter(DataIter):
    """LibSVM text format -> CSR data batches (src/io/iter_libsvm.cc)."""

    def __init__(self, data_libsvm, data_shape, label_libsvm=None, label_shape=(1,), batch_size=1,
                 round_batch=True, **kwargs):
        super().__init__(batch_size)
        ncol = int(np.prod(data_shape))
        self._data, labels = _read_libsvm(data_libsvm, ncol)
        if label_libsvm is not None:
            lcol = int(np.prod(label_shape))
            self._label, _ = _read_libsvm(label_libsvm, lcol)
            if tuple(label_shape) == (1,):
                self._label = self._label.reshape(-1)
        else:
            self._label = np.array(labels, dtype=np.float32)
        self._cursor = 0
        self._batch = None
        self.provide_data = [DataDesc('data', (batch_size, ncol))]
        self.provide_label = [DataDesc('softmax_label', (batch_size,) + tuple(self._label.shape[1:]))]
        self._round = round_batch

    def getdata(self):
        return self._batch.data[0] if self._batch is not None else None

    get_data = getdata

    def getlabel(self):
        return self._batch.label[0] if self._batch is not None else None

    def reset(self):
        self._cursor = 0

    def next(self):
        n = self._data.shape[0]
        if self._cursor >= n:
            raise StopIteration
        idx = np.arange(self._cursor, self._cursor + self.batch_size)
        pad = max(0, idx[-1] + 1 - n)
        if pad and not self._round:
            raise StopIteration
        idx = idx % n
        self._cursor += self.batch_size
        data = nd.sparse.csr_matrix(self._data[idx])
        self._batch = DataBatch([data], [nd.array(self._label[idx])], pad=pad)
        return self._batch


# ---------------------------------------------------------------------------
# ImageRecordIter family (src/io/iter_image_recordio_2.cc, image_aug_default.cc):
# native RecordIO prefetch + engine decode tasks + native augmenter (image_record.py)
# ---------------------------------------------------------------------------

class ImageRecordIter(DataIter, ImageRecordPipeline):
    """Iterate over an image .rec file: decode, augment, normalise, batch (NCHW float32 by default).

    Accepts every ImageRecordIter argument of the reference (augmenter, normaliser, parser and
    prefetcher fields; see io/image_record.py)."""

    def __init__(self, path_imgrec=None, data_shape=None, batch_size=None, **kwargs):
        if data_shape is None or batch_size is None:
            raise MXNetError('ImageRecordIter: data_shape and batch_size are required')
        super().__init__(int(batch_size))
        self._setup(path_imgrec, data_shape, int(batch_size), kwargs)
        p = self._p
        self.provide_data = [DataDesc(p['data_name'], self._batch_shape, np.dtype(self.dtype), self.layout)]
        lshape = (self.batch_size,) if self.label_width == 1 else (self.batch_size, self.label_width)
        self.provide_label = [DataDesc(p['label_name'], lshape, np.float32)]
        self.reset()

    def reset(self):
        self._restart()

    def next(self):
        return self._next_batch(DataBatch)


class ImageRecordUInt8Iter(ImageRecordIter):
    """ImageRecordIter producing raw uint8 pixels."""
    _default_dtype = 'uint8'


class ImageRecordInt8Iter(ImageRecordIter):
    """ImageRecordIter producing int8 pixels (value - round(mean), saturated)."""
    _default_dtype = 'int8'


class ImageDetRecordIter(DetRecordPipeline, ImageRecordIter):
    """Detection variant: labels are variable-length object lists padded with -1."""

    def __init__(self, path_imgrec=None, data_shape=None, batch_size=None, label_pad_width=350, **kwargs):
        kwargs.setdefault('label_width', label_pad_width)
        ImageRecordIter.__init__(self, path_imgrec, data_shape, batch_size, **kwargs)
        self._det_setup(label_pad_width)
        self.provide_label = [DataDesc(self._p['label_name'], (self.batch_size, self.label_pad_width),
                                       np.float32)]
