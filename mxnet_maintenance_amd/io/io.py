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

__all__ = ['DataDesc', 'DataBatch', 'DataIter', 'ResizeIter', 'PrefetchingIter', 'NDArrayIter', 'MXDataIter',
           'CSVIter', 'MNISTIter', 'ImageRecordIter', 'ImageRecordUInt8Iter', 'LibSVMIter', 'ImageDetRecordIter']


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
# ImageRecordIter (src/io/iter_image_recordio_2.cc): native RecordIO read +
# threaded PIL decode/augment + batching, prefetched one batch ahead.
# ---------------------------------------------------------------------------

class ImageRecordIter(DataIter):
    """Iterate over an image .rec file: decode, augment, normalise, batch (NCHW float32 by default)."""

    def __init__(self, path_imgrec, data_shape, batch_size, path_imgidx=None, label_width=1, shuffle=False,
                 rand_crop=False, rand_mirror=False, mean_r=0.0, mean_g=0.0, mean_b=0.0, std_r=1.0, std_g=1.0,
                 std_b=1.0, scale=1.0, resize=-1, preprocess_threads=4, prefetch_buffer=2, round_batch=True,
                 data_name='data', label_name='softmax_label', dtype='float32', layout='NCHW', seed=0,
                 num_parts=1, part_index=0, max_random_scale=1.0, min_random_scale=1.0, **kwargs):
        super().__init__(batch_size)
        from .. import recordio
        self.path = path_imgrec
        self.data_shape = tuple(data_shape)
        self.label_width = label_width
        self.shuffle = shuffle
        self.rand_crop = rand_crop
        self.rand_mirror = rand_mirror
        self.mean = np.array([mean_r, mean_g, mean_b], dtype=np.float32)
        self.std = np.array([std_r, std_g, std_b], dtype=np.float32)
        self.scale = scale
        self.resize = resize
        self.threads = max(1, preprocess_threads)
        self.round_batch = round_batch
        self.dtype = dtype
        self.layout = layout
        self.rng = np.random.RandomState(seed)
        # index: byte offsets of every record
        if path_imgidx and os.path.exists(path_imgidx):
            offs = []
            with open(path_imgidx) as f:
                for line in f:
                    p = line.strip().split('\t')
                    if len(p) == 2:
                        offs.append(int(p[1]))
        else:
            offs = []
            rd = recordio.MXRecordIO(path_imgrec, 'r')
            while True:
                pos = rd.handle.tell()
                if rd.read() is None:
                    break
                offs.append(pos)
            rd.close()
        n = len(offs) // num_parts
        self.offsets = offs[part_index * n:(part_index + 1) * n] if num_parts > 1 else offs
        c, h, w = self.data_shape
        shape = (batch_size, c, h, w) if layout == 'NCHW' else (batch_size, h, w, c)
        self.provide_data = [DataDesc(data_name, shape, np.float32, layout)]
        lshape = (batch_size,) if label_width == 1 else (batch_size, label_width)
        self.provide_label = [DataDesc(label_name, lshape, np.float32)]
        # decode + augmentation run as dependency-engine tasks (src/native/engine.cc worker threads; PIL
        # releases the GIL while decoding): one engine variable per batch slot, and the next batch is
        # pushed as soon as the current one is handed out, so decoding overlaps the training step
        from .. import engine
        self._engine = engine
        self._slot_vars = [engine.new_var('imrec_slot%d' % i) for i in range(batch_size)]
        self._inflight = None
        self.reset()

    def reset(self):
        self._drain()
        order = list(self.offsets)
        if self.shuffle:
            self.rng.shuffle(order)
        self._order = order
        self._cursor = 0
        try:
            from .._lib import _native
            self._reader = _native.RecordPrefetcher(self.path, [int(o) for o in order], 4 * self.batch_size)
        except Exception:
            self._reader = None
            from .. import recordio
            self._pyreader = recordio.MXRecordIO(self.path, 'r')

    def _read_one(self, off):
        if self._reader is not None:
            return self._reader.next()
        self._pyreader.handle.seek(off)
        return self._pyreader.read()

    def _decode(self, rec, seed):
        from ..recordio import unpack
        from ..image import imdecode_np
        header, img = unpack(rec)
        arr = imdecode_np(img, 1)
        rng = np.random.RandomState(seed)
        c, h, w = self.data_shape
        from PIL import Image
        im = Image.fromarray(arr)
        if self.resize > 0:
            W, H = im.size
            s = self.resize / min(W, H)
            im = im.resize((max(1, int(W * s + 0.5)), max(1, int(H * s + 0.5))), Image.BILINEAR)
        W, H = im.size
        if W < w or H < h:
            im = im.resize((max(W, w), max(H, h)), Image.BILINEAR)
            W, H = im.size
        if self.rand_crop:
            x0 = rng.randint(0, W - w + 1)
            y0 = rng.randint(0, H - h + 1)
        else:
            x0, y0 = (W - w) // 2, (H - h) // 2
        im = im.crop((x0, y0, x0 + w, y0 + h))
        a = np.asarray(im, dtype=np.float32)
        if a.ndim == 2:
            a = a[:, :, None].repeat(3, 2)
        if self.rand_mirror and rng.rand() < 0.5:
            a = a[:, ::-1]
        a = (a - self.mean[:a.shape[2]]) / self.std[:a.shape[2]] * self.scale
        if self.layout == 'NCHW':
            a = a.transpose(2, 0, 1)
        label = header.label
        return np.ascontiguousarray(a), label

    def _launch(self):
        """Read the next batch's records and push their decode tasks; None at the end of the epoch."""
        n = len(self._order)
        if self._cursor >= n:
            return None
        bs = self.batch_size
        take = min(bs, n - self._cursor)
        if take < bs and not self.round_batch:
            return None
        recs = [self._read_one(self._order[self._cursor + i]) for i in range(take)]
        pad = bs - take
        if pad:
            recs += [recs[i % take] for i in range(pad)]
        self._cursor += bs
        seeds = self.rng.randint(0, 2 ** 31 - 1, size=len(recs))
        out = [None] * len(recs)

        def task(i, rec, seed):
            out[i] = self._decode(rec, seed)
        for i, (rec, seed) in enumerate(zip(recs, seeds)):
            self._engine.push(lambda i=i, rec=rec, seed=int(seed): task(i, rec, seed),
                              mutable_vars=[self._slot_vars[i]], name='imrec_decode')
        return out, pad

    def _drain(self):
        if getattr(self, '_inflight', None) is not None:
            for v in self._slot_vars:
                try:
                    self._engine.wait_for_var(v)
                except Exception:     # pylint: disable=broad-except
                    pass
        self._inflight = None

    def next(self):
        job = self._inflight if self._inflight is not None else self._launch()
        self._inflight = None
        if job is None:
            raise StopIteration
        out, pad = job
        for v in self._slot_vars[:len(out)]:
            self._engine.wait_for_var(v)      # re-raises a decode task's exception here
        self._inflight = self._launch()       # prefetch: decode the next batch while this one trains
        data = np.stack([o[0] for o in out])
        labels = np.array([np.asarray(o[1], dtype=np.float32).reshape(-1)[:self.label_width] for o in out],
                          dtype=np.float32)
        if self.label_width == 1:
            labels = labels.reshape(-1)
        return DataBatch([nd.array(data, dtype=self.dtype)], [nd.array(labels)], pad=pad)


class ImageRecordUInt8Iter(ImageRecordIter):
    def __init__(self, *args, **kwargs):
        kwargs['dtype'] = 'uint8'
        super().__init__(*args, **kwargs)


class ImageDetRecordIter(ImageRecordIter):
    """Detection variant: labels are variable-length object lists (padded with -1)."""

    def __init__(self, *args, label_pad_width=350, **kwargs):
        kwargs.setdefault('label_width', label_pad_width)
        super().__init__(*args, **kwargs)
        self.label_pad_width = label_pad_width

    def _decode(self, rec, seed):
        a, label = super()._decode(rec, seed)
        lab = np.full(self.label_pad_width, -1.0, dtype=np.float32)
        l = np.asarray(label, dtype=np.float32).reshape(-1)[:self.label_pad_width]
        lab[:len(l)] = l
        return a, lab
