"""DataLoader (parity: python/mxnet/gluon/data/dataloader.py).

Workers: ``num_workers == 0`` loads in the calling thread; ``thread_pool=True``
uses a thread pool (good for PIL/numpy transforms that release the GIL);
otherwise a process pool whose workers batchify into numpy arrays that travel
back through pickling (the parent turns them into NDArrays, optionally in
pinned host memory so the H2D copy onto the MI355X is asynchronous).
``prefetch`` batches (default ``2 * num_workers``) are kept in flight.
"""
import multiprocessing
import os
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from ... import ndarray as nd
from ...ndarray.ndarray import NDArray
from ...context import Context, cpu_pinned
from . import sampler as _sampler

__all__ = ['DataLoader', 'default_batchify_fn', 'default_mp_batchify_fn']


def default_batchify_fn(data):
    """Stack a list of samples into a batch (recursing into tuples)."""
    if isinstance(data[0], NDArray):
        return nd.stack(*data)
    if isinstance(data[0], tuple):
        data = zip(*data)
        return [default_batchify_fn(i) for i in data]
    data = np.asarray(data)
    return nd.array(data, dtype=data.dtype if data.dtype != np.float64 else np.float32)


def default_mp_batchify_fn(data):
    """Worker-side batchify: produces numpy arrays (cheap to ship to the parent)."""
    if isinstance(data[0], NDArray):
        return np.stack([d.asnumpy() for d in data])
    if isinstance(data[0], tuple):
        return [default_mp_batchify_fn(i) for i in zip(*data)]
    data = np.asarray(data)
    return data.astype(np.float32) if data.dtype == np.float64 else data


def _to_nd(x, pin):
    if isinstance(x, np.ndarray):
        return nd.array(x, ctx=cpu_pinned() if pin else None, dtype=x.dtype)
    if isinstance(x, (list, tuple)):
        return [_to_nd(i, pin) for i in x]
    if pin and isinstance(x, NDArray):
        return x.as_in_context(cpu_pinned())
    return x


_worker_dataset = None


def _worker_init(dataset):
    global _worker_dataset
    _worker_dataset = dataset
    os.environ.setdefault('OMP_NUM_THREADS', '1')


def _worker_fn(samples, batchify_fn):
    return batchify_fn([_worker_dataset[i] for i in samples])


def _thread_fn(samples, batchify_fn, dataset):
    return batchify_fn([dataset[i] for i in samples])


class _MultiWorkerIter:
    def __init__(self, pool, batchify_fn, batch_sampler, pin_memory=False, worker_fn=_worker_fn, prefetch=0,
                 dataset=None, timeout=120, to_nd=True):
        self._pool = pool
        self._batchify_fn = batchify_fn
        self._batch_sampler = batch_sampler
        self._data_buffer = {}
        self._rcvd_idx = 0
        self._sent_idx = 0
        self._iter = iter(self._batch_sampler)
        self._worker_fn = worker_fn
        self._pin_memory = pin_memory
        self._dataset = dataset
        self._timeout = timeout
        self._to_nd = to_nd
        for _ in range(prefetch):
            self._push_next()

    def __len__(self):
        return len(self._batch_sampler)

    def _push_next(self):
        r = next(self._iter, None)
        if r is None:
            return
        if self._dataset is None:
            fut = self._pool.apply_async(self._worker_fn, (r, self._batchify_fn))
        else:
            fut = self._pool.submit(self._worker_fn, r, self._batchify_fn, self._dataset)
        self._data_buffer[self._sent_idx] = fut
        self._sent_idx += 1

    def __next__(self):
        self._push_next()
        if self._rcvd_idx == self._sent_idx:
            assert not self._data_buffer, 'Data buffer should be empty at this moment'
            raise StopIteration
        assert self._rcvd_idx < self._sent_idx, 'rcvd_idx must be smaller than sent_idx'
        assert self._rcvd_idx in self._data_buffer, 'fatal error with _push_next, rcvd_idx missing'
        fut = self._data_buffer.pop(self._rcvd_idx)
        batch = fut.get(self._timeout) if hasattr(fut, 'get') else fut.result(self._timeout)
        self._rcvd_idx += 1
        return _to_nd(batch, self._pin_memory) if self._to_nd else batch

    def next(self):
        return self.__next__()

    def __iter__(self):
        return self


class DataLoader:
    """Load mini-batches from a Dataset with optional multi-process/thread workers."""

    def __init__(self, dataset, batch_size=None, shuffle=False, sampler=None, last_batch=None,
                 batch_sampler=None, batchify_fn=None, num_workers=0, pin_memory=False, pin_device_id=0,
                 prefetch=None, thread_pool=False, timeout=120, auto_reload=False):
        self._dataset = dataset
        self._pin_memory = pin_memory
        self._pin_device_id = pin_device_id
        self._thread_pool = thread_pool
        self._timeout = timeout
        if batch_sampler is None:
            if batch_size is None:
                raise ValueError('batch_size must be specified unless batch_sampler is specified')
            if sampler is None:
                sampler = _sampler.RandomSampler(len(dataset)) if shuffle else \
                    _sampler.SequentialSampler(len(dataset))
            elif shuffle:
                raise ValueError('shuffle must not be specified if sampler is specified')
            batch_sampler = _sampler.BatchSampler(sampler, batch_size, last_batch if last_batch else 'keep')
        elif batch_size is not None or shuffle or sampler is not None or last_batch is not None:
            raise ValueError('batch_size, shuffle, sampler and last_batch must not be specified if '
                             'batch_sampler is specified.')
        self._batch_sampler = batch_sampler
        self._num_workers = num_workers if num_workers >= 0 else 0
        self._worker_pool = None
        self._prefetch = max(0, int(prefetch) if prefetch is not None else 2 * self._num_workers)
        self._auto_reload = auto_reload
        if batchify_fn is None:
            self._batchify_fn = default_mp_batchify_fn if (num_workers > 0 and not thread_pool) else \
                default_batchify_fn
        else:
            self._batchify_fn = batchify_fn
        if self._num_workers > 0 and self._auto_reload is False:
            self.refresh()

    def refresh(self):
        self.clean()
        if self._num_workers > 0:
            if self._thread_pool:
                self._worker_pool = ThreadPoolExecutor(self._num_workers)
            else:
                ctx = multiprocessing.get_context('fork')
                self._worker_pool = ctx.Pool(self._num_workers, initializer=_worker_init,
                                             initargs=[self._dataset])

    def clean(self):
        if self._worker_pool is not None:
            if self._thread_pool:
                self._worker_pool.shutdown(wait=False)
            else:
                self._worker_pool.terminate()
            self._worker_pool = None

    def __iter__(self):
        if self._num_workers == 0:
            def same_process_iter():
                for batch in self._batch_sampler:
                    ret = self._batchify_fn([self._dataset[idx] for idx in batch])
                    yield _to_nd(ret, self._pin_memory) if self._pin_memory else ret
            return same_process_iter()
        if self._worker_pool is None:
            self.refresh()
        if self._thread_pool:
            return _MultiWorkerIter(self._worker_pool, self._batchify_fn, self._batch_sampler,
                                    pin_memory=self._pin_memory, worker_fn=_thread_fn, prefetch=self._prefetch,
                                    dataset=self._dataset, timeout=self._timeout,
                                    to_nd=self._pin_memory)
        return _MultiWorkerIter(self._worker_pool, self._batchify_fn, self._batch_sampler,
                                pin_memory=self._pin_memory, worker_fn=_worker_fn, prefetch=self._prefetch,
                                timeout=self._timeout)

    def __len__(self):
        return len(self._batch_sampler)

    def __del__(self):
        try:
            self.clean()
        except Exception:
            pass
