"""DataLoader (API parity: python/mxnet/gluon/data/dataloader.py).

Worker modes:

* ``num_workers == 0``: batches are built in the calling thread;
* ``thread_pool=True``: a thread pool (PIL / numpy transforms release the GIL);
* otherwise worker *processes* started from a ``forkserver`` (never a bare
  ``fork`` of a process that already runs torch threads or a HIP runtime --
  that is what deadlocked the previous pool).  Each worker holds its own copy
  of the dataset, batchifies into numpy arrays and ships them back through
  POSIX shared memory: one segment per batch, every array of the batch packed
  into it, only a small descriptor goes through the result queue.  The parent
  copies the arrays out (into pinned host memory when ``pin_memory``, so the
  host-to-MI355X copy can be asynchronous) and unlinks the segment.

``prefetch`` batches (default ``2 * num_workers``) are in flight; results are
delivered in sampler order.  Workers are shut down (sentinel, join, then
terminate) when the loader is cleaned up or garbage collected.
"""
import multiprocessing
import os
import queue as _queue
import threading
from concurrent.futures import ThreadPoolExecutor
from multiprocessing import shared_memory

import numpy as np

from ... import ndarray as nd
from ...ndarray.ndarray import NDArray
from ...context import cpu_pinned
from . import sampler as _sampler

__all__ = ['DataLoader', 'default_batchify_fn', 'default_mp_batchify_fn']


def default_batchify_fn(data):
    """Stack a list of samples into a batch (recursing into tuples)."""
    if isinstance(data[0], NDArray):
        return nd.stack(*data)
    if isinstance(data[0], tuple):
        return [default_batchify_fn(list(col)) for col in zip(*data)]
    arr = np.asarray(data)
    return nd.array(arr, dtype=arr.dtype if arr.dtype != np.float64 else np.float32)


def default_mp_batchify_fn(data):
    """Worker-side batchify: numpy arrays (shipped to the parent through shared memory)."""
    if isinstance(data[0], NDArray):
        return np.stack([d.asnumpy() for d in data])
    if isinstance(data[0], tuple):
        return [default_mp_batchify_fn(list(col)) for col in zip(*data)]
    arr = np.asarray(data)
    return arr.astype(np.float32) if arr.dtype == np.float64 else arr


def _to_nd(x, pin):
    if isinstance(x, np.ndarray):
        return nd.array(x, ctx=cpu_pinned() if pin else None, dtype=x.dtype)
    if isinstance(x, (list, tuple)):
        return [_to_nd(i, pin) for i in x]
    if pin and isinstance(x, NDArray):
        return x.as_in_context(cpu_pinned())
    return x


# ------------------------------------------------------------------ shared-memory batch transport
def _flatten_arrays(obj, out):
    """Replace numpy arrays in a nested list/tuple by slot numbers; collect them in ``out``."""
    if isinstance(obj, np.ndarray):
        out.append(np.ascontiguousarray(obj))
        return ('@', len(out) - 1)
    if isinstance(obj, (list, tuple)):
        return (type(obj).__name__, [_flatten_arrays(o, out) for o in obj])
    return ('=', obj)


def _unflatten(desc, arrays):
    kind, val = desc
    if kind == '@':
        return arrays[val]
    if kind in ('list', 'tuple'):
        items = [_unflatten(d, arrays) for d in val]
        return items if kind == 'list' else tuple(items)
    return val


def _pack_batch(batch):
    """Put every array of ``batch`` into one new shared-memory segment; return its descriptor."""
    arrays = []
    structure = _flatten_arrays(batch, arrays)
    offs, total = [], 0
    for a in arrays:
        total = (total + 63) // 64 * 64
        offs.append(total)
        total += a.nbytes
    shm = shared_memory.SharedMemory(create=True, size=max(total, 1))
    try:
        for a, off in zip(arrays, offs):
            np.ndarray(a.shape, a.dtype, buffer=shm.buf, offset=off)[...] = a
        meta = [(a.shape, a.dtype.str, off) for a, off in zip(arrays, offs)]
        name = shm.name
    finally:
        shm.close()
    # the parent unlinks the segment; keep this process's resource tracker from "cleaning it up"
    try:
        from multiprocessing import resource_tracker
        resource_tracker.unregister('/' + name if not name.startswith('/') else name, 'shared_memory')
    except Exception:   # pylint: disable=broad-except
        pass
    return name, meta, structure


def _unpack_batch(name, meta, structure, pin):
    shm = shared_memory.SharedMemory(name=name)
    try:
        arrays = []
        for shape, dt, off in meta:
            view = np.ndarray(shape, np.dtype(dt), buffer=shm.buf, offset=off)
            arrays.append(nd.array(view, ctx=cpu_pinned() if pin else None, dtype=view.dtype))   # copies
        return _unflatten(structure, arrays)
    finally:
        shm.close()
        shm.unlink()


def _worker_loop(dataset, batchify_fn, tasks, results):
    """Body of a worker process: (seq, indices) in, (seq, descriptor | error) out, None = stop."""
    os.environ.setdefault('OMP_NUM_THREADS', '1')
    while True:
        job = tasks.get()
        if job is None:
            return
        tag, seq, indices = job
        try:
            batch = batchify_fn([dataset[i] for i in indices])
            results.put((tag, seq, 'ok', _pack_batch(batch)))
        except Exception as e:   # pylint: disable=broad-except
            import traceback
            results.put((tag, seq, 'err', '%s\n%s' % (e, traceback.format_exc())))


def _release(payload):
    try:
        shm = shared_memory.SharedMemory(name=payload[0])
        shm.close()
        shm.unlink()
    except Exception:   # pylint: disable=broad-except
        pass


def _discard_pending(results):
    """Unlink the segments of results nobody will read (abandoned iterators, shutdown)."""
    while True:
        try:
            _tag, _seq, status, payload = results.get(timeout=0.05)
        except Exception:   # pylint: disable=broad-except
            return
        if status == 'ok':
            _release(payload)


def _export_package_path():
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    parts = [p for p in os.environ.get('PYTHONPATH', '').split(os.pathsep) if p]
    if root not in parts:
        os.environ['PYTHONPATH'] = os.pathsep.join([root] + parts)


class _ProcessPool:
    """Fixed set of dataset-holding worker processes fed round-robin."""

    def __init__(self, num_workers, dataset, batchify_fn):
        # forkserver: children fork from a clean server process, never from this (threaded, possibly
        # HIP-initialised) one.  As with 'spawn', a script's top-level code must sit under
        # ``if __name__ == '__main__':``.  MXAMD_DATALOADER_START_METHOD overrides.
        method = os.environ.get('MXAMD_DATALOADER_START_METHOD', 'forkserver')
        ctx = multiprocessing.get_context(method)
        if method == 'forkserver':
            # the server imports the framework (torch included) once; every worker forks with it loaded.
            # It is a fresh interpreter: make the package importable there even when this process found
            # it through a runtime sys.path insertion (scripts run from a checkout)
            _export_package_path()
            ctx.set_forkserver_preload(['numpy', 'mxnet_maintenance_amd'])
        self._results = ctx.Queue()
        self._tasks = []
        self._procs = []
        for _ in range(num_workers):
            q = ctx.Queue()
            p = ctx.Process(target=_worker_loop, args=(dataset, batchify_fn, q, self._results), daemon=True)
            p.start()
            self._tasks.append(q)
            self._procs.append(p)
        self._next = 0
        self._closed = False

    def submit(self, tag, seq, indices):
        self._tasks[self._next].put((tag, seq, list(indices)))
        self._next = (self._next + 1) % len(self._tasks)

    def get(self, timeout):
        return self._results.get(timeout=timeout)

    def close(self):
        if self._closed:
            return
        self._closed = True
        for q in self._tasks:
            try:
                q.put(None)
            except Exception:   # pylint: disable=broad-except
                pass
        for p in self._procs:
            p.join(timeout=2)
            if p.is_alive():
                p.terminate()
                p.join(timeout=2)
        _discard_pending(self._results)
        for q in self._tasks + [self._results]:
            q.close()
            q.join_thread()


class _ProcessIter:
    """In-order iterator over batches computed by a ``_ProcessPool``."""

    _tags = iter(range(1 << 62))

    def __init__(self, pool, batch_sampler, pin_memory, prefetch, timeout):
        self._loader = None
        self._pool = pool
        self._tag = next(_ProcessIter._tags)
        self._sampler_iter = iter(batch_sampler)
        self._len = len(batch_sampler)
        self._pin = pin_memory
        self._timeout = timeout
        self._sent = 0
        self._rcvd = 0
        self._ready = {}
        for _ in range(max(1, prefetch)):
            self._push()

    def __len__(self):
        return self._len

    def _push(self):
        idx = next(self._sampler_iter, None)
        if idx is not None:
            self._pool.submit(self._tag, self._sent, idx)
            self._sent += 1

    def __next__(self):
        self._push()
        if self._rcvd == self._sent:
            raise StopIteration
        while self._rcvd not in self._ready:
            try:
                tag, seq, status, payload = self._pool.get(self._timeout)
            except _queue.Empty:
                raise RuntimeError('DataLoader worker timed out after %ss' % self._timeout) from None
            if tag != self._tag:          # left over from an abandoned iterator of this loader
                if status == 'ok':
                    _release(payload)
                continue
            self._ready[seq] = (status, payload)
        status, payload = self._ready.pop(self._rcvd)
        self._rcvd += 1
        if status == 'err':
            raise RuntimeError('DataLoader worker failed: %s' % payload)
        return _unpack_batch(*payload, pin=self._pin)

    next = __next__

    def __iter__(self):
        return self

    def __del__(self):
        # results already received but not consumed: release their segments now; results still in
        # flight are released by the next iterator of the same pool (or when the pool closes)
        for status, payload in self._ready.values():
            if status == 'ok':
                _release(payload)
        self._ready = {}


class _ThreadIter:
    def __init__(self, executor, dataset, batchify_fn, batch_sampler, pin_memory, prefetch, timeout):
        self._ex = executor
        self._dataset = dataset
        self._fn = batchify_fn
        self._it = iter(batch_sampler)
        self._len = len(batch_sampler)
        self._pin = pin_memory
        self._timeout = timeout
        self._futs = []
        for _ in range(max(1, prefetch)):
            self._push()

    def __len__(self):
        return self._len

    def _push(self):
        idx = next(self._it, None)
        if idx is not None:
            self._futs.append(self._ex.submit(lambda ix: self._fn([self._dataset[i] for i in ix]), idx))

    def __next__(self):
        self._push()
        if not self._futs:
            raise StopIteration
        batch = self._futs.pop(0).result(self._timeout)
        return _to_nd(batch, self._pin) if self._pin else batch

    next = __next__

    def __iter__(self):
        return self


class DataLoader:
    """Mini-batches from a Dataset, optionally with worker threads / processes."""

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
        self._num_workers = max(0, num_workers)
        self._worker_pool = None
        self._prefetch = max(0, int(prefetch) if prefetch is not None else 2 * self._num_workers)
        self._auto_reload = auto_reload
        if batchify_fn is None:
            batchify_fn = default_mp_batchify_fn if (self._num_workers > 0 and not thread_pool) else \
                default_batchify_fn
        self._batchify_fn = batchify_fn
        self._lock = threading.Lock()
        if self._num_workers > 0 and not auto_reload:
            self.refresh()

    def refresh(self):
        """(Re)start the workers."""
        self.clean()
        if self._num_workers == 0:
            return
        if self._thread_pool:
            self._worker_pool = ThreadPoolExecutor(self._num_workers)
        else:
            self._worker_pool = _ProcessPool(self._num_workers, self._dataset, self._batchify_fn)

    def clean(self):
        """Stop the workers and release their resources."""
        pool, self._worker_pool = self._worker_pool, None
        if pool is None:
            return
        if self._thread_pool:
            pool.shutdown(wait=False)
        else:
            pool.close()

    def __iter__(self):
        if self._num_workers == 0:
            def same_process_iter():
                for idx in self._batch_sampler:
                    batch = self._batchify_fn([self._dataset[i] for i in idx])
                    yield _to_nd(batch, self._pin_memory) if self._pin_memory else batch
            return same_process_iter()
        with self._lock:
            if self._worker_pool is None:
                self.refresh()
        if self._thread_pool:
            it = _ThreadIter(self._worker_pool, self._dataset, self._batchify_fn, self._batch_sampler,
                             self._pin_memory, self._prefetch, self._timeout)
            it._loader = self
            return it
        it = _ProcessIter(self._worker_pool, self._batch_sampler, self._pin_memory, self._prefetch,
                          self._timeout)
        it._loader = self          # the loader (and its worker pool) lives as long as the iterator
        return it

    def __len__(self):
        return len(self._batch_sampler)

    def __del__(self):
        try:
            self.clean()
        except Exception:   # pylint: disable=broad-except
            pass
