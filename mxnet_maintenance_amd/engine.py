"""Dependency engine front-end.

Parity: python/mxnet/engine.py (bulk, set_bulk_size) and src/engine/*
(Engine::Get()->PushAsync / WaitForVar / WaitForAll, MXNET_ENGINE_TYPE,
MXNET_CPU_WORKER_NTHREADS).

The C++ engine (src/native/engine.cc) schedules work with reader/writer
dependencies on engine variables:

* host ops (``push``) run on a worker pool (decode, file writes, callbacks);
* device ops (``push_device``, the reference's ThreadedEnginePerDevice path) are
  issued on a given HIP stream once granted; ordering against work on other
  streams/devices is enforced on the GPU with HIP events (the issuing worker
  never waits for the GPU), and host ops touching a device-written variable
  synchronise on its event first;
* ``stream_wait_var`` makes a consumer stream wait for a variable's device
  write without blocking the host on GPU execution.

``MXNET_ENGINE_TYPE=NaiveEngine`` runs everything synchronously (the reference's
debugging mode); ``MXNET_ENGINE_DEBUG=1`` turns on the race detector (every op
validates the version / exclusive access of its variables when it starts, and
``debug_access`` reports undeclared direct accesses that overlap an engine op).
"""
import os
import threading
from contextlib import contextmanager

__all__ = ['bulk', 'set_bulk_size', 'get', 'push', 'push_device', 'stream_wait_var', 'new_var', 'wait_for_var',
           'wait_all', 'native_available', 'Engine', 'debug_access', 'race_violations', 'var_of']

_engine = None
_lock = threading.Lock()
_bulk_size = 15


def _load_native():
    try:
        from ._lib import _native
        return _native
    except Exception:  # pragma: no cover - depends on build
        return None


def native_available():
    return _load_native() is not None


class _PyVar:
    def __init__(self, name=''):
        self.name = name
        self.version = 0


class _PyEngine:
    """Synchronous fallback used only when the native library is not built."""
    naive = True
    num_workers = 0
    pending = 0
    executed = 0

    def new_var(self, name=''):
        return _PyVar(name)

    def push(self, fn, const_vars, mutable_vars, priority=0, name=''):
        fn()
        for v in mutable_vars:
            v.version += 1
        self.executed += 1

    def push_device(self, fn, const_vars, mutable_vars, stream, device, priority=0, name=''):
        self.push(fn, const_vars, mutable_vars, priority, name)

    def stream_wait_var(self, v, stream, device):
        pass

    debug = False
    violations = 0
    last_violation = ''
    device_ops = 0

    def debug_access(self, v, write=False):
        pass

    def push_write_file(self, path, data, const_vars, mutable_vars):
        with open(path, 'wb') as f:
            f.write(data)

    def wait_for_var(self, v):
        pass

    def wait_for_all(self):
        pass


def get():
    """Return the process-wide engine (created on first use)."""
    global _engine
    if _engine is None:
        with _lock:
            if _engine is None:
                nat = _load_native()
                etype = os.environ.get('MXNET_ENGINE_TYPE', 'ThreadedEnginePerDevice')
                nthreads = int(os.environ.get('MXNET_CPU_WORKER_NTHREADS', '4'))
                if nat is None:
                    _engine = _PyEngine()
                else:
                    _engine = nat.Engine(nthreads, etype == 'NaiveEngine',
                                         os.environ.get('MXNET_ENGINE_DEBUG', '0') == '1')
    return _engine


Engine = get


def new_var(name=''):
    return get().new_var(name)


def push(fn, const_vars=(), mutable_vars=(), priority=0, name=''):
    """Schedule ``fn()`` after all writers of ``const_vars`` and all users of
    ``mutable_vars`` pushed before it have finished."""
    get().push(fn, list(const_vars), list(mutable_vars), priority, name)


def _stream_of(stream):
    """(torch stream, raw hipStream_t handle, device index) -- (None, 0, -1) without a GPU."""
    import torch
    if stream is None:
        if not torch.cuda.is_available():
            return None, 0, -1
        stream = torch.cuda.current_stream()
    return stream, int(stream.cuda_stream), int(stream.device.index)


def push_device(fn, const_vars=(), mutable_vars=(), stream=None, priority=0, name=''):
    """Schedule a device op: once its variables are granted, ``fn()`` runs on a worker with ``stream``
    (default: the caller's current stream) as the current stream and must only *enqueue* work; the
    op completes when issued.  Other streams reading/writing the same variables are ordered after
    it with HIP events, host ops synchronise on it."""
    s, handle, dev = _stream_of(stream)
    if s is None:
        run = fn
    else:
        def run():
            import torch
            with torch.cuda.device(dev), torch.cuda.stream(s):
                fn()
    get().push_device(run, list(const_vars), list(mutable_vars), handle, dev, priority, name)


def stream_wait_var(var, stream=None):
    """Make ``stream`` (default: current) wait on the GPU for the last device write of ``var``."""
    s, handle, dev = _stream_of(stream)
    if s is None:
        get().wait_for_var(var)
        return
    get().stream_wait_var(var, handle, dev)


def debug_access(var, write=False):
    """Debug mode: declare a direct access to ``var`` made outside the engine."""
    get().debug_access(var, write)


def race_violations():
    """(count, last message) of the race detector (MXNET_ENGINE_DEBUG=1)."""
    e = get()
    return e.violations, e.last_violation


def var_of(arr):
    """The engine variable attached to an NDArray (created on first use; shared by its views)."""
    v = getattr(arr, '_engine_var', None)
    if v is None:
        v = new_var('ndarray%d' % id(arr))
        try:
            arr._engine_var = v
        except AttributeError:
            pass
    return v


def push_write_file(path, data, const_vars=(), mutable_vars=()):
    get().push_write_file(path, data, list(const_vars), list(mutable_vars))


def wait_for_var(var):
    get().wait_for_var(var)


def wait_all():
    if _engine is not None:
        _engine.wait_for_all()


# ------------------------------------------------------------------ deferred operator failures
# Reference semantics (src/engine/threaded_engine.cc): an operator that fails on a worker stores
# the exception on its output variables; any operator reading such a variable fails the same way;
# WaitForVar rethrows (and clears) a variable's exception, WaitForAll rethrows the first one and
# clears them all.  Here a failed output carries a shared one-slot "box" holding the exception
# (views of an array share it, like the reference's shared variable).
_failed = []          # boxes whose exception has not been rethrown yet
_failed_lock = threading.Lock()


def record_failure(exc):
    """A new failure box for ``exc``, registered for the next ``waitall``."""
    box = [exc]
    with _failed_lock:
        _failed.append(box)
    return box


# Every sampler writes the shared random-number resource (the reference's kRandom resource
# variable), so a sampler that fails leaves its failure on that resource and the samplers after it
# fail the same way (sharing the box) until the failure is rethrown somewhere.
_rng_box = [None]


def rng_failure():
    """The failure box held by the random resource, if still pending."""
    b = _rng_box[0]
    return b if b is not None and b[0] is not None else None


def set_rng_failure(box):
    _rng_box[0] = box


def rethrow(box):
    """Raise (once) the failure held by ``box``; it is cleared so later reads succeed."""
    if box is None or box[0] is None:
        return
    exc, box[0] = box[0], None
    with _failed_lock:
        try:
            _failed.remove(box)
        except ValueError:
            pass
    raise _as_mxnet_error(exc) from exc


def _as_mxnet_error(exc):
    from .base import MXNetError, MXNetValueError
    return (MXNetValueError if isinstance(exc, ValueError) else MXNetError)(str(exc))


def rethrow_all():
    """WaitForAll: raise the oldest pending failure and clear every pending one."""
    with _failed_lock:
        boxes = list(_failed)
        del _failed[:]
    first = None
    for b in boxes:
        if b[0] is not None and first is None:
            first = b[0]
        b[0] = None
    if first is not None:
        raise _as_mxnet_error(first) from first


def set_bulk_size(size):
    """Set the op bulking size; returns the previous value.  Device work is
    already batched on the HIP stream (and HIP graphs), so this only records
    the value for API parity."""
    global _bulk_size
    prev = _bulk_size
    _bulk_size = int(size)
    return prev


@contextmanager
def bulk(size):
    prev = set_bulk_size(size)
    try:
        yield
    finally:
        set_bulk_size(prev)
