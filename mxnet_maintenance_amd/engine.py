"""Dependency engine front-end.

Parity: python/mxnet/engine.py (bulk, set_bulk_size) and src/engine/*
(Engine::Get()->PushAsync / WaitForVar / WaitForAll, MXNET_ENGINE_TYPE,
MXNET_CPU_WORKER_NTHREADS).

The C++ engine (src/native/engine.cc) schedules host-side work with
reader/writer dependencies on engine variables.  ``MXNET_ENGINE_TYPE=NaiveEngine``
runs everything synchronously (the reference's debugging mode).
"""
import os
import threading
from contextlib import contextmanager

__all__ = ['bulk', 'set_bulk_size', 'get', 'push', 'new_var', 'wait_for_var', 'wait_all',
           'native_available', 'Engine']

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
                    _engine = nat.Engine(nthreads, etype == 'NaiveEngine')
    return _engine


Engine = get


def new_var(name=''):
    return get().new_var(name)


def push(fn, const_vars=(), mutable_vars=(), priority=0, name=''):
    """Schedule ``fn()`` after all writers of ``const_vars`` and all users of
    ``mutable_vars`` pushed before it have finished."""
    get().push(fn, list(const_vars), list(mutable_vars), priority, name)


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
