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
import weakref
from contextlib import contextmanager

__all__ = ['bulk', 'set_bulk_size', 'get', 'push', 'push_device', 'stream_wait_var', 'new_var', 'wait_for_var',
           'wait_all', 'native_available', 'Engine', 'debug_access', 'race_violations', 'var_of', 'copy_stream',
           'host_to_device', 'wait_host_reads', 'register_owned_pinned', 'unregister_owned_pinned']

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

    def clear_exception(self, v):
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
    ``mutable_vars`` pushed before it have finished.  Inside ``bulk(n)`` (n > 1) host ops are
    gathered and pushed as one engine op per ``n`` ops (see ``set_bulk_size``)."""
    if _bulk_size > 1 and _bulking.active:
        _bulking.add(fn, const_vars, mutable_vars, priority, name)
        return
    get().push(fn, list(const_vars), list(mutable_vars), priority, name)


class _Bulk(threading.local):
    """Host ops gathered by ``bulk``: flushed as ONE engine op (the reference's bulk execution,
    threaded_engine.h BulkAppend / BulkFlush: fewer scheduling round trips for chains of small ops).
    The bulk op reads the union of the gathered reads and writes the union of the writes; the
    functions run in push order, so their mutual dependencies are respected."""

    def __init__(self):
        self.active = False
        self.ops = []

    def add(self, fn, const_vars, mutable_vars, priority, name):
        self.ops.append((fn, list(const_vars), list(mutable_vars), priority, name))
        if len(self.ops) >= _bulk_size:
            self.flush()

    def flush(self):
        if not self.ops:
            return
        ops, self.ops = self.ops, []
        writes = []
        for _, _, m, _, _ in ops:
            writes.extend(v for v in m if all(v is not w for w in writes))
        reads = []
        for _, c, _, _, _ in ops:
            reads.extend(v for v in c if all(v is not w for w in writes + reads))
        fns = [op[0] for op in ops]

        def run_bulk():
            for f in fns:
                f()
        get().push(run_bulk, reads, writes, max(op[3] for op in ops), 'bulk[%d]' % len(fns))


_bulking = _Bulk()


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
    _bulking.flush()      # a device op ordered after gathered host ops sees them pushed first
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
    _bulking.flush()
    s, handle, dev = _stream_of(stream)
    if s is None:
        get().wait_for_var(var)
        return
    get().stream_wait_var(var, handle, dev)


def clear_exception(var):
    """Drop a pending failure of ``var`` (one already reported through another variable)."""
    get().clear_exception(var)


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
    _bulking.flush()
    get().wait_for_var(var)


def wait_all():
    _bulking.flush()
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
    """Set the op bulking size (MXNET_EXEC_BULK_EXEC_* in the reference); returns the previous
    value.  Inside ``bulk(size)`` host ops pushed through ``push`` are grouped ``size`` at a time
    into single engine ops.  Device work needs no bulking here: it is already batched on the HIP
    stream, and whole steps are captured into HIP graphs (gluon.GraphStep)."""
    global _bulk_size
    prev = _bulk_size
    _bulk_size = int(size)
    return prev


@contextmanager
def bulk(size):
    """Group the host ops pushed in this block ``size`` at a time (flushed at exit)."""
    prev = set_bulk_size(size)
    outer = _bulking.active
    _bulking.active = True
    try:
        yield
    finally:
        _bulking.flush()
        _bulking.active = outer
        set_bulk_size(prev)


# ------------------------------------------------------------------ host <-> device transfers
# Reference: CopyFromTo pushed to the ThreadedEnginePerDevice copy workers / streams
# (src/ndarray/ndarray.cc, src/engine/threaded_engine_perdevice.cc:47,95).  A host -> GPU copy is
# an engine device op on the GPU's dedicated copy stream, reading from pinned memory; the
# consumer stream waits for it with a HIP event (stream_wait_var), so the copy overlaps whatever
# compute is still queued and the host never blocks on the GPU.
_COPY_STREAMS = {}
_ASYNC_MIN_BYTES = int(os.environ.get('MXAMD_ASYNC_COPY_MIN_BYTES', str(64 << 10)))

# pinned host ranges we do not own with a pending device read: (base, nbytes, engine var of the copy)
_HOST_READS = []
_HOST_READS_MAX = 256


# pinned host ranges whose producer recycles them only after wait_host_reads (e.g. the
# ImageRecordIter batch ring): H2D copies read them in place.  Any other pinned source (a cpu_pinned
# NDArray, a DataLoader pin_memory batch) may be overwritten by host code at any time, so its copy
# reads a private pinned snapshot instead (no write-after-read race on the source).
_OWNED_PINNED = []


def register_owned_pinned(ptr, nbytes):
    """Declare ``[ptr, ptr + nbytes)`` as pinned memory whose producer calls ``wait_host_reads``
    before overwriting it."""
    _OWNED_PINNED.append((int(ptr), int(nbytes)))


def unregister_owned_pinned(ptr):
    _OWNED_PINNED[:] = [(b, n) for (b, n) in _OWNED_PINNED if b != int(ptr)]


def _is_owned_pinned(t):
    p = t.data_ptr()
    end = p + t.numel() * t.element_size()
    return any(b <= p and end <= b + n for (b, n) in _OWNED_PINNED)


_COMM_STREAMS = {}


def comm_stream(dev):
    """The communication stream of device ``dev`` (kvstore reduce/broadcast engine ops)."""
    import torch
    s = _COMM_STREAMS.get(dev)
    if s is None:
        s = _COMM_STREAMS[dev] = torch.cuda.Stream(device=dev)
    return s


def copy_stream(dev):
    """The dedicated H2D copy stream of device ``dev`` (a torch.device)."""
    import torch
    s = _COPY_STREAMS.get(dev)
    if s is None:
        s = _COPY_STREAMS[dev] = torch.cuda.Stream(device=dev)
    return s


def _note_host_read(src, var):
    _HOST_READS.append((src.data_ptr(), src.numel() * src.element_size(), var))
    if len(_HOST_READS) > _HOST_READS_MAX:
        wait_for_var(_HOST_READS.pop(0)[2])


def wait_host_reads(ptr, nbytes):
    """Block until every pending H2D copy reading ``[ptr, ptr + nbytes)`` has finished (producers
    that recycle pinned buffers call this before overwriting one)."""
    keep = []
    for base, n, var in _HOST_READS:
        if base < ptr + nbytes and ptr < base + n:
            wait_for_var(var)
        else:
            keep.append((base, n, var))
    _HOST_READS[:] = keep


def host_to_device(src, dev, out=None, var=None, name='h2d'):
    """Copy host tensor ``src`` to GPU ``dev`` as an engine device op on the copy stream.

    Returns the device tensor (``out`` when given -- the copy then first waits for the work already
    queued on the consumer stream, which may still read ``out``) and its engine variable; the
    caller's current stream on ``dev`` is made to wait for the copy on the GPU.  Pinned sources
    the caller does not own are registered so their producer can ``wait_host_reads``."""
    import torch
    src = src.detach().contiguous()
    borrowed = src.is_pinned() and _is_owned_pinned(src)
    if not borrowed:
        # private pinned snapshot: later host writes to the source cannot reach the pending DMA
        snap = torch.empty(src.shape, dtype=src.dtype, pin_memory=True)
        snap.copy_(src)
        src = snap
    cs = copy_stream(dev)
    consumer = torch.cuda.current_stream(dev)
    if out is None:
        # from the copy stream's pool: a block the compute stream freed may still be read by its
        # queued kernels, and the copy stream does not wait for them
        with torch.cuda.stream(cs):
            out = torch.empty(src.shape, dtype=src.dtype, device=dev)
    else:
        cs.wait_stream(consumer)       # write-after-read on an existing destination
    var = var if var is not None else new_var(name)
    if borrowed:
        _note_host_read(src, var)
    push_device(lambda dst=out, s=src: dst.copy_(s, non_blocking=True), (), (var,), stream=cs, name=name)
    stream_wait_var(var, consumer)
    out.record_stream(consumer)
    return out, var


def async_copy_ok(src, dev):
    """Whether a host -> device copy of ``src`` takes the engine path (big enough, not recorded)."""
    import torch
    return (dev.type == 'cuda' and src.device.type == 'cpu' and not (src.requires_grad and torch.is_grad_enabled())
            and src.numel() * src.element_size() >= _ASYNC_MIN_BYTES)


# ---------------------------------------------------------------- imperative GPU ops on worker streams
# Reference: ThreadedEnginePerDevice (src/engine/threaded_engine_perdevice.cc) runs GPU operators on
# MXNET_GPU_WORKER_NTHREADS worker streams per device; an operator waits for the writers of the arrays
# it reads and for the readers / writer of the arrays it writes, so independent chains overlap.
# Here, with MXNET_GPU_WORKER_NTHREADS = N > 1, every imperative operator is issued (from the calling
# thread: no hand-off, so no added latency) on one of N streams of its device -- slot 0 is the caller's
# current stream, slots 1..N-1 are worker streams.  The dependency state is kept by the native
# engine's Dispatcher (src/native/engine.{h,cc}) on the engine variables of the arrays (one variable
# per storage, shared by views): a chain stays on the stream that produced its inputs, cross-slot
# inputs and in-place targets are waited for on the GPU with lazily recorded HIP events, and
# host-visible points -- asnumpy / wait_to_read / waitall, copies, setitem, optimizer and kvstore
# updates -- join the worker slots into the caller's stream (join_workers).
# The default (1) keeps everything on the caller's stream.
GPU_WORKERS = max(1, int(os.environ.get('MXNET_GPU_WORKER_NTHREADS', '1') or 1))


class _Workers:
    def __init__(self):
        self.streams = {}     # device index -> [None, stream 1, ..., stream N-1]
        self.depth = 0        # > 0 while an operator body runs (nested operators stay on its stream)
        self.pending = []     # (device, slot, read vars) of the operators being issued (a stack)
        self.dirty = {}       # device index -> True when a worker slot has work since the last join
        # device index -> weak references to outputs produced on worker slots since the last join: the
        # caching allocator ties their blocks to the worker stream, so the join records them on the
        # caller's stream too (else a block freed while the caller's stream still reads it could be
        # handed to the next worker-stream allocation)
        self.produced = {}
        self.disp = None

    def dispatcher(self):
        if self.disp is None:
            nat = _load_native()
            if nat is None:
                raise RuntimeError('worker-stream dispatch needs the native engine (tools/build_native.py)')
            self.disp = nat.Dispatcher(False)
        return self.disp

    def stream(self, dev, sid):
        import torch
        if sid == 0:
            return torch.cuda.current_stream(dev)
        lst = self.streams.get(dev)
        if lst is None or len(lst) != GPU_WORKERS:
            old = lst or [None]
            lst = self.streams[dev] = [None] + [old[i] if i < len(old) else torch.cuda.Stream(device=dev)
                                                for i in range(1, GPU_WORKERS)]
            self.dispatcher().set_streams(dev, [int(x.cuda_stream) for x in lst[1:]])
        return lst[sid]


_workers = _Workers()


def set_gpu_workers(n):
    """Number of streams imperative GPU operators spread over per device (1 = the caller's stream
    only); returns the previous value.  Joins the current worker streams first."""
    global GPU_WORKERS
    join_workers()
    prev, GPU_WORKERS = GPU_WORKERS, max(1, int(n))
    if GPU_WORKERS > 1 and _load_native() is None:
        GPU_WORKERS = 1           # the dependency state lives in the native engine
    return prev


def _gpu_device(tensors):
    for t in tensors:
        if t is not None and t.is_cuda:
            return t.device.index
    return None


def _dvar(t):
    """The engine variable of tensor ``t``'s storage (views share their base's)."""
    base = t._base if t._base is not None else t
    v = getattr(base, '_mx_var', None)
    if v is None:
        v = base._mx_var = get().new_var('')
    return v


def slot_of(t):
    """Worker slot that last wrote tensor (or NDArray) ``t`` through dispatch; None when it was
    written outside operator dispatch (on the caller's stream)."""
    t = getattr(t, '_data', t)
    base = t._base if t._base is not None else t
    v = getattr(base, '_mx_var', None)
    if v is None or _load_native() is None:
        return None
    s = _load_native().Dispatcher.slot_of(v)
    return s if s >= 0 else None


def op_stream(tensors):
    """(slot, stream) an imperative operator on the input ``tensors`` runs on, with the GPU waits for
    inputs produced on other slots issued by the native dispatcher; (None, None) without a GPU input."""
    dev = _gpu_device(tensors)
    if dev is None:
        return None, None
    _workers.stream(dev, 1)                 # worker streams exist and are known to the dispatcher
    import torch
    cur = torch.cuda.current_stream(dev)
    reads = [_dvar(t) for t in tensors if t is not None and t.is_cuda]
    sid = _workers.dispatcher().begin(dev, int(cur.cuda_stream), reads)
    stream = _workers.stream(dev, sid)
    if sid:
        for t in tensors:
            if t is not None and t.is_cuda:
                t.record_stream(stream)     # the caching allocator keeps inputs alive for this stream
    _workers.pending.append((dev, sid, reads))
    return sid, stream


def op_written(t, sid, stream):
    """Before an in-place write of tensor ``t`` on slot ``sid``: wait for its writer and readers."""
    if t.is_cuda:
        import torch
        dev = t.device.index
        _workers.dispatcher().write(dev, int(torch.cuda.current_stream(dev).cuda_stream), sid, _dvar(t))
        _workers.dispatcher().end(dev, sid, [], [_dvar(t)])


def op_done(tensors, sid):
    """Mark output ``tensors`` as produced on slot ``sid`` (closes the operator op_stream opened)."""
    if not _workers.pending:
        return
    dev, slot, reads = _workers.pending.pop()
    ts = [t for t in tensors if isinstance(t, _torch_tensor()) and t.is_cuda]
    _workers.dispatcher().end(dev, slot, reads, [_dvar(t) for t in ts])
    if slot:
        _workers.dirty[dev] = True
        lst = _workers.produced.setdefault(dev, [])
        for t in ts:
            lst.append(weakref.ref(t))


def _torch_tensor():
    import torch
    return torch.Tensor


_JOIN_HOOKS = []


def add_join_hook(fn):
    """``fn()`` runs at every host-visible point (join_workers): other side streams' joins."""
    if fn not in _JOIN_HOOKS:
        _JOIN_HOOKS.append(fn)


def run_join_hooks():
    for fn in _JOIN_HOOKS:
        fn()


def join_workers(dev=None):
    """Make the caller's current stream (of ``dev``, default every device) wait on the GPU for all
    work issued on the worker slots so far (a host-visible point: starts a new epoch)."""
    if _workers.depth:
        return            # inside an operator body: its own stream is already the right one
    for fn in _JOIN_HOOKS:
        fn()
    if not _workers.dirty:
        return
    import torch
    devs = [dev] if dev is not None else list(_workers.dirty)
    for d in devs:
        if not _workers.dirty.pop(d, False):
            continue
        produced = _workers.produced.pop(d, ())
        cur = torch.cuda.current_stream(d)
        _workers.dispatcher().join(d, int(cur.cuda_stream))
        for ref in produced:
            t = ref()
            if t is not None:
                t.record_stream(cur)
