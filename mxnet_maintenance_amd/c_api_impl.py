"""Python half of the C API (src/capi/c_api.cc, include/mxamd/c_api.h).

Parity: include/mxnet/c_api.h -- NDArray (MXNDArrayCreate*, SyncCopy*, Save/Load, Reshape/Slice/At,
GetShape/DType/Context/Grad), imperative invoke (NNGetOpHandle, MXImperativeInvoke, autograd
record/train/mark/backward), Symbol (CreateFromJSON/File, SaveToJSON, List*, CreateVariable,
CreateAtomicSymbol + Compose, InferShape), Executor (Bind/Forward/Backward/Outputs) and KVStore
(Create/Init/Push/Pull).  The C layer passes plain Python values and opaque object references;
each function here does the framework call and returns plain values.  Device type codes follow
the reference (1 cpu, 2 gpu, 3 cpu_pinned), dtype codes mshadow's (0 f32, 1 f64, 2 f16, 3 u8,
4 i32, 5 i8, 6 i64, 7 bool, 12 bf16).
"""
import numpy as np

from . import ndarray as nd
from . import symbol as sym
from . import autograd
from .context import Context

VERSION = 10900

_DTYPES = {0: 'float32', 1: 'float64', 2: 'float16', 3: 'uint8', 4: 'int32', 5: 'int8', 6: 'int64', 7: 'bool',
           12: 'bfloat16'}
_CODES = {v: k for k, v in _DTYPES.items()}
_REQ = {0: 'null', 1: 'write', 2: 'write', 3: 'add'}   # kNullOp, kWriteTo, kWriteInplace, kAddTo


def _ctx(dev_type, dev_id):
    return Context({1: 'cpu', 2: 'gpu', 3: 'cpu_pinned'}.get(dev_type, 'cpu'), dev_id)


def nd_create(shape, dev_type, dev_id, dtype):
    return nd.zeros(tuple(shape), ctx=_ctx(dev_type, dev_id), dtype=_DTYPES[dtype])


def nd_none():
    return nd.NDArray(__import__('torch').empty(0))


def nd_shape(a):
    return [int(s) for s in a.shape]


def nd_dtype(a):
    name = str(a.dtype) if str(a.dtype) == 'bfloat16' else np.dtype(a.dtype).name
    return _CODES[name]


def nd_context(a):
    c = a.context
    return ({'cpu': 1, 'gpu': 2, 'cpu_pinned': 3}.get(c.device_type, 1), int(c.device_id))


def nd_from_bytes(a, buf, count):
    """Copy ``count`` elements of the array's dtype from the bytes ``buf`` into ``a``."""
    if count != int(np.prod(a.shape)):
        raise ValueError('SyncCopyFromCPU: size %d does not match the array size %d' % (count, np.prod(a.shape)))
    if str(a.dtype) == 'bfloat16':
        import torch
        t = torch.frombuffer(bytearray(buf), dtype=torch.bfloat16).reshape(a.shape)
        a[:] = nd.NDArray(t)
        return
    arr = np.frombuffer(buf, dtype=np.dtype(a.dtype), count=count).reshape(a.shape)
    a[:] = arr


def nd_to_bytes(a, count):
    if count != int(np.prod(a.shape)):
        raise ValueError('SyncCopyToCPU: size %d does not match the array size %d' % (count, np.prod(a.shape)))
    if str(a.dtype) == 'bfloat16':
        return a._data.detach().cpu().contiguous().view(__import__('torch').int16).numpy().tobytes()
    return np.ascontiguousarray(a.asnumpy()).tobytes()


def nd_wait(a):
    a.wait_to_read()


def nd_waitall():
    nd.waitall()


def nd_save(fname, arrays, keys):
    if keys:
        nd.save(fname, dict(zip(keys, arrays)))
    else:
        nd.save(fname, list(arrays))


def nd_load(fname):
    data = nd.load(fname)
    if isinstance(data, dict):
        names = list(data.keys())
        return [data[k] for k in names], names
    return list(data), []


def nd_reshape(a, dims):
    return a.reshape(tuple(dims))


def nd_slice(a, begin, end):
    return a[begin:end]


def nd_at(a, idx):
    return a[idx]


def nd_grad(a):
    return a.grad


def op_names():
    from .ops.registry import list_ops
    return sorted(list_ops())


def op_exists(name):
    from .ops import registry
    return bool(registry.has(name))


def invoke(name, inputs, keys, vals, outputs):
    """MXImperativeInvoke: run operator ``name``; ``outputs`` (optional arrays) receive the results."""
    fn = getattr(nd, name, None) or getattr(nd._internal, name, None) or getattr(nd.op, name, None)
    if fn is None:
        raise ValueError('operator %s is not registered' % name)
    kwargs = dict(zip(keys, vals))
    if outputs:
        kwargs['out'] = outputs if len(outputs) > 1 else outputs[0]
    res = fn(*inputs, **kwargs)
    return list(res) if isinstance(res, (list, tuple)) else [res]


def set_recording(flag):
    return int(autograd.set_recording(bool(flag)))


def set_training(flag):
    return int(autograd.set_training(bool(flag)))


def mark_variables(arrays, reqs, grads):
    autograd.mark_variables(list(arrays), list(grads), [_REQ.get(int(r), 'write') for r in reqs])


def backward(outputs, ograds, retain):
    og = None if not ograds or all(g is None for g in ograds) else list(ograds)
    autograd.backward(list(outputs), og, retain_graph=bool(retain))


# ---- Symbol
def sym_from_json(js):
    return sym.load_json(js)


def sym_from_file(fname):
    return sym.load(fname)


def sym_to_json(s):
    return s.tojson()


def sym_list(s, which):
    return {0: s.list_arguments, 1: s.list_outputs, 2: s.list_auxiliary_states}[which]()


def sym_var(name):
    return sym.Variable(name)


def sym_name(s):
    n = s.name
    return (n, 1) if n is not None else ('', 0)


class _Atomic:
    """An operator with its attributes, not yet composed with inputs (MXSymbolCreateAtomicSymbol)."""

    def __init__(self, op, attrs):
        self.op, self.attrs = op, attrs


def sym_atomic(op, keys, vals):
    return _Atomic(op, dict(zip(keys, vals)))


def sym_compose(atom, name, keys, args):
    """Compose an atomic symbol with its inputs; returns the composed Symbol."""
    fn = getattr(sym, atom.op, None) or getattr(sym._internal, atom.op, None)
    if fn is None:
        raise ValueError('operator %s is not registered' % atom.op)
    kw = dict(atom.attrs)
    if name:
        kw['name'] = name
    if keys:
        kw.update(dict(zip(keys, args)))
        return fn(**kw)
    return fn(*args, **kw)


def sym_infer_shape(s, keys, shapes):
    kw = dict(zip(keys, [tuple(x) for x in shapes])) if keys else {}
    if keys:
        a, o, x = s.infer_shape(**kw)
    else:
        a, o, x = s.infer_shape(*[tuple(x) for x in shapes])
    complete = a is not None and all(t is not None and all(d > 0 for d in t) for t in (a or []) + (o or []))
    conv = lambda lst: [list(t) if t is not None else [] for t in (lst or [])]   # noqa: E731
    return conv(a), conv(o), conv(x), int(bool(complete))


# ---- Executor
def bind(s, dev_type, dev_id, args, grads, reqs, aux):
    names = s.list_arguments()
    req = {n: _REQ.get(int(r), 'write') for n, r in zip(names, reqs)}
    grad_map = {n: g for n, g in zip(names, grads) if g is not None}
    return s.bind(_ctx(dev_type, dev_id), list(args), args_grad=grad_map or None, grad_req=req,
                  aux_states=list(aux) if aux else None)


def exec_forward(e, is_train):
    e.forward(is_train=bool(is_train))


def exec_backward(e, head_grads):
    e.backward(list(head_grads) if head_grads else None)


def exec_outputs(e):
    return list(e.outputs)


# ---- KVStore
def kv_create(kind):
    from . import kvstore
    return kvstore.create(kind)


def kv_init(kv, keys, vals):
    kv.init(list(keys), list(vals))


def kv_push(kv, keys, vals, priority):
    kv.push(list(keys), list(vals), priority=priority)


def kv_pull(kv, keys, vals, priority):
    kv.pull(list(keys), out=list(vals), priority=priority)


# ================================================================ round 6: wider C API surface
# Parity: include/mxnet/c_api.h -- NDArray extras (:983 MXNDArrayGetData, :910 GetStorageType,
# :713/:723 raw bytes, :810 SyncCopyFromNDArray, :1125 Detach, :1132 grad state), autograd (:1291,
# :1353 MXAutogradBackwardEx), CachedOp (:1372-1417), profiler (:303-482), data iterators
# (:2609-2698), RecordIO (:3151-3217), KVStore extras (:2762-3086, :2947 MXKVStorePushPull), runtime
# (:255 MXRandomSeed, :282, :491-524, :498 MXEngineSetBulkSize, :1303 numpy shape) and Symbol /
# Executor extras (:1535-1708, :2245).
_STYPES = {'default': 0, 'row_sparse': 1, 'csr': 2}


def nd_data_ptr(a):
    """Address of the array's first element (host memory for CPU arrays, device memory for GPU
    arrays, like the reference's dptr); the array must be contiguous."""
    t = a._data
    if not t.is_contiguous():
        raise ValueError('MXNDArrayGetData: the array is not contiguous')
    if t.is_cuda:
        a.wait_to_read()
    return int(t.data_ptr())


def nd_storage_type(a):
    return _STYPES.get(getattr(a, 'stype', 'default'), -1)


def nd_detach(a):
    return a.detach()


def nd_set_grad_state(a, state):
    a._fresh_grad = bool(state)


def nd_get_grad_state(a):
    return int(bool(getattr(a, '_fresh_grad', False)))


def nd_save_raw(a):
    import io as _io
    from .ndarray import utils as U
    buf = _io.BytesIO()
    U._write_array(buf, a)
    return buf.getvalue()


def nd_load_raw(buf):
    from .ndarray import utils as U
    return U._read_array(U._Reader(buf))


def nd_copy_from_nd(dst, src, i):
    """i = -1: copy src's data into dst; i >= 0: copy src's i-th auxiliary array (sparse indices)."""
    if i < 0:
        src.copyto(dst)
        return
    aux = src._aux[i] if hasattr(src, '_aux') else None
    if aux is None:
        raise ValueError('MXNDArraySyncCopyFromNDArray: source has no auxiliary array %d' % i)
    dst[:] = nd.NDArray(aux)


def nd_wait_write(a):
    fn = getattr(a, 'wait_to_write', None)
    (fn or a.wait_to_read)()


def is_recording():
    return int(autograd.is_recording())


def is_training():
    return int(autograd.is_training())


def backward_ex(outputs, ograds, variables, retain, create_graph, is_train):
    """MXAutogradBackwardEx: gradients of ``variables`` returned (autograd.grad) when given, else a
    backward pass into the marked variables' .grad buffers."""
    og = None if not ograds or all(g is None for g in ograds) else list(ograds)
    if variables:
        with autograd.train_mode() if is_train else autograd.predict_mode():
            gs = autograd.grad(list(outputs), list(variables), head_grads=og, retain_graph=bool(retain),
                               create_graph=bool(create_graph))
        return list(gs), [nd_storage_type(g) for g in gs]
    autograd.backward(list(outputs), og, retain_graph=bool(retain), train_mode=bool(is_train))
    return [], []


# ---- CachedOp
def cached_op_create(s, keys, vals):
    return nd.CachedOp(s, list(zip(keys, vals)))


def cached_op_invoke(op, inputs, outputs):
    if outputs:
        op(*inputs, out=outputs if len(outputs) > 1 else outputs[0])
        return list(outputs), [nd_storage_type(o) for o in outputs]
    res = op(*inputs)
    res = list(res) if isinstance(res, (list, tuple)) else [res]
    return res, [nd_storage_type(r) for r in res]


# ---- profiler
def prof_config(keys, vals):
    from . import profiler
    kw = {}
    for k, v in zip(keys, vals):
        lv = v.lower()
        kw[k] = True if lv in ('true', '1') else False if lv in ('false', '0') else v
    profiler.set_config(**kw)


def prof_state(state):
    from . import profiler
    profiler.set_state('run' if state else 'stop')


def prof_dump(finished):
    from . import profiler
    profiler.dump(finished=bool(finished))


def prof_dumps(reset):
    from . import profiler
    return profiler.dumps(reset=bool(reset))


def prof_pause(paused):
    from . import profiler
    (profiler.pause if paused else profiler.resume)()


def prof_domain(name):
    from . import profiler
    return profiler.Domain(name)


def prof_task(domain, name):
    from . import profiler
    return profiler.Task(domain, name)


def prof_start(h):
    h.start()


def prof_stop(h):
    h.stop()


def prof_marker(domain, name, scope):
    from . import profiler
    profiler.Marker(domain, name).mark(scope or 'process')


# ---- data iterators (the reference's C++ iterators; NDArrayIter is Python-only there too)
_ITERS = ('CSVIter', 'ImageDetRecordIter', 'ImageRecordInt8Iter', 'ImageRecordIter', 'ImageRecordUInt8Iter',
          'LibSVMIter', 'MNISTIter')


def iter_names():
    from . import io as mio
    return [n for n in _ITERS if hasattr(mio, n)]


def _parse_val(v):
    import ast
    try:
        return ast.literal_eval(v)
    except (ValueError, SyntaxError):
        return v


def iter_create(name, keys, vals):
    from . import io as mio
    return _CIter(getattr(mio, name)(**{k: _parse_val(v) for k, v in zip(keys, vals)}))


def iter_info(name):
    import inspect
    from . import io as mio
    cls = getattr(mio, name)
    doc = (inspect.getdoc(cls) or name).split('\n')[0]
    try:
        params = [p for p in inspect.signature(cls.__init__).parameters.values()
                  if p.name != 'self' and p.kind not in (p.VAR_POSITIONAL, p.VAR_KEYWORD)]
    except (TypeError, ValueError):
        params = []
    names = [p.name for p in params]
    types = ['%s, optional, default=%r' % (type(p.default).__name__, p.default)
             if p.default is not p.empty else 'required' for p in params]
    return name, doc, names, types, [''] * len(names)


class _CIter:
    """C-side iterator state: the current batch of a framework DataIter."""

    def __init__(self, it):
        self.it, self.batch = it, None

    def next(self):
        try:
            self.batch = self.it.next()
            return 1
        except StopIteration:
            self.batch = None
            return 0

    def reset(self):
        self.it.reset()
        self.batch = None


def iter_next(c):
    return c.next()


def iter_reset(c):
    c.reset()


def _cur(c):
    if c.batch is None:
        raise ValueError('data iterator: no current batch (call MXDataIterNext first)')
    return c.batch


def iter_data(c):
    return _cur(c).data[0]


def iter_label(c):
    return _cur(c).label[0]


def iter_pad(c):
    return int(_cur(c).pad or 0)


def iter_index(c):
    idx = _cur(c).index
    if idx is None:
        return []
    return [int(i) for i in np.asarray(idx).reshape(-1)]


# ---- RecordIO
def rec_writer(uri):
    from .recordio import MXRecordIO
    return MXRecordIO(uri, 'w')


def rec_reader(uri):
    from .recordio import MXRecordIO
    return MXRecordIO(uri, 'r')


def rec_write(r, buf):
    r.write(bytes(buf))


def rec_read(r):
    b = r.read()
    return b if b is not None else None


def rec_tell(r):
    return int(r.tell())


def rec_seek(r, pos):
    r.handle.seek(int(pos))     # byte offset (MXIndexedRecordIO.seek takes a record index instead)


def rec_close(r):
    r.close()


# ---- KVStore extras
def _runs(keys, items):
    """[(key, [items...])] for runs of equal consecutive keys (the C arrays list a key's values
    next to each other)."""
    groups = []
    for k, x in zip(keys, items):
        if groups and groups[-1][0] == k:
            groups[-1][1].append(x)
        else:
            groups.append((k, [x]))
    return groups


def kv_pushpull(kv, vkeys, okeys, vals, outs, priority):
    vg, og = _runs(vkeys, vals), _runs(okeys, outs)
    if [k for k, _ in vg] != [k for k, _ in og]:
        raise ValueError('MXKVStorePushPull: push and pull keys must match')
    for (k, v), (_, o) in zip(vg, og):
        kv.pushpull(k, v if len(v) > 1 else v[0], out=o if len(o) > 1 else o[0], priority=priority)


def kv_type(kv):
    return kv.type


def kv_rank(kv):
    return int(kv.rank)


def kv_group_size(kv):
    return int(kv.num_workers)


def kv_barrier(kv):
    fn = getattr(kv, '_barrier', None) or getattr(kv, 'barrier', None)
    if fn is not None:
        fn()


# ---- runtime
def random_seed(seed, dev_type, dev_id):
    from . import random as mxrandom
    if dev_type < 0:
        mxrandom.seed(seed)
    else:
        mxrandom.seed(seed, ctx=_ctx(dev_type, dev_id))


def notify_shutdown():
    nd.waitall()


def set_omp_threads(n):
    import torch
    torch.set_num_threads(max(1, int(n)))


def gpu_count():
    from .context import num_gpus
    return int(num_gpus())


def gpu_memory(dev):
    from .context import gpu_memory_info
    free, total = gpu_memory_info(dev)
    return int(free), int(total)


def set_bulk_size(n):
    from . import engine
    return int(engine.set_bulk_size(int(n)))


def set_np_shape(flag):
    from . import util
    return int(util.set_np_shape(bool(flag)))


def is_np_shape():
    from . import util
    return int(util.is_np_shape())


# ---- Symbol / Executor extras
def sym_copy(s):
    import copy
    return copy.deepcopy(s)


def sym_print(s):
    return s.debug_str()


def sym_get_attr(s, key):
    v = s.attr(key)
    return (v, 1) if v is not None else ('', 0)


def sym_set_attr(s, key, value):
    s._set_attr(**{key: value})


def sym_internals(s):
    return s.get_internals()


def sym_output(s, i):
    return s[int(i)]


def sym_num_outputs(s):
    return len(s.list_outputs())


def sym_group(syms):
    return sym.Group(list(syms))


def sym_save(s, fname):
    s.save(fname)


def sym_children(s):
    return s.get_children()


def exec_print(e):
    return e.debug_str()
