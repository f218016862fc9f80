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
