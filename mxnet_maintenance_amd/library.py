"""Dynamically loaded operator libraries: ``mx.library.load(path)``.

Parity: python/mxnet/library.py + the framework side of the extension ABI in src/c_api/c_api.cc
(MXLoadLib).  A library is compiled against the reference's ``include/mxnet/lib_api.h`` +
``src/lib_api.cc`` (ABI version <= 11, e.g. example/extensions/lib_custom_op/gemm_lib.cc) and
exports plain C entry points (``initialize``, ``_opVersion``, ``_opRegSize``, ``_opRegGet``,
``_opCallParseAttrs``, ``_opCallInferShape``, ``_opCallInferType``, ``_opCallFCompute``,
``_opCallCreateOpState``, ``_opCallFStatefulCompute``, ``_msgSize``/``_msgGet``, ...).  This module
drives them through ctypes: every operator the library registers becomes an operator of this
framework (``mx.nd.<name>``, ``mx.sym.<name>``, hybridized blocks), with

* attribute parsing, shape and type inference delegated to the library,
* forward / backward computed by the library's CPU or GPU functions on this framework's buffers
  (GPU: device pointers plus the current HIP stream), workspace requests served by callbacks that
  allocate from torch,
* stateful operators (``setCreateOpState``): one library state object per forward call, kept
  for its backward and destroyed with it,
* gradients through autograd: the library's backward receives ``[out grads, inputs, outputs]``
  and writes the input gradients (the lib_api convention).

Graph passes, partitioners and subgraph operators the library registers are driven by
library_graph.py: ``Symbol.optimize_for(<pass or partitioner name>, args, aux, **options)``.
"""
import ctypes
import importlib.util
import json
import os
import weakref

import torch

from .base import MXNetError

__all__ = ['load', 'loaded_libraries', 'compiled_with_gcc_cxx11_abi']

MX_LIBRARY_VERSION = 11
_LIBS = {}

# mshadow type flags <-> torch
_FLAG_DT = {0: torch.float32, 1: torch.float64, 2: torch.float16, 3: torch.uint8, 4: torch.int32, 5: torch.int8,
            6: torch.int64, 12: torch.bfloat16}
_DT_FLAG = {v: k for k, v in _FLAG_DT.items()}

_c_p = ctypes.c_void_p
_c_pp = ctypes.POINTER(ctypes.c_void_p)
_MALLOC = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int)
_SPARSE_MALLOC = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.POINTER(ctypes.c_int64)),
                                  ctypes.POINTER(ctypes.POINTER(ctypes.c_int64)))


def compiled_with_gcc_cxx11_abi():
    """Libraries must use the same libstdc++ ABI as the framework's native modules (the new ABI)."""
    return True


def loaded_libraries():
    """Paths of the libraries loaded so far -> the operator names each one registered."""
    return {p: list(v[1]) for p, v in _LIBS.items()}


def _strs(values):
    arr = (ctypes.c_char_p * max(1, len(values)))()
    for i, v in enumerate(values):
        arr[i] = v.encode() if isinstance(v, str) else v
    return arr


class _Workspace:
    """Serves the library's ``res.alloc_cpu`` / ``res.alloc_gpu`` requests for one call."""

    def __init__(self, device):
        self.device = device
        self.keep = []
        self.cpu = _MALLOC(lambda _ctx, size: self._alloc(size, torch.device('cpu')))
        self.gpu = _MALLOC(lambda _ctx, size: self._alloc(size, device))
        self.sparse = _SPARSE_MALLOC(self._sparse)

    def _alloc(self, size, device):
        t = torch.empty(max(1, int(size)), dtype=torch.uint8, device=device)
        self.keep.append(t)
        return t.data_ptr()

    @staticmethod
    def _sparse(*_args):
        raise MXNetError('extension library: sparse outputs are not supported by this loader')


class _Lib:
    def __init__(self, path):
        self.path = path
        self.dll = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        d = self.dll
        d._opVersion.restype = ctypes.c_int
        self.version = d._opVersion()
        if self.version > MX_LIBRARY_VERSION:
            raise MXNetError('library %s has extension ABI version %d; this framework supports <= %d'
                             % (path, self.version, MX_LIBRARY_VERSION))
        d.initialize.restype = ctypes.c_int
        # the framework version the library may check (MXNET_VERSION of the reference: 1.9.0)
        if not d.initialize(ctypes.c_int(10900)):
            raise MXNetError('library %s failed to initialize: %s' % (path, self.messages()))
        d._opRegSize.restype = ctypes.c_int
        d._opCallFree.argtypes = [ctypes.c_void_p]

    def messages(self):
        d = self.dll
        if not hasattr(d, '_msgSize'):
            return ''
        d._msgSize.restype = ctypes.c_int
        out = []
        for i in range(d._msgSize()):
            m = ctypes.c_char_p()
            d._msgGet(ctypes.c_int(i), ctypes.byref(m))
            out.append(m.value.decode(errors='replace') if m.value else '')
        return '; '.join(out)

    def check(self, rc, what, name):
        if not rc:
            raise MXNetError('extension op %s: %s failed: %s' % (name, what, self.messages()))


class _LibOp:
    """One operator registered by a library (the table _opRegGet returns)."""

    def __init__(self, lib, idx):
        self.lib = lib
        d = lib.dll
        name = ctypes.c_char_p()
        is_sg = ctypes.c_int()
        f_ctx, b_ctx, c_ctx = (ctypes.POINTER(ctypes.c_char_p)() for _ in range(3))
        f_fp, b_fp, c_fp = (_c_pp() for _ in range(3))
        f_n, b_n, c_n = (ctypes.c_int() for _ in range(3))
        parse, typ, styp, shp, mut = (ctypes.c_void_p() for _ in range(5))
        d._opRegGet(ctypes.c_int(idx), ctypes.byref(name), ctypes.byref(is_sg),
                    ctypes.byref(f_ctx), ctypes.byref(f_fp), ctypes.byref(f_n),
                    ctypes.byref(b_ctx), ctypes.byref(b_fp), ctypes.byref(b_n),
                    ctypes.byref(c_ctx), ctypes.byref(c_fp), ctypes.byref(c_n),
                    ctypes.byref(parse), ctypes.byref(typ), ctypes.byref(styp), ctypes.byref(shp),
                    ctypes.byref(mut))
        self.name = name.value.decode()
        self.is_subgraph_op = bool(is_sg.value)
        self.forward = {f_ctx[i].decode(): f_fp[i] for i in range(f_n.value)}
        self.backward = {b_ctx[i].decode(): b_fp[i] for i in range(b_n.value)}
        self.create_state = {c_ctx[i].decode(): c_fp[i] for i in range(c_n.value)}
        self.parse, self.infer_type, self.infer_shape_fp = parse, typ, shp

    # ---- attribute / shape / type callbacks
    @staticmethod
    def _kv(attrs):
        items = [(k, v if isinstance(v, str) else str(v)) for k, v in attrs.items()
                 if not (k.startswith('__') and k.endswith('__'))]
        return _strs([k for k, _ in items]), _strs([v for _, v in items]), len(items)

    def num_inouts(self, attrs):
        keys, vals, n = self._kv(attrs)
        nin, nout = ctypes.c_int(), ctypes.c_int()
        rc = self.lib.dll._opCallParseAttrs(self.parse, keys, vals, ctypes.c_int(n), ctypes.byref(nin),
                                            ctypes.byref(nout))
        self.lib.check(rc, 'parseAttrs', self.name)
        return nin.value, nout.value

    def out_shapes(self, attrs, in_shapes, nout):
        keys, vals, n = self._kv(attrs)
        nin = len(in_shapes)
        bufs = [(ctypes.c_uint * max(1, len(s)))(*s) for s in in_shapes]
        inshapes = (ctypes.POINTER(ctypes.c_uint) * max(1, nin))(*[ctypes.cast(b, ctypes.POINTER(ctypes.c_uint))
                                                                 for b in bufs])
        indims = (ctypes.c_int * max(1, nin))(*[len(s) for s in in_shapes])
        mod_in, mod_dims = ctypes.POINTER(ctypes.POINTER(ctypes.c_uint))(), ctypes.POINTER(ctypes.c_int)()
        outs, outdims = ctypes.POINTER(ctypes.POINTER(ctypes.c_uint))(), ctypes.POINTER(ctypes.c_int)()
        rc = self.lib.dll._opCallInferShape(self.infer_shape_fp, keys, vals, ctypes.c_int(n), inshapes, indims,
                                            ctypes.c_int(nin), ctypes.byref(mod_in), ctypes.byref(mod_dims),
                                            ctypes.byref(outs), ctypes.byref(outdims), ctypes.c_int(nout))
        self.lib.check(rc, 'inferShape', self.name)
        res = [tuple(outs[i][j] for j in range(outdims[i])) for i in range(nout)]
        free = self.lib.dll._opCallFree
        for i in range(nin):
            free(ctypes.cast(mod_in[i], ctypes.c_void_p))
        for i in range(nout):
            free(ctypes.cast(outs[i], ctypes.c_void_p))
        for p in (mod_in, mod_dims, outs, outdims):
            free(ctypes.cast(p, ctypes.c_void_p))
        return res

    def out_types(self, attrs, in_dtypes, nout):
        keys, vals, n = self._kv(attrs)
        nin = len(in_dtypes)
        intypes = (ctypes.c_int * max(1, nin))(*[_DT_FLAG[t] for t in in_dtypes])
        outtypes = (ctypes.c_int * max(1, nout))(*([-1] * nout))
        rc = self.lib.dll._opCallInferType(self.infer_type, keys, vals, ctypes.c_int(n), intypes, ctypes.c_int(nin),
                                           outtypes, ctypes.c_int(nout))
        self.lib.check(rc, 'inferType', self.name)
        return [_FLAG_DT[outtypes[i]] for i in range(nout)]

    # ---- compute
    @staticmethod
    def _arrays(tensors):
        n = len(tensors)
        shape_bufs = [(ctypes.c_int64 * max(1, t.dim()))(*t.shape) for t in tensors]
        shapes = (ctypes.POINTER(ctypes.c_int64) * max(1, n))(
            *[ctypes.cast(b, ctypes.POINTER(ctypes.c_int64)) for b in shape_bufs])
        dims = (ctypes.c_int * max(1, n))(*[t.dim() for t in tensors])
        data = (ctypes.c_void_p * max(1, n))(*[t.data_ptr() for t in tensors])
        types = (ctypes.c_int * max(1, n))(*[_DT_FLAG[t.dtype] for t in tensors])
        ids = (ctypes.c_size_t * max(1, n))(*range(n))
        devt = _strs(['gpu' if t.is_cuda else 'cpu' for t in tensors])
        devi = (ctypes.c_int * max(1, n))(*[t.device.index or 0 for t in tensors])
        stypes = (ctypes.c_int * max(1, n))(*([0] * n))
        return shape_bufs, [shapes, dims, data, types, ids, devt, devi], stypes

    def _compute_args(self, inputs, outputs):
        dev = inputs[0].device if inputs else (outputs[0].device if outputs else torch.device('cpu'))
        ws = _Workspace(dev)
        kin, ain, sin = self._arrays(inputs)
        kout, aout, sout = self._arrays(outputs)
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream) if dev.type == 'cuda' else None
        nulls = [None] * 4
        zeros = [None] * 4
        tail = [ctypes.cast(ws.cpu, ctypes.c_void_p), None, ctypes.cast(ws.gpu, ctypes.c_void_p), None, stream,
                ctypes.cast(ws.sparse, ctypes.c_void_p), None, sin, sout] + nulls + zeros + [None, None]
        keep = (ws, kin, kout, ain, aout)
        return ([*ain, ctypes.c_int(len(inputs)), *aout, ctypes.c_int(len(outputs))], tail, keep)

    def _ctx_key(self, table, dev):
        key = 'gpu' if dev.type == 'cuda' else 'cpu'
        if key not in table:
            raise MXNetError('extension op %s has no %s implementation (registered: %s)'
                             % (self.name, key, sorted(table)))
        return key

    def fcompute(self, table, attrs, inputs, outputs):
        fp = table[self._ctx_key(table, inputs[0].device if inputs else outputs[0].device)]
        keys, vals, n = self._kv(attrs)
        head, tail, keep = self._compute_args(inputs, outputs)
        rc = self.lib.dll._opCallFCompute(ctypes.c_void_p(fp), keys, vals, ctypes.c_int(n), *head, *tail)
        del keep
        self.lib.check(rc, 'compute', self.name)

    def make_state(self, attrs, inputs):
        key = self._ctx_key(self.create_state, inputs[0].device)
        keys, vals, n = self._kv(attrs)
        bufs = [(ctypes.c_uint * max(1, t.dim()))(*t.shape) for t in inputs]
        inshapes = (ctypes.POINTER(ctypes.c_uint) * max(1, len(inputs)))(
            *[ctypes.cast(b, ctypes.POINTER(ctypes.c_uint)) for b in bufs])
        indims = (ctypes.c_int * max(1, len(inputs)))(*[t.dim() for t in inputs])
        intypes = (ctypes.c_int * max(1, len(inputs)))(*[_DT_FLAG[t.dtype] for t in inputs])
        state = ctypes.c_void_p()
        rc = self.lib.dll._opCallCreateOpState(ctypes.c_void_p(self.create_state[key]), keys, vals, ctypes.c_int(n),
                                               key.encode(), ctypes.c_int(inputs[0].device.index or 0), inshapes,
                                               indims, ctypes.c_int(len(inputs)), intypes, ctypes.byref(state))
        self.lib.check(rc, 'createOpState', self.name)
        st = _State(self.lib, state.value)
        return st

    def stateful(self, is_forward, state, inputs, outputs):
        head, tail, keep = self._compute_args(inputs, outputs)
        rc = self.lib.dll._opCallFStatefulCompute(ctypes.c_int(int(is_forward)), ctypes.c_void_p(state.ptr), *head,
                                                  *tail)
        del keep
        self.lib.check(rc, 'stateful %s' % ('forward' if is_forward else 'backward'), self.name)


class _State:
    """A library-side CustomStatefulOp; destroyed when the last autograd reference goes."""

    def __init__(self, lib, ptr):
        self.ptr = ptr
        weakref.finalize(self, lib.dll._opCallDestroyOpState, ctypes.c_void_p(ptr))


def _alloc_outputs(op, attrs, inputs):
    nin, nout = op.num_inouts(attrs)
    if nin != len(inputs):
        raise MXNetError('extension op %s expects %d inputs, got %d' % (op.name, nin, len(inputs)))
    shapes = op.out_shapes(attrs, [tuple(t.shape) for t in inputs], nout)
    types = op.out_types(attrs, [t.dtype for t in inputs], nout)
    dev = inputs[0].device
    return [torch.empty(s, dtype=dt, device=dev) for s, dt in zip(shapes, types)]


class _LibFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, op, attrs, *inputs):
        inputs = [t.contiguous() for t in inputs]
        outs = _alloc_outputs(op, attrs, inputs)
        state = None
        if op.create_state:
            state = op.make_state(attrs, inputs)
            op.stateful(True, state, inputs, outs)
        else:
            op.fcompute(op.forward, attrs, inputs, outs)
        ctx.op, ctx.attrs, ctx.state = op, attrs, state
        ctx.save_for_backward(*inputs, *outs)
        ctx.nin = len(inputs)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        op = ctx.op
        saved = ctx.saved_tensors
        inputs, outs = list(saved[:ctx.nin]), list(saved[ctx.nin:])
        ograds = [(g if g is not None else torch.zeros_like(o)).contiguous() for g, o in zip(grads, outs)]
        igrads = [torch.zeros_like(t) for t in inputs]
        if ctx.state is not None:
            op.stateful(False, ctx.state, ograds + inputs + outs, igrads)
        elif op.backward:
            op.fcompute(op.backward, ctx.attrs, ograds + inputs + outs, igrads)
        else:
            raise MXNetError('extension op %s has no backward' % op.name)
        return (None, None) + tuple(igrads)


def _make_fn(op):
    def fn(*inputs, **attrs):
        if inputs and inputs[0].device.type == 'meta':
            # shape / type inference: the library's own inference, nothing to compute
            outs = _alloc_outputs(op, dict(attrs), list(inputs))
            return outs[0] if len(outs) == 1 else tuple(outs)
        outs = _LibFunction.apply(op, dict(attrs), *inputs)
        return outs[0] if len(outs) == 1 else tuple(outs)
    fn.__name__ = op.name
    return fn


# ---------------------------------------------------------------- the framework's own minimal ABI
# ``mxamd_ext_ops()`` JSON + ``<name>_forward`` / ``<name>_backward`` (see tests/test_library.py):
# a smaller C ABI for gfx950 kernels built with ``hipcc -shared``, output shape = first input's.
_SIMPLE_DT = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}
_DT = _SIMPLE_DT
_LOADED = _LIBS


def _stream_of(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream) if t.is_cuda else ctypes.c_void_p(0)


def _make_function(lib, name, n_in, has_backward):
    fwd = getattr(lib, name + '_forward')
    fwd.restype = ctypes.c_int
    bwd = getattr(lib, name + '_backward', None) if has_backward else None
    if bwd is not None:
        bwd.restype = ctypes.c_int

    def ptrs(ts):
        return (ctypes.c_void_p * len(ts))(*[ctypes.c_void_p(t.data_ptr()) for t in ts])

    def shape_args(t):
        return (ctypes.c_int64 * max(1, t.dim()))(*t.shape), ctypes.c_int(t.dim())

    class _ExtFn(torch.autograd.Function):
        @staticmethod
        def forward(ctx, *inputs):
            ins = [i.contiguous() for i in inputs]
            if ins[0].dtype not in _DT:
                raise MXNetError('%s: unsupported dtype %s' % (name, ins[0].dtype))
            out = torch.empty_like(ins[0])
            shp, nd_ = shape_args(out)
            rc = fwd(ctypes.c_int(len(ins)), ptrs(ins), ctypes.c_void_p(out.data_ptr()), shp, nd_,
                     ctypes.c_int(_DT[out.dtype]), _stream_of(out))
            if rc != 0:
                raise MXNetError('%s_forward failed with status %d' % (name, rc))
            ctx.save_for_backward(*ins)
            return out

        @staticmethod
        def backward(ctx, gout):
            if bwd is None:
                raise MXNetError('operator %s from an extension library has no backward' % name)
            ins = ctx.saved_tensors
            gout = gout.contiguous()
            grads = [torch.empty_like(i) for i in ins]
            shp, nd_ = shape_args(gout)
            rc = bwd(ctypes.c_int(len(ins)), ptrs(ins), ctypes.c_void_p(gout.data_ptr()), ptrs(grads), shp, nd_,
                     ctypes.c_int(_DT[gout.dtype]), _stream_of(gout))
            if rc != 0:
                raise MXNetError('%s_backward failed with status %d' % (name, rc))
            return tuple(grads)

    def op(*inputs):
        if len(inputs) != n_in:
            raise MXNetError('%s expects %d inputs, got %d' % (name, n_in, len(inputs)))
        if any(i.shape != inputs[0].shape for i in inputs):
            raise MXNetError('%s: inputs must share one shape' % name)
        if inputs[0].device.type == 'meta':     # shape / type inference: no data to run on
            return torch.empty_like(inputs[0])
        return _ExtFn.apply(*inputs)
    return op


def _load_simple_abi(path, verbose):
    lib = ctypes.CDLL(path)
    if not hasattr(lib, 'mxamd_ext_ops'):
        raise MXNetError('%s exports no mxamd_ext_ops(): not an extension library' % path)
    lib.mxamd_ext_ops.restype = ctypes.c_char_p
    specs = json.loads(lib.mxamd_ext_ops().decode('utf-8'))
    from .ops import registry
    names = []
    for spec in specs:
        name, n_in = spec['name'], int(spec.get('num_inputs', 1))
        fn = _make_function(lib, name, n_in, bool(spec.get('backward', False)))
        arg_names = tuple('data' if n_in == 1 else 'data%d' % i for i in range(n_in))
        registry.register(name, fn, arg_names=arg_names, doc=spec.get('doc', 'extension operator'))
        names.append(name)
        if verbose:
            print('library %s: registered operator %s (%d inputs%s)' % (
                os.path.basename(path), name, n_in, ', backward' if spec.get('backward') else ''))
    return lib, names


def _load_python(path, verbose):
    from .ops import registry
    before = set(registry.list_ops())
    spec = importlib.util.spec_from_file_location('mxamd_ext_%d' % len(_LOADED), path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    names = sorted(set(registry.list_ops()) - before)
    if verbose:
        print('library %s: registered %s' % (os.path.basename(path), names))
    return mod, names


def _load_lib_api(path, verbose):
    lib = _Lib(path)
    from .ops import registry
    names = []
    from . import library_graph
    for i in range(lib.dll._opRegSize()):
        op = _LibOp(lib, i)
        if op.is_subgraph_op:
            # runs the subgraph a library partitioner formed (library_graph.register_subgraph_op)
            library_graph.register_subgraph_op(op)
            names.append(op.name)
            continue
        registry.register(op.name, _make_fn(op),
                          arg_names=(lambda op: lambda attrs: ['data%d' % j
                                                               for j in range(op.num_inouts(attrs)[0])])(op),
                          num_outputs=(lambda op: lambda attrs: op.num_inouts(attrs)[1])(op),
                          extra_params=True)
        names.append(op.name)
    passes, parts = library_graph.register_library(lib)
    if verbose:
        print('library %s (extension ABI v%d): registered operators %s, graph passes %s, partitioners %s' % (
            os.path.basename(path), lib.version, names, passes, parts))
    return lib, names


def load(path, verbose=True):
    """Load an operator library (absolute path to a ``.so`` / ``.py``) and register its operators.

    A ``.so`` built against the reference's lib_api.h (exports ``_opRegSize``) goes through the
    extension ABI above; one exporting ``mxamd_ext_ops`` through the minimal ABI; a ``.py`` file is
    imported as a plugin that registers operators itself.  Parity: python/mxnet/library.py load()."""
    if not os.path.exists(path):
        raise MXNetError('load path %s does NOT exist' % path)
    if not os.path.isabs(path):
        raise MXNetError('load path %s is not an absolute path' % path)
    ext = os.path.splitext(path)[1]
    if ext not in ('.so', '.py'):
        raise MXNetError('load path %s is NOT a library file (.so or .py)' % path)
    if path in _LIBS:
        return None
    if ext == '.py':
        _LIBS[path] = _load_python(path, verbose)
    else:
        probe = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        _LIBS[path] = _load_lib_api(path, verbose) if hasattr(probe, '_opRegSize') else \
            _load_simple_abi(path, verbose)
    # make the new operators visible as attributes right away
    from . import ndarray as nd
    from . import symbol as sym
    from .ndarray import register as _nd_register
    from .symbol.symbol import _op_func
    for name in _LIBS[path][1]:
        setattr(nd, name, _nd_register.make_op_function(name))
        setattr(sym, name, _op_func(name))
    return None
