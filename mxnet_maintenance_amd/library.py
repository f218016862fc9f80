"""Load operator libraries at run time (API parity: python/mxnet/library.py ``load``).

The reference dlopens a C++ library that registers operators through its
extension ABI (include/mxnet/lib_api.h).  Here an extension library is a shared
object (typically ``hipcc --offload-arch=gfx950 -shared`` output) exporting a
small C ABI that this loader turns into registered operators -- usable as
``mx.nd.<op>`` / ``mx.sym.<op>`` and in hybridized graphs:

``const char* mxamd_ext_ops(void)``
    JSON list of operator descriptions, each ``{"name": str, "num_inputs": int,
    "backward": bool}`` (output shape/dtype = first input's);
``int <name>_forward(int n_in, const void** in, void* out, const int64_t* shape,
int ndim, int dtype, void* stream)``
    dtype codes: 0 f32, 1 f16, 2 bf16; ``stream`` is the current HIP stream
    (NULL for host tensors); returns 0 on success;
``int <name>_backward(int n_in, const void** in, const void* grad_out,
void** grad_in, const int64_t* shape, int ndim, int dtype, void* stream)``
    optional; ``in`` are the forward inputs.

``.py`` files are also accepted: they are imported as plugins (they register
operators with ``mx.operator.register`` or the op registry themselves).
"""
import ctypes
import importlib.util
import json
import os

import torch

from .base import MXNetError

__all__ = ['load', 'loaded_libraries']

_DT = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}
_LOADED = {}


def loaded_libraries():
    """Paths of the libraries loaded so far -> the operator names each one registered."""
    return {p: list(v[1]) for p, v in _LOADED.items()}


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


def _load_native(path, verbose):
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


def load(path, verbose=True):
    """Load an operator library (absolute path to ``.so`` / ``.py``) and register its operators."""
    if not os.path.exists(path):
        raise MXNetError('load path %s does NOT exist' % path)
    if not os.path.isabs(path):
        raise MXNetError('load path %s is not an absolute path' % path)
    ext = os.path.splitext(path)[1]
    if ext not in ('.so', '.py'):
        raise MXNetError('load path %s is NOT a library file (.so or .py)' % path)
    if path in _LOADED:
        return None
    _LOADED[path] = _load_native(path, verbose) if ext == '.so' else _load_python(path, verbose)
    # make the new operators visible as attributes right away
    from . import ndarray as nd
    from . import symbol as sym
    from .ndarray import register as _nd_register
    from .symbol.symbol import _op_func
    for name in _LOADED[path][1]:
        setattr(nd, name, _nd_register.make_op_function(name))
        setattr(sym, name, _op_func(name))
    return None

