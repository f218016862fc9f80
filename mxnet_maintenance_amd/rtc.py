"""Runtime-compiled HIP kernels (parity: python/mxnet/rtc.py ``CudaModule`` / ``CudaKernel``).

The reference compiles CUDA C with NVRTC.  Here the HIP C++ source is
compiled for gfx950 at runtime by ``hipcc --genco`` into a code object
(cached by content hash under ``~/.cache/mxamd_rtc``), loaded with
``hipModuleLoad`` and launched with ``hipModuleLaunchKernel`` on the current
HIP stream through ctypes — no CUDA, no NVRTC.

::

    source = r'''
    extern "C" __global__ void axpy(const float* x, float* y, float alpha) {
        int i = blockIdx.x * blockDim.x + threadIdx.x;
        y[i] += alpha * x[i];
    }'''
    module = mx.rtc.CudaModule(source, exports=['axpy'])
    axpy = module.get_kernel('axpy', 'const float* x, float* y, float alpha')
    axpy.launch([x, y, 3.0], mx.gpu(0), (1, 1, 1), (10, 1, 1))
"""
import ctypes
import hashlib
import os
import re
import subprocess
import tempfile

from .base import MXNetError

__all__ = ['CudaModule', 'CudaKernel', 'HipModule', 'HipKernel']

_ARCH = os.environ.get('MXAMD_OFFLOAD_ARCH', 'gfx950')
_HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
_hip = None

_TYPES = {
    'float': ctypes.c_float, 'double': ctypes.c_double, 'int': ctypes.c_int32, 'int32_t': ctypes.c_int32,
    'unsigned': ctypes.c_uint32, 'uint32_t': ctypes.c_uint32, 'int64_t': ctypes.c_int64, 'long': ctypes.c_int64,
    'size_t': ctypes.c_uint64, 'uint64_t': ctypes.c_uint64, 'char': ctypes.c_int8, 'int8_t': ctypes.c_int8,
    'uint8_t': ctypes.c_uint8, 'short': ctypes.c_int16, 'bool': ctypes.c_bool, '__half': ctypes.c_uint16,
    'half': ctypes.c_uint16,
}


def _lib():
    global _hip
    if _hip is None:
        for name in ('libamdhip64.so', '/opt/rocm/lib/libamdhip64.so'):
            try:
                _hip = ctypes.CDLL(name)
                break
            except OSError:
                continue
        if _hip is None:
            raise MXNetError('rtc: libamdhip64.so not found')
    return _hip


def _check(err, what):
    if err != 0:
        lib = _lib()
        lib.hipGetErrorString.restype = ctypes.c_char_p
        raise MXNetError('rtc: %s failed: %s' % (what, lib.hipGetErrorString(err).decode()))


def compile_source(source, options=(), arch=_ARCH):
    """Compile HIP source to a gfx950 code object; returns its path (content-hash cached)."""
    key = hashlib.sha1((source + '\0' + ' '.join(options) + arch).encode()).hexdigest()[:20]
    cache = os.path.join(os.environ.get('MXAMD_RTC_CACHE', os.path.expanduser('~/.cache/mxamd_rtc')))
    os.makedirs(cache, exist_ok=True)
    out = os.path.join(cache, key + '.hsaco')
    if os.path.exists(out):
        return out
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, 'k.hip')
        with open(src, 'w') as f:
            f.write('#include <hip/hip_runtime.h>\n#include <hip/hip_fp16.h>\n' + source)
        tmp = os.path.join(d, 'k.hsaco')
        cmd = [_HIPCC, '--genco', '--offload-arch=' + arch, '-O3', *options, src, '-o', tmp]
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if r.returncode != 0:
            raise MXNetError('rtc: compilation failed:\n' + r.stdout)
        os.replace(tmp, out)
    return out


def _parse_signature(signature):
    args = []
    for part in [p.strip() for p in signature.split(',') if p.strip()]:
        is_ptr = '*' in part
        is_const = part.startswith('const') or ' const' in part
        toks = re.sub(r'[*&]', ' ', part).replace('const', ' ').split()
        if len(toks) < 2:
            raise MXNetError('rtc: cannot parse argument "%s" (need type and name)' % part)
        tname = ' '.join(toks[:-1])
        tname = tname.replace('unsigned int', 'unsigned').replace('long long', 'int64_t')
        if not is_ptr and tname not in _TYPES:
            raise MXNetError('rtc: unsupported argument type "%s"' % tname)
        args.append((is_ptr, is_const, tname))
    return args


class CudaModule:
    """A compiled HIP module (named CudaModule for API compatibility with the reference)."""

    def __init__(self, source, options=(), exports=()):
        self.source = source
        self.options = tuple(options)
        self.exports = tuple(exports)
        self.path = compile_source(source, self.options)
        self._handle = None

    def _module(self):
        if self._handle is None:
            h = ctypes.c_void_p()
            _check(_lib().hipModuleLoad(ctypes.byref(h), self.path.encode()), 'hipModuleLoad')
            self._handle = h
        return self._handle

    def get_kernel(self, name, signature):
        return CudaKernel(self, name, _parse_signature(signature))


class CudaKernel:
    def __init__(self, module, name, args):
        self.module = module
        self.name = name
        self.args = args
        self._fn = None

    def _function(self):
        if self._fn is None:
            f = ctypes.c_void_p()
            _check(_lib().hipModuleGetFunction(ctypes.byref(f), self.module._module(), self.name.encode()),
                   'hipModuleGetFunction(%s)' % self.name)
            self._fn = f
        return self._fn

    def launch(self, args, ctx, grid_dims, block_dims, shared_mem=0):
        """Launch on ``ctx`` (a GPU context) with ``args`` (NDArrays for pointers, numbers for scalars)."""
        import torch
        from .ndarray.ndarray import NDArray
        if len(args) != len(self.args):
            raise MXNetError('rtc: %s expects %d arguments, got %d' % (self.name, len(self.args), len(args)))
        holders = []
        for a, (is_ptr, _const, tname) in zip(args, self.args):
            if is_ptr:
                t = a._data if isinstance(a, NDArray) else a
                if not t.is_cuda:
                    raise MXNetError('rtc: pointer arguments must live on a GPU context')
                holders.append(ctypes.c_void_p(t.data_ptr()))
            else:
                holders.append(_TYPES[tname](a))
        params = (ctypes.c_void_p * len(holders))(*[ctypes.cast(ctypes.pointer(h), ctypes.c_void_p)
                                                    for h in holders])
        dev = ctx.device_id if hasattr(ctx, 'device_id') else 0
        with torch.cuda.device(dev):
            stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
            g = tuple(grid_dims) + (1,) * (3 - len(grid_dims))
            b = tuple(block_dims) + (1,) * (3 - len(block_dims))
            _check(_lib().hipModuleLaunchKernel(self._function(), g[0], g[1], g[2], b[0], b[1], b[2],
                                                ctypes.c_uint(shared_mem), stream, params, None),
                   'hipModuleLaunchKernel(%s)' % self.name)


HipModule = CudaModule
HipKernel = CudaKernel
