"""Loader + autograd wrappers for the gfx950 HIP kernel extension.

The extension ``mxnet_maintenance_amd/_lib/_hip_kernels*.so`` is built in-tree
by ``tools/build_native.py`` (hipcc --offload-arch=gfx950) from
``src/kernels/*.hip``.  Launch functions take raw device pointers plus the
current HIP stream, so every kernel is capturable in a HIP graph.
"""
import os

_mod = None
_err = None
_tried = False


def _load():
    global _mod, _err, _tried
    if _tried:
        return _mod
    _tried = True
    try:
        from .._lib import _hip_kernels as m  # noqa
        _mod = m
    except Exception as e:  # pragma: no cover - depends on build
        _err = repr(e)
        _mod = None
    return _mod


def available():
    return _load() is not None


def load_error():
    _load()
    return _err


def enabled():
    return os.environ.get('MXAMD_DISABLE_HIP', '0') != '1'


def lib():
    m = _load()
    if m is None:
        raise RuntimeError('HIP kernel extension not available: %s' % _err)
    return m


# Operator wrappers and their shape/dtype predicates (which calls the kernels support; anything
# else takes the torch path, itself MIOpen / hipBLASLt on ROCm) live next to the kernels they drive.
from .kernel_fns import *  # noqa: E402,F401,F403
from .kernel_fns import bn_ok, ce_ok, gap_ok, conv_ok, conv_tee_ok, pool_ok, bnrelu_pool_ok  # noqa: E402,F401
from .nlp_fns import *  # noqa: E402,F401,F403
from .nlp_fns import ln_ok, ew_ok, gemm_ok, embedding_ok  # noqa: E402,F401
