"""Where this framework's native libraries and headers live (reference: python/mxnet/libinfo.py:25).

The native parts are built in-tree by ``tools/build_native.py`` into ``mxnet_maintenance_amd/_lib``:
``libmxamd.so`` (C API), ``libmxamd_predict.so`` (C predict API), ``_native`` (engine, storage,
RecordIO) and ``_hip_kernels`` (the gfx950 kernels).  ``MXNET_LIBRARY_PATH`` /
``MXNET_INCLUDE_PATH`` override the search like the reference's.
"""
import glob
import logging
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_DIR = os.path.join(_HERE, '_lib')
_ROOT = os.path.dirname(_HERE)

__version__ = '1.9.1.amd0'


def _env_path(var, is_ok):
    p = os.environ.get(var)
    if not p:
        return None
    if not is_ok(p):
        logging.warning("%s '%s' doesn't exist", var, p)
        return None
    if not os.path.isabs(p):
        logging.warning('%s should be an absolute path, instead of: %s', var, p)
        return None
    return p


def find_lib_path(prefix='libmxamd'):
    """Paths of the native library files named ``prefix*.so`` (default: the C API library).

    ``prefix='libmxnet'`` (the reference's default) is taken to mean the C API library too."""
    env = _env_path('MXNET_LIBRARY_PATH', os.path.isfile)
    if env:
        return [env]
    if prefix == 'libmxnet':
        prefix = 'libmxamd'
    dirs = [_LIB_DIR] + [d.strip() for d in os.environ.get('LD_LIBRARY_PATH', '').split(':') if d.strip()]
    found = []
    for d in dirs:
        for p in [os.path.join(d, prefix + '.so')]:
            if os.path.isfile(p) and p not in found:
                found.append(p)
    if not found:
        raise RuntimeError('Cannot find the %s library (build it with tools/build_native.py).\n'
                           'Searched:\n%s' % (prefix, '\n'.join(dirs)))
    return found


def find_include_path():
    """Directory of the C API headers (``mxamd/c_api.h``, ``mxamd/c_predict_api.h``)."""
    env = _env_path('MXNET_INCLUDE_PATH', os.path.isdir)
    if env:
        return env
    for p in (os.path.join(_HERE, 'include'), os.path.join(_ROOT, 'include')):
        if os.path.isdir(p):
            return p + os.sep
    raise RuntimeError('Cannot find the include directory next to %s' % _HERE)


def find_conf_path(prefix='tvmop'):
    """The reference locates TVM-generated operator configs; there is no TVM backend here (operators
    are hand-written gfx950 kernels), so only an explicit ``MXNET_CONF_PATH`` is honoured."""
    env = _env_path('MXNET_CONF_PATH', os.path.isfile)
    if env:
        return [env]
    raise RuntimeError('No %s config: this framework has no TVM operator backend' % prefix)
