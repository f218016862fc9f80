"""pytest plugin for running the reference MXNet unit tests against this framework.

Importing it installs a meta-path finder that resolves ``mxnet`` and every
``mxnet.<sub>`` import to ``mxnet_maintenance_amd`` / ``mxnet_maintenance_amd.<sub>``
(the same module objects, so ``mxnet.nd.NDArray is mxnet_maintenance_amd.nd.NDArray``).
Used by tests/test_reference_conformance.py with ``-p mxalias``; the ``nose``
package next to this file is a minimal stand-in for the helpers the
reference tests import from nose.tools.
"""
import importlib
import importlib.abc
import importlib.util
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

_SRC = 'mxnet'
_DST = 'mxnet_maintenance_amd'


class _AliasLoader(importlib.abc.Loader):
    def __init__(self, target):
        self._target = target

    def create_module(self, spec):
        return importlib.import_module(self._target)

    def exec_module(self, module):
        return None


class _AliasFinder(importlib.abc.MetaPathFinder):
    def find_spec(self, fullname, path=None, target=None):
        if fullname != _SRC and not fullname.startswith(_SRC + '.'):
            return None
        real = _DST + fullname[len(_SRC):]
        try:
            if importlib.util.find_spec(real) is None:
                return None
        except ModuleNotFoundError:
            return None
        return importlib.util.spec_from_loader(fullname, _AliasLoader(real), is_package=True)


if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
    sys.meta_path.insert(0, _AliasFinder())

# The reference tests were written against NumPy 1.x; restore the aliases NumPy 2 removed so that
# failures measure this framework, not the NumPy version of the image.
import numpy as _np   # noqa: E402
for _old, _new in (('NaN', 'nan'), ('Inf', 'inf'), ('Infinity', 'inf'), ('PINF', 'inf'), ('NINF', None),
                   ('float_', 'float64'), ('round_', 'round'), ('product', 'prod'), ('cumproduct', 'cumprod'),
                   ('alltrue', 'all'), ('sometrue', 'any'), ('complex_', 'complex128'), ('unicode_', 'str_'), ('string_', 'bytes_')):
    if not hasattr(_np, _old):
        setattr(_np, _old, -_np.inf if _new is None else getattr(_np, _new))

_np_nonzero = _np.nonzero


def _nonzero_1x(a):
    """NumPy 1.x treated a 0-d array as 1-d in nonzero (NumPy 2 raises)."""
    a = _np.asarray(a)
    return _np_nonzero(_np.atleast_1d(a)) if a.ndim == 0 else _np_nonzero(a)


_np.nonzero = _nonzero_1x
