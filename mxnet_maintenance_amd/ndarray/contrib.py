"""Contrib operators (mx.nd.contrib), parity: python/mxnet/ndarray/contrib.py"""
from . import register as _register
from ..ops import registry as _registry
from ..ops import load_all as _load_all
_load_all()
for _n in _registry.list_ops():
    if _n.startswith('_contrib_'):
        globals()[_n[len('_contrib_'):]] = _register.make_op_function(_n)
