"""Linear algebra operators (mx.nd.linalg), parity: src/operator/tensor/la_op.cc"""
from . import register as _register
from ..ops import registry as _registry
from ..ops import load_all as _load_all
_load_all()
for _n in _registry.list_ops():
    if _n.startswith('_linalg_'):
        globals()[_n[len('_linalg_'):]] = _register.make_op_function(_n)
