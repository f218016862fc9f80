"""Symbol operators with prefix _linalg_ (mx.sym.linalg)."""
from ..ops import registry as _registry
from .symbol import _op_func
for _n in _registry.list_ops():
    if _n.startswith('_linalg_'):
        globals()[_n[len('_linalg_'):]] = _op_func(_n)
