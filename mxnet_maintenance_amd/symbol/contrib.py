"""Symbol operators with prefix _contrib_ (mx.sym.contrib)."""
from ..ops import registry as _registry
from .symbol import _op_func
for _n in _registry.list_ops():
    if _n.startswith('_contrib_'):
        globals()[_n[len('_contrib_'):]] = _op_func(_n)
