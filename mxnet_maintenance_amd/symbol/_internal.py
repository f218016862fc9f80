"""Internal symbol operators (mx.sym._internal)."""
from ..ops import registry as _registry
from .symbol import _op_func
for _n in _registry.list_ops():
    if _n.startswith('_'):
        globals()[_n] = _op_func(_n)
