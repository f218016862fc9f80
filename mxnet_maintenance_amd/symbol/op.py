"""All operators as Symbol constructors (mx.sym.op)."""
from ..ops import registry as _registry
from .symbol import _op_func
for _n in _registry.list_ops():
    globals()[_n] = _op_func(_n)
