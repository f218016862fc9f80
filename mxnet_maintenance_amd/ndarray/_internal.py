"""Internal operators (names starting with an underscore), mx.nd._internal."""
from . import register as _register
from ..ops import registry as _registry
from ..ops import load_all as _load_all
_load_all()
for _n in _registry.list_ops():
    if _n.startswith('_'):
        globals()[_n] = _register.make_op_function(_n)
