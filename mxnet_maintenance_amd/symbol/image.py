"""Symbol operators with prefix _image_ (mx.sym.image)."""
from ..ops import registry as _registry
from .symbol import _op_func
for _n in _registry.list_ops():
    if _n.startswith('_image_'):
        globals()[_n[len('_image_'):]] = _op_func(_n)
