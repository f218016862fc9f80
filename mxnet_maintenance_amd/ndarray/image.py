"""Image operators (mx.nd.image), parity: src/operator/image/*"""
from . import register as _register
from ..ops import registry as _registry
from ..ops import load_all as _load_all
_load_all()
for _n in _registry.list_ops():
    if _n.startswith('_image_'):
        globals()[_n[len('_image_'):]] = _register.make_op_function(_n)
