"""All registered operators as functions (mx.nd.op)."""
from . import register as _register
from ..ops import load_all as _load_all
_load_all()
_register.populate(globals())
