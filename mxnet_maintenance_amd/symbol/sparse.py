"""Sparse symbol helpers (mx.sym.sparse): same operators, storage type as attribute."""
from ..ops import registry as _registry
from .symbol import _op_func
for _n in ('dot', 'cast_storage', 'retain', 'elemwise_add', 'elemwise_sub', 'elemwise_mul',
           'broadcast_add', 'broadcast_mul', 'Embedding', 'FullyConnected', 'add_n', 'sum', 'mean',
           'zeros_like', 'abs', 'sqrt', 'square', 'clip'):
    if _registry.has(_n):
        globals()[_n] = _op_func(_n)


def __getattr__(name):
    # every other operator is available here with dense-storage semantics (reference: generated
    # mx.sym.sparse.<op> functions fall back to dense storage)
    from .. import symbol as _sym
    if name.startswith('__'):
        raise AttributeError(name)
    try:
        return getattr(_sym, name)
    except AttributeError:
        raise AttributeError("module 'symbol.sparse' has no attribute %r" % name) from None
