"""Sparse symbol helpers (mx.sym.sparse): same operators, storage type as attribute."""
from ..ops import registry as _registry
from .symbol import _op_func
for _n in ('dot', 'cast_storage', 'retain', 'elemwise_add', 'elemwise_sub', 'elemwise_mul',
           'broadcast_add', 'broadcast_mul', 'Embedding', 'FullyConnected', 'add_n', 'sum', 'mean',
           'zeros_like', 'abs', 'sqrt', 'square', 'clip'):
    if _registry.has(_n):
        globals()[_n] = _op_func(_n)
