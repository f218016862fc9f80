"""Neural network layers (mx.gluon.nn).  Parity: python/mxnet/gluon/nn/__init__.py."""
from .activations import *  # noqa: F401,F403
from .basic_layers import *  # noqa: F401,F403
from .conv_layers import *  # noqa: F401,F403
from ..block import Block, HybridBlock, SymbolBlock  # noqa: F401
