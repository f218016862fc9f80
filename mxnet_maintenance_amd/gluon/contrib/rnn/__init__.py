"""Contributed recurrent cells (parity: python/mxnet/gluon/contrib/rnn)."""
from .conv_rnn_cell import *  # noqa: F401,F403
from .rnn_cell import VariationalDropoutCell, LSTMPCell, dynamic_unroll  # noqa: F401
from . import rnn_cell  # noqa: F401
