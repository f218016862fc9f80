"""Contributed recurrent cells (parity: python/mxnet/gluon/contrib/rnn)."""
from .conv_rnn_cell import *  # noqa: F401,F403
from ...rnn.rnn_cell import VariationalDropoutCell, LSTMPCell  # noqa: F401
