"""Legacy symbolic RNN API (``mx.rnn``): cells that build Symbol graphs, unrolling, the
bucketing sentence iterator and RNN checkpoint helpers.

API parity: python/mxnet/rnn/ (rnn_cell.py, io.py, rnn.py).
"""
from .rnn_cell import *  # noqa: F401,F403
from .io import *        # noqa: F401,F403
from .rnn import *       # noqa: F401,F403
from . import rnn_cell, io, rnn  # noqa: F401
