"""Contributed neural network layers (parity: python/mxnet/gluon/contrib/nn)."""
from .basic_layers import *  # noqa: F401,F403
