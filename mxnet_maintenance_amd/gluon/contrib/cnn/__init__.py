"""Contributed convolution layers (parity: python/mxnet/gluon/contrib/cnn)."""
from .conv_layers import *  # noqa: F401,F403
