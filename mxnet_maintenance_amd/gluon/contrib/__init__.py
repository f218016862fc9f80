"""Contributed Gluon components (parity: python/mxnet/gluon/contrib)."""
from . import nn, cnn, rnn, data, estimator  # noqa: F401
