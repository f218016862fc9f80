"""Contrib optimizers (parity: python/mxnet/optimizer/contrib.py)."""
from .optimizer import GroupAdaGrad  # noqa: F401
