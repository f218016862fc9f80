"""Notebook helpers (parity: python/mxnet/notebook)."""
from . import callback  # noqa: F401
