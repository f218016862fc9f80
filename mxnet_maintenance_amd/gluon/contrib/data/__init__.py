"""Contributed data utilities (parity: python/mxnet/gluon/contrib/data)."""
from ...data.sampler import IntervalSampler  # noqa: F401
from .text import WikiText2, WikiText103  # noqa: F401
