"""Data iterators (mx.io).  Parity: python/mxnet/io/__init__.py."""
from .io import *  # noqa: F401,F403
from . import utils  # noqa: F401
