"""Optimizers (mx.optimizer).  Parity: python/mxnet/optimizer/__init__.py."""
from .optimizer import *  # noqa: F401,F403
from .optimizer import Optimizer, Updater, get_updater, create, register  # noqa: F401
from . import contrib  # noqa: F401
