"""Stochastic variance-reduced gradient training (``mx.contrib.svrg_optimization``).

API parity: python/mxnet/contrib/svrg_optimization/ (``SVRGModule``).
"""
from .svrg_module import SVRGModule  # noqa: F401
from . import svrg_module  # noqa: F401
from . import svrg_optimizer  # noqa: F401
