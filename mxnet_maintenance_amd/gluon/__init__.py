"""Gluon: imperative/hybrid neural network API (mx.gluon).  Parity: python/mxnet/gluon/__init__.py."""
from .parameter import *  # noqa: F401,F403
from .parameter import Parameter, Constant, ParameterDict, DeferredInitializationError  # noqa: F401
from .block import *  # noqa: F401,F403
from . import nn  # noqa: F401
from . import rnn  # noqa: F401
from .trainer import *  # noqa: F401,F403
from . import loss  # noqa: F401
from . import utils  # noqa: F401
from . import data  # noqa: F401
from . import model_zoo  # noqa: F401
from . import contrib  # noqa: F401
from .graph_step import GraphStep  # noqa: F401
