"""Automatic mixed precision (mx.contrib.amp).  Parity: python/mxnet/contrib/amp/__init__.py."""
from .amp import *  # noqa: F401,F403
from .loss_scaler import LossScaler  # noqa: F401
from . import lists  # noqa: F401
