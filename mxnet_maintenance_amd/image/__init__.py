"""Image API (mx.image).  Parity: python/mxnet/image/__init__.py."""
from .image import *  # noqa: F401,F403
from .image import imdecode_np, _get_interp_method  # noqa: F401
from .detection import *  # noqa: F401,F403
