"""Experimental / contributed APIs (mx.contrib).  Parity: python/mxnet/contrib/__init__.py."""
from . import amp  # noqa: F401
from . import quantization  # noqa: F401
from . import quantization as quant  # noqa: F401  (reference alias mx.contrib.quant)
from . import text  # noqa: F401
from . import svrg_optimization  # noqa: F401
from . import autograd  # noqa: F401
from . import io  # noqa: F401
from . import tensorboard  # noqa: F401
from .. import ndarray as _nd
from .. import symbol as _sym
ndarray = _nd.contrib
symbol = _sym.contrib
nd = ndarray        # reference aliases (mx.contrib.nd / mx.contrib.sym)
sym = symbol
