"""Host NumPy fallbacks of ``numpy.linalg`` functions without a device implementation
(parity: python/mxnet/numpy/fallback_linalg.py); installed into ``mx.np.linalg``."""
from .fallback import _LINALG

__all__ = list(_LINALG)
