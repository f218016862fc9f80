"""IO helpers (parity: python/mxnet/io/utils.py)."""
from .io import _init_data  # noqa: F401


def _has_instance(data, dtype):
    for item in data:
        if isinstance(item[1], dtype):
            return True
    return False
