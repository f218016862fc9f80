"""Key-value store (mx.kv).  Parity: python/mxnet/kvstore/__init__.py."""
from .kvstore import KVStoreBase, KVStore, TestStore, create  # noqa: F401
from .compression import GradientCompression  # noqa: F401
from .kvstore_server import KVStoreServer  # noqa: F401
base = __import__(__name__ + '.kvstore', fromlist=['KVStoreBase'])
