"""Multi-GPU / multi-process parallelism for MI355X nodes.

* ``dist``    : process group (one process per GPU, RCCL over xGMI; gloo on CPU)
* ``buckets`` : flat gradient buckets + all-reduce overlapped with backward (DP)
* ``sync_bn`` : cross-process BatchNorm statistics (SyncBatchNorm)
"""
from . import dist, buckets  # noqa: F401
from .dist import init, rank, world_size, local_rank, barrier  # noqa: F401
from .buckets import GradBuckets  # noqa: F401
