"""mxnet_maintenance_amd: an MI355X-native deep learning framework with MXNet 1.x's API.

Usage mirrors the reference (geloescht/mxnet-maintenance, python/mxnet/__init__.py)::

    import mxnet_maintenance_amd as mx
    x = mx.nd.ones((2, 3), ctx=mx.gpu(0))
    net = mx.gluon.model_zoo.vision.resnet50_v1b(layout='NHWC')

Compute path: PyTorch-ROCm tensors + hand-written gfx950 HIP kernels (src/kernels),
RCCL over xGMI for data parallelism (kvstore 'device'), a native C++ dependency
engine / storage / RecordIO runtime (src/native).
"""
__version__ = '1.9.1.amd0'

import torch as _torch

import os
from . import base
from .base import MXNetError
from .context import Context, cpu, gpu, cpu_pinned, current_context, num_gpus, gpu_memory_info, Device
from . import context
from . import ops as _ops
_ops.load_all()
from . import engine
from . import ndarray
from . import ndarray as nd
from . import autograd
from . import random
from . import name
from . import attribute
from .attribute import AttrScope
from . import symbol
from . import symbol as sym
from . import executor
from . import initializer
from . import initializer as init
from . import optimizer
from . import lr_scheduler
from . import metric
from . import kvstore
from . import kvstore as kv
from . import gluon
from . import io
from . import recordio
from . import callback
from . import model
from . import module
from . import module as mod
from . import rnn
from . import library
from . import monitor
from . import monitor as mon
from . import profiler
from . import runtime
from . import test_utils
from . import registry
from . import error
from . import executor_manager
from . import notebook
from . import util
from . import operator
from . import image
from . import image as img
from . import visualization
from . import visualization as viz
from . import contrib
from . import parallel
from . import models
from . import utils
from . import numpy
from . import numpy as np
from . import numpy_extension
from . import numpy_dispatch_protocol
from . import numpy_extension as npx
from . import rtc
from . import numpy_op_signature
from . import log
from . import libinfo
from .util import is_np_array, is_np_shape, set_np, reset_np, use_np, np_shape, np_array, set_np_shape, use_np_shape, use_np_array

# A process launched as a dist_async server (DMLC_ROLE=server / scheduler) serves and exits at import,
# as the reference's kvstore_server module does.
if os.environ.get('DMLC_ROLE') in ('server', 'scheduler'):
    from .kvstore import kvstore_server as _kvs
    if _kvs._init_kvstore_server_module():
        import sys as _sys
        _sys.exit(0)
