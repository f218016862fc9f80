"""Runtime feature detection (parity: python/mxnet/runtime.py, src/libinfo.cc)."""
import collections

import torch


Feature = collections.namedtuple('Feature', ['name', 'enabled'])


def _hip_loaded():
    from .ops import kernels
    return kernels.available()


def _native_loaded():
    from . import engine
    return engine.native_available()


def feature_list():
    feats = {
        'ROCM': torch.version.hip is not None,
        'HIP': torch.version.hip is not None,
        'HIP_KERNELS_GFX950': _hip_loaded(),
        'RCCL': torch.distributed.is_available() and torch.distributed.is_nccl_available(),
        'NATIVE_ENGINE': _native_loaded(),
        'CUDA': False, 'CUDNN': False, 'NCCL': False, 'TENSORRT': False,
        'CPU_SSE': True, 'CPU_AVX': True, 'OPENMP': True, 'MKLDNN': False,
        'BLAS_OPEN': True, 'LAPACK': True, 'OPENCV': False, 'DIST_KVSTORE': True,
        'INT64_TENSOR_SIZE': True, 'SIGNAL_HANDLER': True, 'DEBUG': False,
        'BF16': True, 'F16C': True,
    }
    return [Feature(k, v) for k, v in feats.items()]


class Features(collections.OrderedDict):
    """Compile-time/runtime features: ``Features().is_enabled('HIP')``."""
    instance = None

    def __new__(cls):
        if cls.instance is None:
            cls.instance = super().__new__(cls)
            super(Features, cls.instance).__init__([(f.name, f) for f in feature_list()])
        return cls.instance

    def __init__(self):
        pass

    def __repr__(self):
        return str(list(self.values()))

    def is_enabled(self, feature_name):
        feature_name = feature_name.upper()
        if feature_name not in self:
            raise RuntimeError('Feature \'{}\' is unknown, known features are: {}'.format(
                feature_name, list(self.keys())))
        return self[feature_name].enabled
