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
        'MIOPEN': torch.version.hip is not None, 'HIPBLASLT': torch.version.hip is not None,
        'HIP_RTC': torch.version.hip is not None,
        # the reference's feature names (src/libinfo.cc), answered for this build
        'CUDA': False, 'CUDNN': False, 'NCCL': False, 'CUDA_RTC': False, 'TENSORRT': False,
        'CPU_SSE': True, 'CPU_SSE2': True, 'CPU_SSE3': True, 'CPU_SSE4_1': True, 'CPU_SSE4_2': True,
        'CPU_SSE4A': False, 'CPU_AVX': True, 'CPU_AVX2': True, 'OPENMP': True, 'SSE': True, 'F16C': True,
        'JEMALLOC': False, 'BLAS_OPEN': True, 'BLAS_ATLAS': False, 'BLAS_MKL': False, 'BLAS_APPLE': False,
        'LAPACK': True, 'MKLDNN': False, 'OPENCV': False, 'CAFFE': False, 'PROFILER': True, 'DIST_KVSTORE': True,
        'CXX14': True, 'INT64_TENSOR_SIZE': True, 'SIGNAL_HANDLER': True, 'DEBUG': False, 'TVM_OP': False,
        'BF16': True,
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
