"""``mx.npx``: MXNet-specific operators for the NumPy interface.

Parity: python/mxnet/numpy_extension/{__init__,_op,utils,random,image}.py and
src/operator/numpy_extension.  Neural-network operators are the same registered
kernels as the legacy ``mx.nd`` ops (HIP kernels for conv/BN/pool on gfx950),
returning ``mx.np.ndarray``; given Symbols they build graph nodes so they work in
hybridized blocks.
"""
import functools

import torch

from .. import _state
from ..context import cpu, gpu, num_gpus, current_context, cpu_pinned  # noqa: F401
from ..util import (set_np, reset_np, is_np_array, is_np_shape, use_np, use_np_array, use_np_shape,  # noqa: F401
                    np_array, np_shape, set_np_shape)
from ..ndarray.ndarray import NDArray, waitall  # noqa: F401
from ..ndarray import register as _reg
from ..ops import registry as _registry
from ..base import torch_dtype as _torch_dtype
from ..numpy.multiarray import _host_graph


def _is_sym(x):
    from ..symbol.symbol import Symbol
    return isinstance(x, Symbol)


def _op(opname, defaults=None, doc=None, pyname=None):
    def f(*args, **kwargs):
        for k, v in (defaults or {}).items():
            kwargs.setdefault(k, v)
        if any(_is_sym(a) for a in args) or any(_is_sym(v) for v in kwargs.values()):
            from ..symbol.symbol import _op_func
            return _op_func(opname)(*args, **kwargs)
        from ..numpy.multiarray import _np_out
        return _np_out(_reg.invoke_by_name(opname, args, kwargs))
    f.__name__ = pyname or opname
    f.__doc__ = doc or 'npx wrapper of operator ``%s`` (returns mx.np.ndarray).' % opname
    return f


_MAP = {
    'activation': ('Activation', None), 'relu': ('Activation', {'act_type': 'relu'}),
    'sigmoid': ('Activation', {'act_type': 'sigmoid'}), 'softmax': ('softmax', None),
    'log_softmax': ('log_softmax', None), 'masked_softmax': ('masked_softmax', None),
    'masked_log_softmax': ('masked_log_softmax', None), 'batch_norm': ('BatchNorm', None),
    'convolution': ('Convolution', None), 'deconvolution': ('Deconvolution', None), 'pooling': ('Pooling', None),
    'dropout': ('Dropout', None), 'embedding': ('Embedding', None), 'fully_connected': ('FullyConnected', None),
    'layer_norm': ('LayerNorm', None), 'group_norm': ('GroupNorm', None), 'instance_norm': ('InstanceNorm', None),
    'leaky_relu': ('LeakyReLU', None), 'one_hot': ('one_hot', None), 'pick': ('pick', None), 'topk': ('topk', None),
    'rnn': ('RNN', None), 'arange_like': ('_contrib_arange_like', None), 'batch_dot': ('batch_dot', None),
    'batch_flatten': ('Flatten', None), 'broadcast_like': ('broadcast_like', None), 'gamma': ('gamma', None),
    'gammaln': ('gammaln', None), 'erf': ('erf', None), 'erfinv': ('erfinv', None),
    'sequence_mask': ('SequenceMask', None), 'sequence_last': ('SequenceLast', None),
    'sequence_reverse': ('SequenceReverse', None), 'slice': ('slice', None), 'smooth_l1': ('smooth_l1', None),
    'stop_gradient': ('BlockGrad', None), 'shape_array': ('shape_array', None), 'roi_pooling': ('ROIPooling', None),
    'roi_align': ('_contrib_ROIAlign', None), 'ctc_loss': ('CTCLoss', None), 'reshape_like': ('reshape_like', None),
    'index_add': ('_contrib_index_add', None), 'index_update': ('_contrib_index_update', None),
    'constraint_check': ('_npx_constraint_check', None), 'cast': ('Cast', None), 'amp_cast': ('amp_cast', None),
    'softmax_cross_entropy': ('softmax_cross_entropy', None), 'box_nms': ('_contrib_box_nms', None),
    'box_iou': ('_contrib_box_iou', None), 'multibox_prior': ('_contrib_MultiBoxPrior', None),
    'multibox_target': ('_contrib_MultiBoxTarget', None), 'multibox_detection': ('_contrib_MultiBoxDetection', None),
    'bipartite_matching': ('_contrib_bipartite_matching', None),
    'intgemm_maxabsolute': ('_contrib_intgemm_maxabsolute', None),
    'intgemm_prepare_data': ('_contrib_intgemm_prepare_data', None),
    'intgemm_prepare_weight': ('_contrib_intgemm_prepare_weight', None),
    'intgemm_take_weight': ('_contrib_intgemm_take_weight', None),
    'intgemm_fully_connected': ('_contrib_intgemm_fully_connected', None),
}

__all__ = ['set_np', 'reset_np', 'is_np_array', 'is_np_shape', 'use_np', 'use_np_array', 'use_np_shape', 'np_array',
           'np_shape', 'cpu', 'gpu', 'num_gpus', 'current_context', 'waitall', 'save', 'load', 'seed', 'reshape',
           'nonzero', 'random', 'image', 'sigmoid', 'relu'] + list(_MAP)

for _name, (_opn, _defaults) in _MAP.items():
    globals()[_name] = _op(_opn, _defaults, pyname=_name)


def reshape(a, newshape, reverse=False, order='C'):
    """Reshape with npx special codes (-1 infer, -2 copy, -3 drop unit dim, -4 copy rest, -5 merge, -6 split)."""
    if _is_sym(a):
        from ..symbol.symbol import _op_func
        return _op_func('_npx_reshape')(a, newshape=tuple(newshape), reverse=reverse, order=order)
    from ..numpy.multiarray import _call
    return _call('_npx_reshape', a, newshape=tuple(newshape) if not isinstance(newshape, int) else (newshape,),
                 reverse=reverse, order=order)


@_host_graph('npx_nonzero')
def nonzero(a):
    """Indices of non-zero elements as an ``(N, ndim)`` int64 array (a 0-d input counts as 1-d,
    as in src/operator/numpy/np_nonzero_op.cc)."""
    import torch
    from ..numpy import ndarray
    t = a._data
    return ndarray(torch.nonzero(t.reshape(1) if t.dim() == 0 else t))


def seed(seed=None, ctx='all', **kwargs):  # pylint: disable=redefined-outer-name
    from .. import random as _r
    _r.seed(seed if seed is not None else kwargs.get('s'), ctx)


def save(file, arr):
    """Save an ndarray, list or dict of ndarrays (``.params``/npz-like container)."""
    from ..ndarray import utils as _u
    if isinstance(arr, NDArray):
        arr = [arr]
    if isinstance(arr, dict):
        arr = {k: v.as_nd_ndarray() if hasattr(v, 'as_nd_ndarray') else v for k, v in arr.items()}
    else:
        arr = [v.as_nd_ndarray() if hasattr(v, 'as_nd_ndarray') else v for v in arr]
    _u.save(file, arr, np_shape=True)


def load(file):
    from ..ndarray import utils as _u
    from ..util import np_shape as _np_shape
    with _np_shape(True):            # npx.save writes numpy-shape-semantics (V3) records
        r = _u.load(file)
    if isinstance(r, dict):
        return {k: v.as_np_ndarray() for k, v in r.items()}
    return [v.as_np_ndarray() for v in r]


class _Namespace:
    def __init__(self, name, entries):
        self.__name__ = name
        self.__dict__.update(entries)


def _random_ns():
    import torch
    from ..numpy import ndarray, random as nprand

    def bernoulli(prob=None, logit=None, size=None, dtype=None, ctx=None, out=None):
        """Bernoulli samples from ``prob`` or ``logit`` (exactly one of them; probabilities outside
        [0, 1] raise ValueError, as src/operator/numpy/random/np_bernoulli_op.h checks)."""
        from ..numpy.multiarray import _call
        if (prob is None) == (logit is None):
            raise ValueError('bernoulli: exactly one of prob and logit must be given')
        shp = None if size is None else ((size,) if isinstance(size, int) else tuple(size))
        if logit is not None:
            p = torch.sigmoid(logit._data.double()) if isinstance(logit, NDArray) else \
                torch.tensor(1.0 / (1.0 + __import__('math').exp(-logit)), dtype=torch.float64)
        elif isinstance(prob, NDArray):
            p = prob._data
            if p.numel() and (bool((p < 0).any()) or bool((p > 1).any())):
                raise ValueError('bernoulli: prob must lie in [0, 1]')
        else:
            if not 0.0 <= float(prob) <= 1.0:
                raise ValueError('bernoulli: prob must lie in [0, 1]')
            return _call('_npi_bernoulli', prob=float(prob), size=shp or (), ctx=ctx or current_context(),
                         dtype=dtype or 'float32')
        shp = tuple(p.shape) if shp is None else shp
        r = torch.rand(shp, device=p.device, dtype=torch.float64) < p.double()
        res = ndarray(r.to(_torch_dtype(dtype or 'float32')))
        if out is not None:
            out[...] = res
            return out
        return res

    def uniform_n(low=0.0, high=1.0, batch_shape=None, dtype=None, ctx=None):
        # output shape = batch_shape + the parameters' broadcast shape (reference: np_random_n ops)
        return nprand._sample('uniform', (low, high), batch_shape, dtype, ctx, batch=True)

    def normal_n(loc=0.0, scale=1.0, batch_shape=None, dtype=None, ctx=None):
        return nprand._sample('normal', (loc, scale), batch_shape, dtype, ctx, batch=True)
    return _Namespace('mxnet.numpy_extension.random', {'seed': seed, 'bernoulli': bernoulli,
                                                       'uniform_n': uniform_n, 'normal_n': normal_n})


def _image_ns():
    ents = {}
    for n, opn in (('to_tensor', '_image_to_tensor'), ('normalize', '_image_normalize'), ('resize', '_image_resize'),
                   ('crop', '_image_crop'), ('flip_left_right', '_image_flip_left_right'),
                   ('random_flip_left_right', '_image_random_flip_left_right'),
                   ('flip_top_bottom', '_image_flip_top_bottom'),
                   ('random_flip_top_bottom', '_image_random_flip_top_bottom'),
                   ('random_brightness', '_image_random_brightness'), ('random_contrast', '_image_random_contrast'),
                   ('random_saturation', '_image_random_saturation'), ('random_hue', '_image_random_hue'),
                   ('random_color_jitter', '_image_random_color_jitter'), ('adjust_lighting', '_image_adjust_lighting'),
                   ('random_lighting', '_image_random_lighting')):
        if _registry.has(opn):
            ents[n] = _op(opn, pyname=n)
    return _Namespace('mxnet.numpy_extension.image', ents)


random = _random_ns()
image = _image_ns()
