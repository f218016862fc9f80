"""Neural-network operators.

Parity: src/operator/nn/*.cc (convolution, deconvolution, fully_connected,
batch_norm, pooling, activation, leaky_relu, softmax, dropout, layer_norm,
group_norm, lrn, upsampling, ctc_loss, moments), src/operator/*.cc
(softmax_output, regression_output, make_loss, instance_norm,
l2_normalization, roi_pooling, sequence_*, rnn, bilinear_sampler,
grid_generator, spatial_transformer, correlation, crop, svm_output,
identity_attach_KL_sparse_reg).

Layout: every spatial op accepts MXNet's ``layout`` attribute. Channel-last
layouts (NWC/NHWC/NDHWC) are the fast path on MI355X: the tensor is handed to
the HIP kernels (ops/hip_ops.py) directly, and the torch reference path views
it as a channels_last NCHW tensor (zero copies).
"""
import math
import os

import torch
import torch.nn.functional as F

from .. import _state
from ..base import torch_dtype, MXNetError
from .registry import register
from . import hip_ops

# ---------------------------------------------------------------------------
# helpers
# ---------------------------------------------------------------------------


def _acc(t):
    """Accumulation dtype: fp32 for fp16/bf16/fp32 inputs, fp64 stays fp64 (reference CPU semantics)."""
    return t if t.dtype == torch.float64 else t.float()


def _is_channel_last(layout):
    return layout is not None and layout.endswith('C') and len(layout) > 2


def _to_ncx(x, layout):
    """NHWC view -> NCHW view (channels_last strides, no copy)."""
    if _is_channel_last(layout):
        nd = x.dim()
        return x.permute(0, nd - 1, *range(1, nd - 1))
    return x


def _from_ncx(x, layout):
    if _is_channel_last(layout):
        nd = x.dim()
        return x.permute(0, *range(2, nd), 1)
    return x


def _tup(v, n, default):
    if v is None or len(v) == 0:
        return (default,) * n
    if len(v) == 1 and n > 1:
        return tuple(v) * n
    return tuple(v)


# ---------------------------------------------------------------------------
# FullyConnected
# ---------------------------------------------------------------------------

def _fc_args(a):
    nb = a.get('no_bias', False)
    nb = nb if isinstance(nb, bool) else str(nb) in ('True', 'true', '1')
    return ['data', 'weight'] if nb else ['data', 'weight', 'bias']


def _fc_infer(in_shapes, a):
    d = in_shapes[0]
    if d is None:
        return {}
    flatten = a.get('flatten', True)
    k = int(math.prod(d[1:])) if flatten else d[-1]
    res = {1: (a['num_hidden'], k)}
    if not a.get('no_bias', False):
        res[2] = (a['num_hidden'],)
    return res


@register('FullyConnected', arg_names=_fc_args, infer_params=_fc_infer,
          params={'num_hidden': ('int', 0), 'no_bias': ('bool', False), 'flatten': ('bool', True)})
def fully_connected(data, weight, bias=None, num_hidden=0, no_bias=False, flatten=True):
    if flatten and data.dim() != 2:
        data = data.reshape(data.shape[0], -1)
    if bias is not None and bias.dim() != 1:
        bias = bias.reshape(-1)          # a (num_hidden, 1) bias (e.g. row_sparse) is the same vector
    return hip_ops.linear(data, weight, bias)


# ---------------------------------------------------------------------------
# Convolution / Deconvolution
# ---------------------------------------------------------------------------

def _conv_args(a):
    nb = a.get('no_bias', False)
    nb = nb if isinstance(nb, bool) else str(nb) in ('True', 'true', '1')
    return ['data', 'weight'] if nb else ['data', 'weight', 'bias']


def _conv_infer(in_shapes, a):
    d = in_shapes[0]
    if d is None:
        return {}
    k = tuple(a['kernel'])
    layout = a.get('layout') or {1: 'NCW', 2: 'NCHW', 3: 'NCDHW'}[len(k)]
    g = a.get('num_group', 1) or 1
    c = d[-1] if _is_channel_last(layout) else d[1]
    if _is_channel_last(layout):
        w = (a['num_filter'],) + k + (c // g,)
    else:
        w = (a['num_filter'], c // g) + k
    res = {1: w}
    if not a.get('no_bias', False):
        res[2] = (a['num_filter'],)
    return res


_CONV_PARAMS = {'kernel': ('shape', ()), 'stride': ('shape', ()), 'dilate': ('shape', ()),
                'pad': ('shape', ()), 'num_filter': ('int', 0), 'num_group': ('int', 1),
                'workspace': ('int', 1024), 'no_bias': ('bool', False), 'cudnn_tune': ('str?', None),
                'cudnn_off': ('bool', False), 'layout': ('str?', None)}


@register('Convolution', aliases=('Convolution_v1',), arg_names=_conv_args, infer_params=_conv_infer,
          params=_CONV_PARAMS)
def convolution(data, weight, bias=None, kernel=(), stride=(), dilate=(), pad=(), num_filter=0,
                num_group=1, workspace=1024, no_bias=False, cudnn_tune=None, cudnn_off=False, layout=None):
    nsp = len(kernel)
    stride = _tup(stride, nsp, 1)
    dilate = _tup(dilate, nsp, 1)
    pad = _tup(pad, nsp, 0)
    return hip_ops.conv(data, weight, bias, stride, pad, dilate, num_group,
                        _is_channel_last(layout))


@register('_contrib_ConvolutionTee', aliases=('ConvolutionTee',), arg_names=('data', 'weight'),
          infer_params=_conv_infer, num_outputs=2,
          params=dict(_CONV_PARAMS, no_bias=('bool', True), inplace_shortcut_grad=('bool', False)))
def convolution_tee(data, weight, kernel=(1, 1), stride=(), dilate=(), pad=(), num_filter=0, num_group=1,
                    workspace=1024, no_bias=True, cudnn_tune=None, cudnn_off=False, layout=None,
                    inplace_shortcut_grad=False):
    """Channel-last 1x1 convolution that also passes its input through (second output) for an identity
    shortcut; on gfx950 the shortcut's gradient is folded into the dgrad GEMM (beta=1) instead of a
    separate add.  Semantically ``(Convolution(data, weight), data)``.  ``inplace_shortcut_grad``: the
    pass-through output's only consumer returns a freshly allocated gradient for it (e.g. the fused
    BatchNormAddReLU tail), so the GEMM may accumulate into that buffer without a copy."""
    if tuple(kernel) != (1, 1) or tuple(stride or (1, 1)) != (1, 1) or tuple(pad or (0, 0)) != (0, 0) \
            or not _is_channel_last(layout) or num_group != 1:
        raise ValueError('ConvolutionTee: only channel-last 1x1 stride-1 convolutions')
    return hip_ops.conv_tee(data, weight, inplace_shortcut_grad)


def _deconv_infer(in_shapes, a):
    d = in_shapes[0]
    if d is None:
        return {}
    k = tuple(a['kernel'])
    layout = a.get('layout') or {1: 'NCW', 2: 'NCHW', 3: 'NCDHW'}[len(k)]
    g = a.get('num_group', 1) or 1
    c = d[-1] if _is_channel_last(layout) else d[1]
    if _is_channel_last(layout):
        w = (c,) + k + (a['num_filter'] // g,)
    else:
        w = (c, a['num_filter'] // g) + k
    res = {1: w}
    if not a.get('no_bias', True):
        res[2] = (a['num_filter'],)
    return res


def _deconv_args(a):
    nb = a.get('no_bias', True)
    nb = nb if isinstance(nb, bool) else str(nb) in ('True', 'true', '1')
    return ['data', 'weight'] if nb else ['data', 'weight', 'bias']


@register('Deconvolution', arg_names=_deconv_args, infer_params=_deconv_infer,
          params=dict(_CONV_PARAMS, adj=('shape', ()), target_shape=('shape', ()), no_bias=('bool', True)))
def deconvolution(data, weight, bias=None, kernel=(), stride=(), dilate=(), pad=(), adj=(), target_shape=(),
                  num_filter=0, num_group=1, workspace=1024, no_bias=True, cudnn_tune=None,
                  cudnn_off=False, layout=None):
    nsp = len(kernel)
    stride = _tup(stride, nsp, 1)
    dilate = _tup(dilate, nsp, 1)
    pad = list(_tup(pad, nsp, 0))
    adj = list(_tup(adj, nsp, 0))
    x = _to_ncx(data, layout)
    w = _to_ncx(weight, layout)
    if target_shape:
        for i in range(nsp):
            full = (x.shape[2 + i] - 1) * stride[i] + dilate[i] * (kernel[i] - 1) + 1
            tot = full - target_shape[i]
            pad[i] = (tot + 1) // 2
            adj[i] = tot % 2
    if data.is_cuda and hip_ops._use_hip(data):
        # in-tree transposed convolution (the data gradient of a conv, src/kernels/conv_gen.hip)
        from . import conv_gen
        y = conv_gen.deconv(data, weight, bias, stride, pad, dilate, adj, num_group, _is_channel_last(layout))
        if y is not None:
            return y
    fn = {1: F.conv_transpose1d, 2: F.conv_transpose2d, 3: F.conv_transpose3d}[nsp]
    y = fn(x, w, bias, stride=stride, padding=pad, output_padding=adj, groups=num_group, dilation=dilate)
    return _from_ncx(y, layout)


# ---------------------------------------------------------------------------
# BatchNorm
# ---------------------------------------------------------------------------

def _bn_infer(in_shapes, a):
    d = in_shapes[0]
    if d is None:
        return {}
    c = d[a.get('axis', 1) % len(d)]
    return {1: (c,), 2: (c,), 3: (c,), 4: (c,)}


_BN_PARAMS = {'eps': ('float', 1e-3), 'momentum': ('float', 0.9), 'fix_gamma': ('bool', True),
              'use_global_stats': ('bool', False), 'output_mean_var': ('bool', False),
              'axis': ('int', 1), 'cudnn_off': ('bool', False), 'act_type': ('str?', None),
              'min_calib_range': ('float?', None), 'max_calib_range': ('float?', None)}


def _bn_nvis(a):
    o = a.get('output_mean_var', False)
    o = o if isinstance(o, bool) else str(o) in ('True', 'true', '1')
    return 3 if o else 1


@register('BatchNorm', aliases=('BatchNorm_v1', 'CuDNNBatchNorm'),
          arg_names=('data', 'gamma', 'beta'), aux_names=('moving_mean', 'moving_var'),
          num_outputs=3, num_visible_outputs=_bn_nvis, infer_params=_bn_infer, params=_BN_PARAMS,
          output_names=('output', 'mean', 'var'))
def batch_norm(data, gamma, beta, moving_mean, moving_var, eps=1e-3, momentum=0.9, fix_gamma=True,
               use_global_stats=False, output_mean_var=False, axis=1, cudnn_off=False, act_type=None,
               min_calib_range=None, max_calib_range=None):
    training = _state.STATE.training and not use_global_stats
    return hip_ops.batch_norm(data, gamma, beta, moving_mean, moving_var, eps, momentum, fix_gamma,
                              training, axis, act_type, invstd_out=True)


@register('_contrib_BatchNormWithReLU', aliases=('BatchNormWithReLU',),
          arg_names=('data', 'gamma', 'beta'), aux_names=('moving_mean', 'moving_var'),
          num_outputs=3, num_visible_outputs=_bn_nvis, infer_params=_bn_infer, params=_BN_PARAMS)
def batch_norm_relu(data, gamma, beta, moving_mean, moving_var, eps=1e-3, momentum=0.9, fix_gamma=True,
                    use_global_stats=False, output_mean_var=False, axis=1, cudnn_off=False, act_type=None,
                    min_calib_range=None, max_calib_range=None):
    training = _state.STATE.training and not use_global_stats
    return hip_ops.batch_norm(data, gamma, beta, moving_mean, moving_var, eps, momentum, fix_gamma,
                              training, axis, 'relu', invstd_out=True)


_BNPOOL_PARAMS = dict(_BN_PARAMS, kernel=('shape', (3, 3)), stride=('shape', (2, 2)), pad=('shape', (1, 1)))


@register('_contrib_BatchNormReLUMaxPool', aliases=('BatchNormReLUMaxPool',),
          arg_names=('data', 'gamma', 'beta'), aux_names=('moving_mean', 'moving_var'),
          num_outputs=3, num_visible_outputs=_bn_nvis, infer_params=_bn_infer, params=_BNPOOL_PARAMS)
def batch_norm_relu_maxpool(data, gamma, beta, moving_mean, moving_var, eps=1e-3, momentum=0.9, fix_gamma=True,
                            use_global_stats=False, output_mean_var=False, axis=1, cudnn_off=False, act_type=None,
                            min_calib_range=None, max_calib_range=None, kernel=(3, 3), stride=(2, 2), pad=(1, 1)):
    """``Pooling(relu(BatchNorm(data)), pool_type='max')`` (valid convention): the ResNet stem's BatchNorm,
    ReLU and 3x3/2 max pooling as one operator -- the pooling kernel applies the normalisation to each
    window tap, so the normalised full-resolution activation is never written (pool_nhwc.hip). Outputs
    and moving-statistics updates are BatchNorm's; the first output is pooled."""
    training = _state.STATE.training and not use_global_stats
    return hip_ops.batch_norm_relu_maxpool(data, gamma, beta, moving_mean, moving_var, eps, momentum, fix_gamma,
                                           training, axis, _tup(kernel, 2, 1), _tup(stride, 2, 1), _tup(pad, 2, 0),
                                           invstd_out=True)


@register('_contrib_BatchNormAddReLU', aliases=('BatchNormAddReLU',),
          arg_names=('data', 'addend', 'gamma', 'beta'), aux_names=('moving_mean', 'moving_var'),
          num_outputs=3, num_visible_outputs=_bn_nvis,
          infer_params=lambda s, a: {k + 1: v for k, v in _bn_infer(s, a).items() if k + 1 <= 5 and k > 0},
          params=_BN_PARAMS)
def batch_norm_add_relu(data, addend, gamma, beta, moving_mean, moving_var, eps=1e-3, momentum=0.9,
                        fix_gamma=True, use_global_stats=False, output_mean_var=False, axis=1,
                        cudnn_off=False, act_type=None, min_calib_range=None, max_calib_range=None):
    """Fused ``relu(BN(data) + addend)`` (the ResNet bottleneck tail)."""
    training = _state.STATE.training and not use_global_stats
    return hip_ops.batch_norm(data, gamma, beta, moving_mean, moving_var, eps, momentum, fix_gamma,
                              training, axis, 'relu', addend=addend)


# ---------------------------------------------------------------------------
# Pooling
# ---------------------------------------------------------------------------

_POOL_PARAMS = {'kernel': ('shape', ()), 'pool_type': ('str', 'max'), 'global_pool': ('bool', False),
                'cudnn_off': ('bool', False), 'pooling_convention': ('str', 'valid'),
                'stride': ('shape', ()), 'pad': ('shape', ()), 'p_value': ('int?', None),
                'count_include_pad': ('bool?', None), 'layout': ('str?', None)}


@register('Pooling', aliases=('Pooling_v1',), params=_POOL_PARAMS)
def pooling(data, kernel=(), pool_type='max', global_pool=False, cudnn_off=False,
            pooling_convention='valid', stride=(), pad=(), p_value=None, count_include_pad=None,
            layout=None):
    nsp = data.dim() - 2
    if count_include_pad is None:
        count_include_pad = True
    if global_pool:
        return hip_ops.global_pool(data, pool_type, _is_channel_last(layout))
    kernel = _tup(kernel, nsp, 1)
    stride = _tup(stride, nsp, 1)
    if pooling_convention == 'same':
        # the 'same' convention derives its own padding (output = ceil(input / stride))
        if any(int(p) != 0 for p in (pad or ())):
            raise MXNetError('Pooling: pad must be 0 with pooling_convention=same, got %s' % (tuple(pad),))
        pad = (0,) * nsp
    pad = _tup(pad, nsp, 0)
    return hip_ops.pool(data, pool_type, kernel, stride, pad, pooling_convention,
                        count_include_pad, _is_channel_last(layout), p_value)


@register('_contrib_AdaptiveAvgPooling2D', aliases=('AdaptiveAvgPooling2D',), params={'output_size': ('shape', ())})
def adaptive_avg_pool2d(data, output_size=()):
    os_ = tuple(output_size) if output_size else (1, 1)
    if len(os_) == 1:
        os_ = os_ * 2
    return F.adaptive_avg_pool2d(data, os_)


@register('_contrib_BilinearResize2D', aliases=('BilinearResize2D',), arg_names=lambda a: ['data'] if a.get('mode', 'size') != 'like' else ['data', 'like'],
          params={'height': ('int', 1), 'width': ('int', 1), 'scale_height': ('float?', None),
                  'scale_width': ('float?', None), 'mode': ('str', 'size'), 'align_corners': ('bool', True)})
def bilinear_resize2d(data, like=None, height=1, width=1, scale_height=None, scale_width=None, mode='size',
                      align_corners=True):
    if mode == 'like' and like is not None:
        height, width = like.shape[2], like.shape[3]
    elif scale_height is not None:
        height, width = int(data.shape[2] * scale_height), int(data.shape[3] * (scale_width or scale_height))
    elif mode == 'odd_scale':
        pass
    return F.interpolate(data, size=(height, width), mode='bilinear', align_corners=align_corners)


# ---------------------------------------------------------------------------
# Activations
# ---------------------------------------------------------------------------

_ACTS = {
    'relu': torch.relu, 'sigmoid': torch.sigmoid, 'tanh': torch.tanh,
    'softrelu': F.softplus, 'softsign': F.softsign, 'log_sigmoid': F.logsigmoid,
    'mish': F.mish,
}


@register('Activation', params={'act_type': ('str', 'relu')})
def activation(data, act_type='relu'):
    if act_type == 'relu':
        return hip_ops.relu(data)
    return _ACTS[act_type](data)


def _lrelu_args(a):
    return ['data', 'gamma'] if a.get('act_type', 'leaky') == 'prelu' else ['data']


def _lrelu_infer(in_shapes, a):
    if a.get('act_type') != 'prelu' or in_shapes[0] is None:
        return {}
    d = in_shapes[0]
    return {1: (d[1] if len(d) > 1 else 1,)}


@register('LeakyReLU', arg_names=_lrelu_args, infer_params=_lrelu_infer, num_outputs=1,
          params={'act_type': ('str', 'leaky'), 'slope': ('float', 0.25), 'lower_bound': ('float', 0.125),
                  'upper_bound': ('float', 0.334)})
def leaky_relu(data, gamma=None, act_type='leaky', slope=0.25, lower_bound=0.125, upper_bound=0.334):
    if act_type == 'leaky':
        return F.leaky_relu(data, slope)
    if act_type == 'prelu':
        if gamma.dim() > 1:     # a per-(batch, channel) gamma broadcast over trailing axes
            g = gamma.reshape(tuple(gamma.shape) + (1,) * (data.dim() - gamma.dim()))
        else:
            g = gamma.reshape((1, -1) + (1,) * (data.dim() - 2)) if data.dim() > 1 else gamma
        return torch.where(data >= 0, data, data * g)
    if act_type == 'elu':
        return F.elu(data, slope)
    if act_type == 'selu':
        return F.selu(data)
    if act_type == 'gelu':
        return hip_ops.gelu(data)
    if act_type == 'rrelu':
        if _state.STATE.training:
            a = torch.empty_like(data).uniform_(lower_bound, upper_bound)
            return torch.where(data >= 0, data, data * a)
        return F.leaky_relu(data, (lower_bound + upper_bound) / 2)
    raise MXNetError('unknown act_type %s' % act_type)


# ---------------------------------------------------------------------------
# softmax family
# ---------------------------------------------------------------------------

def _softmax_args(a):
    ul = a.get('use_length', False)
    ul = ul if isinstance(ul, bool) else str(ul) in ('True', 'true', '1')
    return ['data', 'length'] if ul else ['data']


def _length_mask(data, length, axis):
    n = data.shape[axis]
    ar = torch.arange(n, device=data.device)
    shape = [1] * data.dim()
    shape[axis] = n
    ar = ar.reshape(shape)
    lshape = list(data.shape)
    lshape[axis] = 1
    return ar < length.reshape(lshape).to(ar.dtype)


_SM_PARAMS = {'axis': ('int', -1), 'temperature': ('float?', None), 'dtype': ('str?', None),
              'use_length': ('bool', False)}


@register('softmax', arg_names=_softmax_args, params=_SM_PARAMS)
def softmax(data, length=None, axis=-1, temperature=None, dtype=None, use_length=False):
    if not (length is not None and use_length) and (dtype is None or torch_dtype(dtype) == data.dtype):
        r = hip_ops.softmax(data, axis, 1.0 / temperature if temperature else 1.0)
        if r is not None:
            return r
    x = data if temperature is None or temperature == 1.0 else data / temperature
    if length is not None and use_length:
        m = _length_mask(x, length, axis % x.dim())
        x = x.masked_fill(~m, float('-inf'))
        r = torch.softmax(_acc(x), dim=axis)
        r = torch.nan_to_num(r, nan=0.0).masked_fill(~m, 0.0)
    else:
        r = torch.softmax(x, dim=axis, dtype=torch.float32) if x.dtype in (torch.float16, torch.bfloat16) else torch.softmax(x, dim=axis)
    return r.to(torch_dtype(dtype) if dtype else data.dtype)


@register('log_softmax', arg_names=_softmax_args, params=_SM_PARAMS)
def log_softmax(data, length=None, axis=-1, temperature=None, dtype=None, use_length=False):
    if dtype is None or torch_dtype(dtype) == data.dtype:
        r = hip_ops.softmax(data, axis, 1.0 / temperature if temperature else 1.0, log=True)
        if r is not None:
            return r
    x = data if temperature is None or temperature == 1.0 else data / temperature
    r = torch.log_softmax(x.float() if x.dtype in (torch.float16, torch.bfloat16) else x, dim=axis)
    return r.to(torch_dtype(dtype) if dtype else data.dtype)


@register('softmin', arg_names=_softmax_args, params=_SM_PARAMS)
def softmin(data, length=None, axis=-1, temperature=None, dtype=None, use_length=False):
    return softmax(-data, length, axis, temperature, dtype, use_length)


@register('SoftmaxActivation', params={'mode': ('str', 'instance')})
def softmax_activation(data, mode='instance'):
    if mode == 'channel':
        return torch.softmax(data, dim=1)
    return torch.softmax(data.reshape(data.shape[0], -1), dim=1).reshape(data.shape)


class _SoftmaxOutputFn(torch.autograd.Function):
    """softmax forward; backward = (p - onehot(label)) * scale (softmax_output-inl.h)."""

    @staticmethod
    def forward(ctx, data, label, grad_scale, ignore_label, multi_output, use_ignore,
                preserve_shape, normalization, smooth_alpha):
        if multi_output:
            n, c = data.shape[0], data.shape[1]
            x = data.reshape(n, c, -1)
            p = torch.softmax(_acc(x), dim=1)
        elif preserve_shape:
            p = torch.softmax(_acc(data), dim=-1)
        else:
            p = torch.softmax(_acc(data.reshape(data.shape[0], -1)), dim=1)
        ctx.save_for_backward(p, label)
        ctx.cfg = (grad_scale, ignore_label, multi_output, use_ignore, preserve_shape, normalization,
                   smooth_alpha, data.shape, data.dtype)
        return p.reshape(data.shape).to(data.dtype)

    @staticmethod
    def backward(ctx, g):
        p, label = ctx.saved_tensors
        grad_scale, ignore_label, multi_output, use_ignore, preserve_shape, norm, alpha, shape, dt = ctx.cfg
        if multi_output:
            n, c = p.shape[0], p.shape[1]
            lab = label.reshape(n, -1).to(torch.int64)
            oh = torch.zeros_like(p).scatter_(1, lab.clamp(0, c - 1).unsqueeze(1), 1.0)
            if alpha:
                oh = oh * (1 - alpha) + (1 - oh) * alpha / (c - 1)
            grad = p - oh
            valid = torch.ones_like(lab, dtype=p.dtype)
            if use_ignore:
                valid = (lab != int(ignore_label)).to(p.dtype)
                grad = grad * valid.unsqueeze(1)
        elif tuple(label.shape) == tuple(shape):
            # a label of the data's shape is a probability distribution (reference: no one-hot)
            p2 = p.reshape(-1, p.shape[-1])
            grad = p2 - label.reshape(p2.shape).to(p2.dtype)
            valid = torch.ones(p2.shape[0], dtype=p.dtype, device=p.device)
        else:
            p2 = p.reshape(-1, p.shape[-1])
            c = p2.shape[-1]
            lab = label.reshape(-1).to(torch.int64)
            oh = torch.zeros_like(p2).scatter_(1, lab.clamp(0, c - 1).unsqueeze(1), 1.0)
            if alpha:
                oh = oh * (1 - alpha) + (1 - oh) * alpha / (c - 1)
            grad = p2 - oh
            valid = torch.ones_like(lab, dtype=p.dtype)
            if use_ignore:
                valid = (lab != int(ignore_label)).to(p.dtype)
                grad = grad * valid.unsqueeze(1)
        if norm == 'batch':
            grad = grad / shape[0]
        elif norm == 'valid':
            grad = grad / torch.clamp(valid.sum(), min=1.0)
        if multi_output and norm != 'valid':
            spatial = 1
            for d in shape[2:]:
                spatial *= d
            grad = grad / spatial       # reference softmax_output-inl.h: per-position average
        grad = grad * grad_scale
        return grad.reshape(shape).to(dt), None, None, None, None, None, None, None, None


@register('SoftmaxOutput', aliases=('Softmax',), arg_names=('data', 'label'),
          params={'grad_scale': ('float', 1.0), 'ignore_label': ('float', -1.0), 'multi_output': ('bool', False),
                  'use_ignore': ('bool', False), 'preserve_shape': ('bool', False),
                  'normalization': ('str', 'null'), 'out_grad': ('bool', False), 'smooth_alpha': ('float', 0.0)},
          infer_params=lambda s, a: ({1: (s[0][0],) if not a.get('multi_output') else (s[0][0],) + tuple(s[0][2:])}
                                     if s[0] is not None else {}))
def softmax_output(data, label, grad_scale=1.0, ignore_label=-1.0, multi_output=False, use_ignore=False,
                   preserve_shape=False, normalization='null', out_grad=False, smooth_alpha=0.0):
    return _SoftmaxOutputFn.apply(data, label, grad_scale, ignore_label, multi_output, use_ignore,
                                  preserve_shape, normalization, smooth_alpha)


class _RegressionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, data, label, kind, grad_scale):
        out = torch.sigmoid(data) if kind == 'logistic' else data.clone()
        ctx.save_for_backward(out, label)
        ctx.kind, ctx.scale = kind, grad_scale
        return out

    @staticmethod
    def backward(ctx, g):
        out, label = ctx.saved_tensors
        lab = label.reshape(out.shape)
        num_output = label.numel() / label.shape[0]
        if ctx.kind == 'mae':
            grad = torch.sign(out - lab)
        else:
            grad = out - lab
        return grad * (ctx.scale / num_output), None, None, None


def _reg(kind):
    def f(data, label, grad_scale=1.0):
        return _RegressionFn.apply(data, label, kind, grad_scale)
    return f


_REG_INFER = lambda s, a: ({1: s[0]} if s[0] is not None else {})
register('LinearRegressionOutput', _reg('linear'), arg_names=('data', 'label'),
         params={'grad_scale': ('float', 1.0)}, infer_params=_REG_INFER)
register('MAERegressionOutput', _reg('mae'), arg_names=('data', 'label'),
         params={'grad_scale': ('float', 1.0)}, infer_params=_REG_INFER)
register('LogisticRegressionOutput', _reg('logistic'), arg_names=('data', 'label'),
         params={'grad_scale': ('float', 1.0)}, infer_params=_REG_INFER)


class _SVMOutputFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, data, label, margin, reg, use_linear):
        ctx.save_for_backward(data, label)
        ctx.cfg = (margin, reg, use_linear)
        return data.clone()

    @staticmethod
    def backward(ctx, g):
        data, label = ctx.saved_tensors
        margin, reg, use_linear = ctx.cfg
        n, c = data.shape
        lab = label.to(torch.int64)
        y = -torch.ones_like(data)
        y.scatter_(1, lab.unsqueeze(1), 1.0)
        viol = (margin - y * data) > 0
        if use_linear:
            grad = torch.where(viol, -y, torch.zeros_like(data)) * reg
        else:
            grad = torch.where(viol, -2 * y * (margin - y * data), torch.zeros_like(data)) * reg
        return grad, None, None, None, None


@register('SVMOutput', arg_names=('data', 'label'),
          params={'margin': ('float', 1.0), 'regularization_coefficient': ('float', 1.0),
                  'use_linear': ('bool', False)},
          infer_params=lambda s, a: ({1: (s[0][0],)} if s[0] is not None else {}))
def svm_output(data, label, margin=1.0, regularization_coefficient=1.0, use_linear=False):
    return _SVMOutputFn.apply(data, label, margin, regularization_coefficient, use_linear)


class _MakeLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, data, grad_scale, valid_thresh, normalization):
        ctx.cfg = (grad_scale, valid_thresh, normalization)
        ctx.save_for_backward(data)
        return data.clone()

    @staticmethod
    def backward(ctx, g):
        data, = ctx.saved_tensors
        scale, thresh, norm = ctx.cfg
        grad = torch.full_like(data, scale)
        if norm == 'batch':
            grad = grad / data.shape[0]
        elif norm == 'valid':
            grad = grad / torch.clamp((data > thresh).sum(), min=1)
        return grad, None, None, None


@register('MakeLoss', aliases=('make_loss',),
          params={'grad_scale': ('float', 1.0), 'valid_thresh': ('float', 0.0), 'normalization': ('str', 'null')})
def make_loss(data, grad_scale=1.0, valid_thresh=0.0, normalization='null'):
    return _MakeLossFn.apply(data, grad_scale, valid_thresh, normalization)


@register('softmax_cross_entropy', arg_names=('data', 'label'))
def softmax_cross_entropy(data, label):
    return hip_ops.softmax_ce(data, label, reduction='sum').reshape(1)


# ---------------------------------------------------------------------------
# Dropout / Embedding
# ---------------------------------------------------------------------------

@register('Dropout', num_outputs=2, num_visible_outputs=1, output_names=('output', 'mask'),
          params={'p': ('float', 0.5), 'mode': ('str', 'training'), 'axes': ('shape', ()),
                  'cudnn_off': ('bool?', False)})
def dropout(data, p=0.5, mode='training', axes=(), cudnn_off=False):
    active = (mode == 'always') or _state.STATE.training
    if not active or p == 0:
        return data, torch.ones_like(data)
    if not axes:
        r = hip_ops.dropout(data, p)
        if r is not None:
            return r
    if axes:
        mshape = [1 if i in axes else s for i, s in enumerate(data.shape)]
        mask = (torch.rand(mshape, device=data.device) >= p).to(data.dtype) / (1 - p)
    else:
        mask = (torch.rand_like(data, dtype=torch.float32) >= p).to(data.dtype) / (1 - p)
    return data * mask, mask


@register('Embedding', arg_names=('data', 'weight'),
          infer_params=lambda s, a: {1: (a['input_dim'], a['output_dim'])},
          params={'input_dim': ('int', 0), 'output_dim': ('int', 0), 'dtype': ('str', 'float32'),
                  'sparse_grad': ('bool', False)})
def embedding(data, weight, input_dim=0, output_dim=0, dtype='float32', sparse_grad=False):
    r = hip_ops.embedding(data, weight)
    if r is not None:
        return r
    idx = torch.clamp(data.to(torch.int64), 0, weight.shape[0] - 1)
    return F.embedding(idx, weight)


# ---------------------------------------------------------------------------
# Normalisation layers
# ---------------------------------------------------------------------------

def _ln_nvis(a):
    o = a.get('output_mean_var', False)
    o = o if isinstance(o, bool) else str(o) in ('True', 'true', '1')
    return 3 if o else 1


@register('LayerNorm', arg_names=('data', 'gamma', 'beta'), num_outputs=3, num_visible_outputs=_ln_nvis,
          infer_params=lambda s, a: ({1: (s[0][a.get('axis', -1)],), 2: (s[0][a.get('axis', -1)],)}
                                     if s[0] is not None else {}),
          params={'axis': ('int', -1), 'eps': ('float', 1e-5), 'output_mean_var': ('bool', False)})
def layer_norm(data, gamma, beta, axis=-1, eps=1e-5, output_mean_var=False):
    axis = axis % data.dim()
    if axis == data.dim() - 1:
        return hip_ops.layer_norm(data, gamma, beta, eps, output_mean_var)
    x = _acc(data)
    mean = x.mean(dim=axis, keepdim=True)
    var = x.var(dim=axis, keepdim=True, unbiased=False)
    std = torch.sqrt(var + eps)
    shape = [1] * data.dim()
    shape[axis] = -1
    y = (x - mean) / std * _acc(gamma.reshape(shape)) + _acc(beta.reshape(shape))
    return y.to(data.dtype), mean.to(data.dtype), std.to(data.dtype)


def _adln_infer(s):
    shape = s[0] if s[0] is not None else s[1]
    if shape is None:
        return {}
    return {0: tuple(shape), 1: tuple(shape), 2: (shape[-1],), 3: (shape[-1],)}


@register('_contrib_add_dropout_layernorm', aliases=('add_dropout_layernorm',),
          arg_names=('data', 'residual', 'gamma', 'beta'),
          infer_params=lambda s, a: _adln_infer(s),
          params={'p': ('float', 0.0), 'eps': ('float', 1e-5), 'fuse_residual_grad': ('bool', False)})
def add_dropout_layernorm(data, residual, gamma, beta, p=0.0, eps=1e-5, fuse_residual_grad=False):
    """LayerNorm(residual + Dropout(data, p)) over the last axis -- the post-LN transformer sub-layer
    tail as one fused operator (the reference composes Dropout, elemwise_add and LayerNorm:
    src/operator/nn/dropout-inl.h, layer_norm-inl.h); dropout is active in training mode only.
    ``fuse_residual_grad``: ``data`` is computed from ``residual`` through a FullyConnected (a
    transformer sub-layer), so that layer's data-gradient GEMM adds the residual gradient (GPU)."""
    active = _state.STATE.training and p > 0
    return hip_ops.add_dropout_layer_norm(residual, data, gamma, beta, eps, p if active else 0.0,
                                          fuse_residual_grad)


@register('GroupNorm', arg_names=('data', 'gamma', 'beta'), num_outputs=3, num_visible_outputs=_ln_nvis,
          infer_params=lambda s, a: {1: (a.get('num_groups', 1),), 2: (a.get('num_groups', 1),)},
          params={'num_groups': ('int', 1), 'eps': ('float', 1e-5), 'output_mean_var': ('bool', False)})
def group_norm(data, gamma, beta, num_groups=1, eps=1e-5, output_mean_var=False):
    n = data.shape[0]
    x = _acc(data.reshape(n, num_groups, -1))
    mean = x.mean(-1, keepdim=True)
    var = x.var(-1, keepdim=True, unbiased=False)
    std = torch.sqrt(var + eps)
    y = ((x - mean) / std).reshape(data.shape)
    gshape = (1, num_groups, -1)
    y = (y.reshape(n, num_groups, -1) * _acc(gamma.reshape(gshape)) + _acc(beta.reshape(gshape))).reshape(data.shape)
    return y.to(data.dtype), mean.reshape(n, num_groups).to(data.dtype), std.reshape(n, num_groups).to(data.dtype)


@register('InstanceNorm', arg_names=('data', 'gamma', 'beta'),
          infer_params=lambda s, a: ({1: (s[0][1],), 2: (s[0][1],)} if s[0] is not None else {}),
          params={'eps': ('float', 1e-3)})
def instance_norm(data, gamma, beta, eps=1e-3):
    x = _acc(data)
    dims = list(range(2, data.dim()))
    mean = x.mean(dims, keepdim=True)
    var = x.var(dims, keepdim=True, unbiased=False)
    shape = (1, -1) + (1,) * (data.dim() - 2)
    y = (x - mean) / torch.sqrt(var + eps) * _acc(gamma.reshape(shape)) + _acc(beta.reshape(shape))
    return y.to(data.dtype)


@register('L2Normalization', params={'eps': ('float', 1e-10), 'mode': ('str', 'instance')})
def l2_normalization(data, eps=1e-10, mode='instance'):
    if mode == 'instance':
        n = torch.sqrt((data.reshape(data.shape[0], -1) ** 2).sum(1) + eps)
        return data / n.reshape((-1,) + (1,) * (data.dim() - 1))
    if mode == 'channel':
        n = torch.sqrt((data ** 2).sum(1, keepdim=True) + eps)
        return data / n
    n = torch.sqrt((data.reshape(data.shape[0], data.shape[1], -1) ** 2).sum(-1) + eps)
    return data / n.reshape(data.shape[:2] + (1,) * (data.dim() - 2))


@register('LRN', num_outputs=2, num_visible_outputs=1, output_names=('output', 'tmp_norm'),
          params={'alpha': ('float', 1e-4), 'beta': ('float', 0.75), 'knorm': ('float', 2.0), 'nsize': ('int', 5)})
def lrn(data, alpha=1e-4, beta=0.75, knorm=2.0, nsize=5):
    sq = (data * data).unsqueeze(1)
    pad = nsize // 2
    sq = F.pad(sq, (0, 0, 0, 0, pad, pad))
    s = F.avg_pool3d(sq, (nsize, 1, 1), stride=1).squeeze(1) * nsize
    norm = (knorm + alpha / nsize * s)
    return data * norm.pow(-beta), norm


@register('moments', num_outputs=2, params={'axes': ('shape?', None), 'keepdims': ('bool', False)})
def moments(data, axes=None, keepdims=False):
    dims = list(axes) if axes else list(range(data.dim()))
    m = data.mean(dims, keepdim=keepdims)
    v = ((data - data.mean(dims, keepdim=True)) ** 2).mean(dims, keepdim=keepdims)
    return m, v


# ---------------------------------------------------------------------------
# UpSampling / spatial
# ---------------------------------------------------------------------------

def _upsampling_args(a):
    if a.get('sample_type', 'nearest') == 'bilinear':
        return ['data', 'weight']
    return ['arg%d' % i for i in range(int(a.get('num_args', 1)))]


def _upsampling_infer(in_shapes, a):
    """Bilinear mode: the depthwise deconvolution weight is (channels, 1, k, k), k = 2s - s%2
    (reference src/operator/nn/upsampling-inl.h InferShape)."""
    if a.get('sample_type', 'nearest') != 'bilinear' or not in_shapes or in_shapes[0] is None:
        return {}
    s = int(a.get('scale', 1))
    k = 2 * s - s % 2
    return {1: (in_shapes[0][1], 1, k, k)}


@register('UpSampling', arg_names=_upsampling_args, infer_params=_upsampling_infer,
          key_var_num_args='num_args',
          params={'scale': ('int', 1), 'num_filter': ('int', 0), 'sample_type': ('str', 'nearest'),
                  'multi_input_mode': ('str', 'concat'), 'num_args': ('int', 1), 'workspace': ('int', 512)})
def upsampling(*data, scale=1, num_filter=0, sample_type='nearest', multi_input_mode='concat',
               num_args=1, workspace=512):
    if sample_type == 'nearest':
        outs = []
        h = data[0].shape[2] * scale
        for d in data:
            s = h // d.shape[2]
            outs.append(F.interpolate(d, scale_factor=s, mode='nearest'))
        if multi_input_mode == 'sum':
            r = outs[0]
            for o in outs[1:]:
                r = r + o
            return r
        return torch.cat(outs, dim=1)
    # bilinear: data[1] is the deconvolution weight (MXNet uses a fixed bilinear deconv)
    x, w = data[0], data[1]
    k = 2 * scale - scale % 2
    p = int(math.ceil((scale - 1) / 2.0))
    return F.conv_transpose2d(x, w, stride=scale, padding=p, groups=x.shape[1])


@register('ROIPooling', arg_names=('data', 'rois'),
          params={'pooled_size': ('shape', ()), 'spatial_scale': ('float', 1.0)})
def roi_pooling(data, rois, pooled_size=(), spatial_scale=1.0):
    ph, pw = pooled_size
    out = []
    for r in rois:
        b = int(r[0])
        x1, y1, x2, y2 = [int(round(float(v) * spatial_scale)) for v in r[1:]]
        h = max(y2 - y1 + 1, 1)
        w = max(x2 - x1 + 1, 1)
        fm = data[b]
        res = torch.full((data.shape[1], ph, pw), 0.0, dtype=data.dtype, device=data.device)
        for i in range(ph):
            hs = min(max(y1 + int(math.floor(i * h / ph)), 0), data.shape[2])
            he = min(max(y1 + int(math.ceil((i + 1) * h / ph)), 0), data.shape[2])
            for j in range(pw):
                ws = min(max(x1 + int(math.floor(j * w / pw)), 0), data.shape[3])
                we = min(max(x1 + int(math.ceil((j + 1) * w / pw)), 0), data.shape[3])
                if he > hs and we > ws:
                    res[:, i, j] = fm[:, hs:he, ws:we].amax(dim=(1, 2))
        out.append(res)
    return torch.stack(out)


# ---------------------------------------------------------------------------
# Sequence ops
# ---------------------------------------------------------------------------

def _seq_args(a):
    u = a.get('use_sequence_length', False)
    u = u if isinstance(u, bool) else str(u) in ('True', 'true', '1')
    return ['data', 'sequence_length'] if u else ['data']


_SEQ_PARAMS = {'use_sequence_length': ('bool', False), 'axis': ('int', 0)}


@register('SequenceMask', arg_names=_seq_args, params=dict(_SEQ_PARAMS, value=('float', 0.0)))
def sequence_mask(data, sequence_length=None, use_sequence_length=False, value=0.0, axis=0):
    if not use_sequence_length or sequence_length is None:
        return data.clone()
    t = data.shape[axis]
    ar = torch.arange(t, device=data.device)
    if axis == 0:
        m = ar.reshape(t, 1) < sequence_length.reshape(1, -1).to(ar.dtype)
    else:
        m = ar.reshape(1, t) < sequence_length.reshape(-1, 1).to(ar.dtype)
    m = m.reshape(m.shape + (1,) * (data.dim() - 2))
    return torch.where(m, data, torch.full_like(data, value))


@register('SequenceLast', arg_names=_seq_args, params=_SEQ_PARAMS)
def sequence_last(data, sequence_length=None, use_sequence_length=False, axis=0):
    if not use_sequence_length or sequence_length is None:
        return data.select(axis, data.shape[axis] - 1).contiguous()
    idx = (sequence_length.to(torch.int64) - 1)
    x = data if axis == 0 else data.transpose(0, 1)
    return x[idx, torch.arange(x.shape[1], device=data.device)]


@register('SequenceReverse', arg_names=_seq_args, params=_SEQ_PARAMS)
def sequence_reverse(data, sequence_length=None, use_sequence_length=False, axis=0):
    if not use_sequence_length or sequence_length is None:
        return torch.flip(data, dims=[0])
    out = data.clone()
    for b in range(data.shape[1]):
        n = int(sequence_length[b])
        out[:n, b] = torch.flip(data[:n, b], dims=[0])
    return out


# ---------------------------------------------------------------------------
# CTC loss
# ---------------------------------------------------------------------------

def _ctc_args(a):
    names = ['data', 'label']
    if str(a.get('use_data_lengths', False)) in ('True', 'true', '1'):
        names.append('data_lengths')
    if str(a.get('use_label_lengths', False)) in ('True', 'true', '1'):
        names.append('label_lengths')
    return names


@register('CTCLoss', aliases=('ctc_loss', '_contrib_CTCLoss', '_contrib_ctc_loss'), arg_names=_ctc_args,
          num_outputs=2, num_visible_outputs=1,
          params={'use_data_lengths': ('bool', False), 'use_label_lengths': ('bool', False),
                  'blank_label': ('str', 'first')})
def ctc_loss(data, label, *lengths, use_data_lengths=False, use_label_lengths=False, blank_label='first'):
    T, N, C = data.shape
    li = 0
    if use_data_lengths:
        dl = lengths[li].to(torch.int64); li += 1
    else:
        dl = torch.full((N,), T, dtype=torch.int64)
    lab = label.to(torch.int64)
    if blank_label == 'first':
        blank = 0
        pad_mask = lab > 0
    else:
        blank = C - 1
        pad_mask = (lab >= 0) & (lab != -1)
    if use_label_lengths:
        ll = lengths[li].to(torch.int64)
    else:
        ll = pad_mask.to(torch.int64).cumprod(1).sum(1)      # labels end at the first padding value
    # frames past a sequence's length never reach the loss or its gradient, whatever they hold
    valid = torch.arange(T, device=data.device)[:, None] < dl.to(data.device)[None, :]
    x = torch.where(valid[:, :, None], data.float(), torch.zeros((), device=data.device))
    logp = torch.log_softmax(x, dim=2)
    loss = F.ctc_loss(logp, lab.clamp(min=0), dl.cpu(), ll.cpu(), blank=blank, reduction='none',
                      zero_infinity=True)
    return loss.to(data.dtype), torch.zeros_like(data)


# ---------------------------------------------------------------------------
# Spatial transformer family
# ---------------------------------------------------------------------------

@register('GridGenerator', num_outputs=2, num_visible_outputs=1,
          params={'transform_type': ('str', 'affine'), 'target_shape': ('shape', (0, 0))})
def grid_generator(data, transform_type='affine', target_shape=(0, 0)):
    if transform_type == 'affine':
        n = data.shape[0]
        h, w = target_shape
        theta = data.reshape(n, 2, 3)
        ys = torch.linspace(-1, 1, h, device=data.device, dtype=data.dtype)
        xs = torch.linspace(-1, 1, w, device=data.device, dtype=data.dtype)
        gy, gx = torch.meshgrid(ys, xs, indexing='ij')
        grid = torch.stack([gx.reshape(-1), gy.reshape(-1), torch.ones_like(gx).reshape(-1)])
        out = torch.matmul(theta, grid).reshape(n, 2, h, w)
        return out, grid
    # warp: data is a flow field (N,2,H,W)
    n, _, h, w = data.shape
    ys = torch.arange(h, device=data.device, dtype=data.dtype)
    xs = torch.arange(w, device=data.device, dtype=data.dtype)
    gy, gx = torch.meshgrid(ys, xs, indexing='ij')
    x = (data[:, 0] + gx) / ((w - 1) / 2.0) - 1
    y = (data[:, 1] + gy) / ((h - 1) / 2.0) - 1
    return torch.stack([x, y], 1), data


@register('BilinearSampler', arg_names=('data', 'grid'), num_outputs=2, num_visible_outputs=1,
          params={'cudnn_off': ('bool?', None)})
def bilinear_sampler(data, grid, cudnn_off=None):
    g = grid.permute(0, 2, 3, 1)
    out = F.grid_sample(data, g, mode='bilinear', padding_mode='zeros', align_corners=True)
    return out, torch.zeros_like(grid)


@register('SpatialTransformer', arg_names=('data', 'loc'), num_outputs=3, num_visible_outputs=1,
          params={'target_shape': ('shape', (0, 0)), 'transform_type': ('str', 'affine'),
                  'sampler_type': ('str', 'bilinear'), 'cudnn_off': ('bool?', None)})
def spatial_transformer(data, loc, target_shape=(0, 0), transform_type='affine', sampler_type='bilinear',
                        cudnn_off=None):
    grid, _ = grid_generator(loc, 'affine', target_shape)
    out, _ = bilinear_sampler(data, grid)
    return out, grid, grid


class _AbsGeZero(torch.autograd.Function):
    """|d| with d/dd = +1 at d == 0 (the reference correlation's sign convention)."""
    @staticmethod
    def forward(ctx, d):
        ctx.save_for_backward(d)
        return d.abs()

    @staticmethod
    def backward(ctx, g):
        d, = ctx.saved_tensors
        return torch.where(d >= 0, g, -g)


@register('Correlation', arg_names=('data1', 'data2'), num_outputs=3, num_visible_outputs=1,
          params={'kernel_size': ('int', 1), 'max_displacement': ('int', 1), 'stride1': ('int', 1),
                  'stride2': ('int', 1), 'pad_size': ('int', 0), 'is_multiply': ('bool', True)})
def correlation(data1, data2, kernel_size=1, max_displacement=1, stride1=1, stride2=1, pad_size=0,
                is_multiply=True):
    n, c, h, w = data1.shape
    if kernel_size <= 0 or kernel_size % 2 == 0 or kernel_size > min(h, w) + 2 * pad_size - 2 * max_displacement:
        raise MXNetError('Correlation: kernel_size %d must be odd and fit the %dx%d input (pad_size %d, '
                         'max_displacement %d)' % (kernel_size, h, w, pad_size, max_displacement))
    p1 = F.pad(data1, (pad_size,) * 4)
    p2 = F.pad(data2, (pad_size,) * 4)
    kr = (kernel_size - 1) // 2
    border = max_displacement + kr
    ph, pw = p1.shape[2], p1.shape[3]
    top_h = int(math.ceil((ph - border * 2) / float(stride1)))
    top_w = int(math.ceil((pw - border * 2) / float(stride1)))
    gr = max_displacement // stride2
    gw = gr * 2 + 1
    outs = []
    for dy in range(-gr, gr + 1):
        for dx in range(-gr, gr + 1):
            s2y, s2x = dy * stride2, dx * stride2
            ys = torch.arange(top_h, device=data1.device) * stride1 + border
            xs = torch.arange(top_w, device=data1.device) * stride1 + border
            acc = 0
            for ky in range(-kr, kr + 1):
                for kx in range(-kr, kr + 1):
                    a = p1[:, :, (ys + ky)][:, :, :, (xs + kx)]
                    b = p2[:, :, (ys + ky + s2y)][:, :, :, (xs + kx + s2x)]
                    acc = acc + (a * b if is_multiply else _AbsGeZero.apply(a - b))
            outs.append(acc.sum(1) / (kernel_size * kernel_size * c))
    out = torch.stack(outs, 1)
    return out, p1, p2


@register('Crop', arg_names=lambda a: ['arg%d' % i for i in range(int(a.get('num_args', 1)))],
          key_var_num_args='num_args',
          params={'num_args': ('int', 1), 'offset': ('shape', (0, 0)), 'h_w': ('shape', (0, 0)),
                  'center_crop': ('bool', False)})
def crop_legacy(*data, num_args=1, offset=(0, 0), h_w=(0, 0), center_crop=False):
    x = data[0]
    if len(data) > 1:
        h, w = data[1].shape[2], data[1].shape[3]
    else:
        h, w = h_w
    if center_crop:
        oy, ox = (x.shape[2] - h) // 2, (x.shape[3] - w) // 2
    else:
        oy, ox = offset
    return x[:, :, oy:oy + h, ox:ox + w].contiguous()


@register('IdentityAttachKLSparseReg', params={'sparseness_target': ('float', 0.1), 'penalty': ('float', 0.001),
                                               'momentum': ('float', 0.9)})
def identity_attach_kl(data, sparseness_target=0.1, penalty=0.001, momentum=0.9):
    return data.clone()


# ---------------------------------------------------------------------------
# Fused RNN (cuDNN-style flat parameter vector; src/operator/rnn-inl.h)
# ---------------------------------------------------------------------------

def _rnn_args(a):
    names = ['data', 'parameters', 'state']
    if a.get('mode') == 'lstm':
        names.append('state_cell')
    if str(a.get('use_sequence_length', False)) in ('True', 'true', '1'):
        names.append('sequence_length')
    return names


_GATES = {'rnn_relu': 1, 'rnn_tanh': 1, 'lstm': 4, 'gru': 3}


def rnn_param_size(mode, num_layers, input_size, state_size, bidirectional, projection_size=None):
    g = _GATES[mode]
    d = 2 if bidirectional else 1
    hp = projection_size or state_size
    size = 0
    for layer in range(num_layers):
        ni = input_size if layer == 0 else hp * d
        size += d * (g * state_size * ni + g * state_size * hp + 2 * g * state_size)
        if projection_size:
            size += d * projection_size * state_size
    return size


def _rnn_nout(a):
    so = str(a.get('state_outputs', False)) in ('True', 'true', '1')
    if not so:
        return 1
    return 3 if a.get('mode') == 'lstm' else 2


def _rnn_infer(in_shapes, a):
    d = in_shapes[0]
    if d is None:
        return {}
    bi = str(a.get('bidirectional', False)) in ('True', 'true', '1')
    nl = int(a.get('num_layers', 1))
    ss = int(a['state_size'])
    ps = a.get('projection_size')
    ps = int(ps) if ps not in (None, 'None', '') else None
    res = {1: (rnn_param_size(a['mode'], nl, d[2], ss, bi, ps),), 2: (nl * (2 if bi else 1), d[1], ps or ss)}
    if a.get('mode') == 'lstm':
        res[3] = (nl * (2 if bi else 1), d[1], ss)
    return res


def unpack_rnn_params(params, mode, num_layers, input_size, state_size, bidirectional, projection_size=None):
    """Split MXNet's flat vector into per-(layer, direction) [w_ih, w_hh, b_ih, b_hh(, w_hr)].

    Layout (src/operator/rnn-inl.h): all weights first — for every layer and
    direction ``i2h``, ``h2h`` (and ``h2r`` with projection) — then all biases
    ``i2h``, ``h2h`` in the same order.
    """
    g = _GATES[mode]
    d = 2 if bidirectional else 1
    hp = projection_size or state_size
    ws = []
    off = 0
    for layer in range(num_layers):
        ni = input_size if layer == 0 else hp * d
        for _ in range(d):
            wi = params[off:off + g * state_size * ni].reshape(g * state_size, ni)
            off += g * state_size * ni
            wh = params[off:off + g * state_size * hp].reshape(g * state_size, hp)
            off += g * state_size * hp
            entry = [wi, wh]
            if projection_size:
                wr = params[off:off + projection_size * state_size].reshape(projection_size, state_size)
                off += projection_size * state_size
                entry.append(wr)
            ws.append(entry)
    k = 0
    for layer in range(num_layers):
        for _ in range(d):
            bi = params[off:off + g * state_size]
            off += g * state_size
            bh = params[off:off + g * state_size]
            off += g * state_size
            wr = ws[k][2:] if projection_size else []
            ws[k] = ws[k][:2] + [bi, bh] + wr
            k += 1
    if off != params.numel():
        # a wrong-size vector would hand empty / truncated views to the fused kernels (which crash)
        raise ValueError('RNN: parameter vector has %d elements, the layer needs %d' % (params.numel(), off))
    return ws


def _kernels_required():
    """MXAMD_REQUIRE_HIP=1: GPU ops must run on the in-tree kernels (no silent vendor fallback)."""
    import os
    return os.environ.get('MXAMD_REQUIRE_HIP', '0') == '1'


def _cell_step(mode, x, h, c, wi, wh, bi, bh, wr, clip):
    gi = F.linear(x, wi, bi)
    gh = F.linear(h, wh, bh)
    if mode == 'lstm':
        i, f, g, o = (gi + gh).chunk(4, -1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(g)
        if clip is not None:
            lo, hi, nan = clip
            c = c.clamp(lo if lo is not None else -float('inf'), hi if hi is not None else float('inf'))
            if nan:
                c = torch.nan_to_num(c, nan=0.0)
        h = torch.sigmoid(o) * torch.tanh(c)
        if wr is not None:
            h = F.linear(h, wr)
        return h, c
    if mode == 'gru':
        ir, iz, in_ = gi.chunk(3, -1)
        hr, hz, hn = gh.chunk(3, -1)
        r = torch.sigmoid(ir + hr)
        z = torch.sigmoid(iz + hz)
        n = torch.tanh(in_ + r * hn)
        return (1 - z) * n + z * h, None
    act = torch.tanh if mode == 'rnn_tanh' else torch.relu
    return act(gi + gh), None


def _rnn_loop(data, ws, h0, c0, mode, num_layers, d, p, train, clip, seq_len):
    """Explicit time loop for the features the fused path lacks (clipping, variable lengths, LSTMP)."""
    T = data.shape[0]
    x = data
    hs, cs = [], []
    lens = seq_len.long() if seq_len is not None else None
    for layer in range(num_layers):
        outs = []
        for di in range(d):
            k = layer * d + di
            w = ws[k]
            wr = w[4] if len(w) > 4 else None
            h = h0[k]
            c = c0[k] if c0 is not None else None
            ys = [None] * T
            steps = range(T - 1, -1, -1) if di == 1 else range(T)
            for t in steps:
                if lens is not None and di == 1:
                    valid = (t < lens).to(x.dtype).unsqueeze(-1)
                else:
                    valid = None
                nh, nc = _cell_step(mode, x[t], h, c, w[0], w[1], w[2], w[3], wr, clip)
                if lens is not None:
                    m = (t < lens).to(x.dtype).unsqueeze(-1) if valid is None else valid
                    h = m * nh + (1 - m) * h
                    if c is not None:
                        c = m * nc + (1 - m) * c
                    ys[t] = nh * m
                else:
                    h, c = nh, nc
                    ys[t] = nh
            outs.append(torch.stack(ys))
            hs.append(h)
            if c is not None:
                cs.append(c)
        x = torch.cat(outs, -1) if d == 2 else outs[0]
        if p > 0 and train and layer < num_layers - 1:
            x = F.dropout(x, p, True)
    return x, torch.stack(hs), (torch.stack(cs) if cs else None)


@register('RNN', arg_names=_rnn_args, num_outputs=_rnn_nout, infer_params=_rnn_infer,
          params={'state_size': ('int', 0), 'num_layers': ('int', 1), 'bidirectional': ('bool', False),
                  'mode': ('str', 'lstm'), 'p': ('float', 0.0), 'state_outputs': ('bool', False),
                  'projection_size': ('int?', None), 'lstm_state_clip_min': ('float?', None),
                  'lstm_state_clip_max': ('float?', None), 'lstm_state_clip_nan': ('bool', False),
                  'use_sequence_length': ('bool', False)})
def rnn(data, parameters, state, state_cell=None, sequence_length=None, state_size=0, num_layers=1,
        bidirectional=False, mode='lstm', p=0.0, state_outputs=False, projection_size=None,
        lstm_state_clip_min=None, lstm_state_clip_max=None, lstm_state_clip_nan=False,
        use_sequence_length=False):
    """Fused multi-layer RNN (src/operator/rnn.cc); TNC layout, MXNet flat parameter vector."""
    ws = unpack_rnn_params(parameters, mode, num_layers, data.shape[2], state_size, bidirectional,
                           projection_size)
    train = _state.STATE.training
    d = 2 if bidirectional else 1
    clip = None
    if mode == 'lstm' and (lstm_state_clip_min is not None or lstm_state_clip_max is not None):
        clip = (lstm_state_clip_min, lstm_state_clip_max, lstm_state_clip_nan)
    if clip is not None or (use_sequence_length and sequence_length is not None):
        out, h, c = _rnn_loop(data, ws, state, state_cell, mode, num_layers, d, p, train, clip,
                              sequence_length if use_sequence_length else None)
        if mode == 'lstm':
            return (out, h, c) if state_outputs else out
        return (out, h) if state_outputs else out
    flat = [t for group in ws for t in group]
    if any(int(x) == 0 for x in tuple(data.shape) + tuple(state.shape)):
        # the fused torch kernels crash on empty inputs (e.g. a shape probe with an unknown dim)
        raise MXNetError('RNN: empty input %s / state %s' % (tuple(data.shape), tuple(state.shape)))
    hsz = projection_size or state_size
    want = (num_layers * d, data.shape[1], hsz)
    if tuple(state.shape) != want or (mode == 'lstm' and state_cell is not None
                                      and tuple(state_cell.shape) != (num_layers * d, data.shape[1], state_size)):
        # the fused torch kernels do not validate state shapes
        raise MXNetError('RNN: state shape %s does not match %s' % (tuple(state.shape), want))
    from . import rnn_fns
    if rnn_fns.available(data) and not projection_size and os.environ.get('MXAMD_RNN_VENDOR', '0') != '1':
        # in-tree gfx950 recurrent kernels (src/kernels/rnn.hip): fused gate GEMM + cell per step
        out, h, c = rnn_fns.fused_rnn(data, ws, state, state_cell, mode, num_layers, bidirectional, p, train)
        if mode == 'lstm':
            return (out, h, c) if state_outputs else out
        return (out, h) if state_outputs else out
    if data.is_cuda and _kernels_required():
        raise MXNetError('RNN: the in-tree recurrent kernels are not available on this GPU build')
    if mode == 'lstm':
        out, h, c = torch._VF.lstm(data, (state, state_cell), flat, True, num_layers, p, train,
                                   bidirectional, False)
        return (out, h, c) if state_outputs else out
    if mode == 'gru':
        out, h = torch._VF.gru(data, state, flat, True, num_layers, p, train, bidirectional, False)
    elif mode == 'rnn_tanh':
        out, h = torch._VF.rnn_tanh(data, state, flat, True, num_layers, p, train, bidirectional, False)
    else:
        out, h = torch._VF.rnn_relu(data, state, flat, True, num_layers, p, train, bidirectional, False)
    return (out, h) if state_outputs else out
