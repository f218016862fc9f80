"""INT8 quantization operators (parity: src/operator/quantization/*).

Scheme (same as the reference): int8 is symmetric, ``q = round(x * 127 /
max(|min|, |max|))``; uint8 is affine over [min, max].  Quantized conv / FC
take int8 data + int8 weight and produce int32 with an output range such that
``float = int32 * range / (2**31 - 1)`` — i.e. the product of the input
scales — which ``requantize`` maps back to int8 with calibrated ranges.

The int32 products are computed exactly (integer values are exactly
representable in fp32 GEMM accumulations up to 2**24 per partial sum; the
reduction is done in fp64 for larger K), so results match an integer GEMM.
"""
import numpy as np
import torch
import torch.nn.functional as F

from .registry import register
from ..base import MXNetError

INT8_MAX = 127.0
UINT8_MAX = 255.0
INT32_MAX = float(2 ** 31 - 1)


def _range_scalar(t):
    return t.reshape(-1)[0].float()


def _quantize_int8(x, mn, mx):
    real = torch.maximum(mn.abs(), mx.abs())
    scale = INT8_MAX / torch.clamp(real, min=1e-30)
    q = torch.clamp(torch.round(x.float() * scale), -INT8_MAX, INT8_MAX).to(torch.int8)
    return q, -real.reshape(1), real.reshape(1)


def _quantize_uint8(x, mn, mx):
    scale = UINT8_MAX / torch.clamp(mx - mn, min=1e-30)
    q = torch.clamp(torch.round((x.float() - mn) * scale), 0, UINT8_MAX).to(torch.uint8)
    return q, mn.reshape(1), mx.reshape(1)


@register('_contrib_quantize', aliases=('quantize',), arg_names=('data', 'min_range', 'max_range'), num_outputs=3,
          params={'out_type': ('str', 'uint8')})
def quantize(data, min_range, max_range, out_type='uint8'):
    mn, mx = _range_scalar(min_range), _range_scalar(max_range)
    return _quantize_int8(data, mn, mx) if out_type == 'int8' else _quantize_uint8(data, mn, mx)


@register('_contrib_quantize_v2', aliases=('quantize_v2',), num_outputs=3,
          params={'out_type': ('str', 'int8'), 'min_calib_range': ('float?', None),
                  'max_calib_range': ('float?', None)})
def quantize_v2(data, out_type='int8', min_calib_range=None, max_calib_range=None):
    if min_calib_range is not None and max_calib_range is not None:
        mn = torch.tensor(min_calib_range, device=data.device)
        mx = torch.tensor(max_calib_range, device=data.device)
    else:
        mn, mx = data.float().min(), data.float().max()
    if out_type == 'auto':
        out_type = 'uint8' if float(mn) >= 0 else 'int8'
    return _quantize_int8(data, mn, mx) if out_type == 'int8' else _quantize_uint8(data, mn, mx)


@register('_contrib_dequantize', aliases=('dequantize',), arg_names=('data', 'min_range', 'max_range'),
          params={'out_type': ('str', 'float32')})
def dequantize(data, min_range, max_range, out_type='float32'):
    mn, mx = _range_scalar(min_range), _range_scalar(max_range)
    if data.dtype == torch.uint8:
        return data.float() * ((mx - mn) / UINT8_MAX) + mn
    if data.dtype == torch.int8:
        return data.float() * (torch.maximum(mn.abs(), mx.abs()) / INT8_MAX)
    # int32
    return data.double().mul(torch.maximum(mn.abs(), mx.abs()).double() / INT32_MAX).float()


@register('_contrib_requantize', aliases=('requantize',), arg_names=('data', 'min_range', 'max_range'),
          num_outputs=3, params={'out_type': ('str', 'int8'), 'min_calib_range': ('float?', None),
                                 'max_calib_range': ('float?', None)})
def requantize(data, min_range, max_range, out_type='int8', min_calib_range=None, max_calib_range=None):
    real = dequantize(data, min_range, max_range)
    if min_calib_range is not None and max_calib_range is not None:
        mn = torch.tensor(min_calib_range, device=data.device)
        mx = torch.tensor(max_calib_range, device=data.device)
    else:
        mn, mx = real.min(), real.max()
    return _quantize_int8(real, mn, mx)


def _int_range(mn_d, mx_d, mn_w, mx_w):
    # float = int32 * (rd/127) * (rw/127)  ->  range = that scale * INT32_MAX
    rd = torch.maximum(mn_d.abs(), mx_d.abs())
    rw = torch.maximum(mn_w.abs(), mx_w.abs())
    r = rd * rw / (INT8_MAX * INT8_MAX) * INT32_MAX
    return -r.reshape(1), r.reshape(1)


def _exact_int(fn, *args):
    # integer-valued operands: fp64 keeps every partial sum exact
    return torch.round(fn(*[a.double() for a in args])).to(torch.int32)


def _hip_int8():
    from . import kernels as K
    return K.lib() if (K.available() and K.enabled()) else None


def _int8_matmul(x, w):
    """int32 ``x @ w.T`` for integer-valued x [M, K] (int8 or uint8) and w [N, K] (int8).

    On a GPU: the gfx950 i8 MFMA GEMM (src/kernels/int8_gemm.hip) -- uint8 data is
    re-centred to int8 (x - 128) and the 128 * sum_k w[n, k] term added back; K is
    zero-padded to a multiple of 64.  Elsewhere: exact fp64 matmul.
    """
    lib = _hip_int8() if x.is_cuda else None
    if lib is None or w.dtype != torch.int8 or x.dtype not in (torch.int8, torch.uint8):
        return _exact_int(lambda a, b: a @ b.t(), x, w)
    M, K = x.shape
    N = w.shape[0]
    shift = x.dtype == torch.uint8
    xa = (x.to(torch.int16) - 128).to(torch.int8) if shift else x
    pad = (-K) % 64
    if pad:
        xa = torch.nn.functional.pad(xa, (0, pad))
        w = torch.nn.functional.pad(w, (0, pad))
    xa = xa.contiguous()
    w = w.contiguous()
    out = torch.empty((M, N), dtype=torch.int32, device=x.device)
    lib.int8_gemm(xa.data_ptr(), w.data_ptr(), out.data_ptr(), M, N, K + pad,
                  torch.cuda.current_stream(x.device).cuda_stream)
    if shift:
        out += 128 * w.to(torch.int32).sum(1).reshape(1, -1)
    return out


def _im2col_nhwc(x, kernel, stride, pad, dilate):
    """[N, H, W, C] -> ([N*Ho*Wo, kh*kw*C], (N, Ho, Wo)) with the (kh, kw, C) order of an NHWC weight."""
    n, h, w_, c = x.shape
    kh, kw = kernel
    sh, sw = stride
    ph, pw = pad
    dh, dw = dilate
    xp = torch.nn.functional.pad(x, (0, 0, pw, pw, ph, ph))
    ho = (h + 2 * ph - dh * (kh - 1) - 1) // sh + 1
    wo = (w_ + 2 * pw - dw * (kw - 1) - 1) // sw + 1
    cols = []
    for i in range(kh):
        for j in range(kw):
            cols.append(xp[:, i * dh:i * dh + sh * (ho - 1) + 1:sh, j * dw:j * dw + sw * (wo - 1) + 1:sw, :])
    return torch.cat(cols, dim=-1).reshape(n * ho * wo, kh * kw * c), (n, ho, wo)


def _qconv_args(a):
    names = ['data', 'weight']
    if not (str(a.get('no_bias', False)) in ('True', 'true', '1')):
        names.append('bias')
    names += ['min_data', 'max_data', 'min_weight', 'max_weight']
    if 'bias' in names:
        names += ['min_bias', 'max_bias']
    return names


@register('_contrib_quantized_conv', arg_names=_qconv_args, num_outputs=3,
          params={'kernel': ('shape', ()), 'stride': ('shape', ()), 'dilate': ('shape', ()), 'pad': ('shape', ()),
                  'num_filter': ('int', 1), 'num_group': ('int', 1), 'no_bias': ('bool', False),
                  'layout': ('str?', None), 'workspace': ('int', 1024), 'cudnn_tune': ('str?', None),
                  'cudnn_off': ('bool', False)})
def quantized_conv(data, weight, *rest, kernel=(), stride=(), dilate=(), pad=(), num_filter=1, num_group=1,
                   no_bias=False, layout=None, workspace=1024, cudnn_tune=None, cudnn_off=False):
    if no_bias:
        bias = None
        mn_d, mx_d, mn_w, mx_w = rest[:4]
    else:
        bias = rest[0]
        mn_d, mx_d, mn_w, mx_w, mn_b, mx_b = rest[1:7]
    nsp = data.dim() - 2
    stride = tuple(stride) or (1,) * nsp
    dilate = tuple(dilate) or (1,) * nsp
    pad = tuple(pad) or (0,) * nsp
    channel_last = layout in ('NHWC', 'NWC', 'NDHWC')
    x, w = data, weight
    if channel_last:
        x = x.permute(0, nsp + 1, *range(1, nsp + 1))
        w = w.permute(0, nsp + 1, *range(1, nsp + 1))
    if data.is_cuda and nsp == 2 and num_group == 1 and weight.dtype == torch.int8 and _hip_int8() is not None:
        # implicit GEMM on the i8 matrix cores: NHWC im2col view x NHWC weight
        xn = data if channel_last else data.permute(0, 2, 3, 1)
        wn = weight if channel_last else weight.permute(0, 2, 3, 1)
        cols, (n_, ho, wo) = _im2col_nhwc(xn, tuple(wn.shape[1:3]), stride, pad, dilate)
        out = _int8_matmul(cols, wn.reshape(wn.shape[0], -1)).reshape(n_, ho, wo, -1)
        out = out.permute(0, 3, 1, 2)        # NCHW view; the channel_last branch below permutes back
    else:
        conv = {1: F.conv1d, 2: F.conv2d, 3: F.conv3d}[nsp]
        out = _exact_int(lambda a, b: conv(a, b, None, stride, pad, dilate, num_group), x, w)
    omin, omax = _int_range(_range_scalar(mn_d), _range_scalar(mx_d), _range_scalar(mn_w), _range_scalar(mx_w))
    if bias is not None:
        # int8 bias rescaled into the int32 output scale
        rb = torch.maximum(_range_scalar(mn_b).abs(), _range_scalar(mx_b).abs()) / INT8_MAX
        b = torch.round(bias.double() * rb.double() * INT32_MAX / omax.double()).to(torch.int32)
        out = out + b.reshape((1, -1) + (1,) * nsp)
    if channel_last:
        out = out.permute(0, *range(2, nsp + 2), 1).contiguous()
    else:
        out = out.contiguous()
    return out, omin, omax


def _qfc_args(a):
    names = ['data', 'weight']
    nb = str(a.get('no_bias', False)) in ('True', 'true', '1')
    if not nb:
        names.append('bias')
    names += ['min_data', 'max_data', 'min_weight', 'max_weight']
    if not nb:
        names += ['min_bias', 'max_bias']
    return names


@register('_contrib_quantized_fully_connected', arg_names=_qfc_args, num_outputs=3,
          params={'num_hidden': ('int', 1), 'no_bias': ('bool', False), 'flatten': ('bool', True)})
def quantized_fully_connected(data, weight, *rest, num_hidden=1, no_bias=False, flatten=True):
    if no_bias:
        bias = None
        mn_d, mx_d, mn_w, mx_w = rest[:4]
    else:
        bias = rest[0]
        mn_d, mx_d, mn_w, mx_w, mn_b, mx_b = rest[1:7]
    x = data.reshape(data.shape[0], -1) if flatten else data
    lead = x.shape[:-1]
    out = _int8_matmul(x.reshape(-1, x.shape[-1]), weight).reshape(*lead, weight.shape[0])
    omin, omax = _int_range(_range_scalar(mn_d), _range_scalar(mx_d), _range_scalar(mn_w), _range_scalar(mx_w))
    if bias is not None:
        rb = torch.maximum(_range_scalar(mn_b).abs(), _range_scalar(mx_b).abs()) / INT8_MAX
        out = out + torch.round(bias.double() * rb.double() * INT32_MAX / omax.double()).to(torch.int32)
    return out, omin, omax


@register('_contrib_quantized_pooling', arg_names=('data', 'min_data', 'max_data'), num_outputs=3,
          params={'kernel': ('shape', ()), 'pool_type': ('str', 'max'), 'global_pool': ('bool', False),
                  'stride': ('shape', ()), 'pad': ('shape', ()), 'pooling_convention': ('str', 'valid'),
                  'layout': ('str?', None), 'cudnn_off': ('bool', False), 'count_include_pad': ('bool?', None),
                  'p_value': ('int?', None)})
def quantized_pooling(data, min_data, max_data, kernel=(), pool_type='max', global_pool=False, stride=(), pad=(),
                      pooling_convention='valid', layout=None, cudnn_off=False, count_include_pad=None,
                      p_value=None):
    from .nn import pooling
    y = pooling(data.float(), kernel=kernel, pool_type=pool_type, global_pool=global_pool, stride=stride, pad=pad,
                pooling_convention=pooling_convention, layout=layout, count_include_pad=count_include_pad)
    if pool_type == 'avg':
        y = torch.round(y)
    return y.to(data.dtype), min_data, max_data


@register('_contrib_quantized_act', arg_names=('data', 'min_data', 'max_data'), num_outputs=3,
          params={'act_type': ('str', 'relu')})
def quantized_act(data, min_data, max_data, act_type='relu'):
    if act_type != 'relu':
        raise ValueError('quantized_act supports relu only')
    return torch.clamp(data, min=0), min_data, max_data


@register('_contrib_quantized_flatten', arg_names=('data', 'min_data', 'max_data'), num_outputs=3)
def quantized_flatten(data, min_data, max_data):
    return data.reshape(data.shape[0], -1), min_data, max_data


@register('_contrib_quantized_elemwise_add', arg_names=('lhs', 'rhs', 'lhs_min', 'lhs_max', 'rhs_min', 'rhs_max'),
          num_outputs=3, params={'min_calib_range': ('float?', None), 'max_calib_range': ('float?', None)})
def quantized_elemwise_add(lhs, rhs, lhs_min, lhs_max, rhs_min, rhs_max, min_calib_range=None, max_calib_range=None):
    a = dequantize(lhs, lhs_min, lhs_max)
    b = dequantize(rhs, rhs_min, rhs_max)
    s = a + b
    if min_calib_range is not None:
        return _quantize_int8(s, torch.tensor(min_calib_range), torch.tensor(max_calib_range))
    r = torch.maximum(s.min().abs(), s.max().abs())
    return _quantize_int8(s, -r, r)


def _qconcat_args(a):
    n = int(a.get('num_args', 1))
    return ['arg%d' % i for i in range(n)] + ['min_arg%d' % i for i in range(n)] + ['max_arg%d' % i for i in range(n)]


@register('_contrib_quantized_concat', arg_names=_qconcat_args, num_outputs=3,
          params={'num_args': ('int', 1), 'dim': ('int', 1)}, key_var_num_args='num_args')
def quantized_concat(*args, num_args=1, dim=1):
    datas = args[:num_args]
    mins = args[num_args:2 * num_args]
    maxs = args[2 * num_args:3 * num_args]
    reals = [dequantize(d, mn, mx) for d, mn, mx in zip(datas, mins, maxs)]
    r = max(float(torch.maximum(_range_scalar(mn).abs(), _range_scalar(mx).abs())) for mn, mx in zip(mins, maxs))
    r = torch.tensor(r)
    return _quantize_int8(torch.cat(reals, dim=dim), -r, r)


# ---------------------------------------------------------------------------
# quantized BatchNorm / elemwise_mul / Embedding / RNN, asymmetric quantize
# ---------------------------------------------------------------------------

def _maxabs(mn, mx):
    return torch.maximum(_range_scalar(mn).abs(), _range_scalar(mx).abs())


def _bn_q_infer(in_shapes, a):
    d = in_shapes[0]
    if d is None:
        return {}
    c = d[a.get('axis', 1) % len(d)]
    return {1: (c,), 2: (c,), 3: (c,), 4: (c,), 5: (1,), 6: (1,)}


@register('_contrib_quantized_batch_norm',
          arg_names=('data', 'gamma', 'beta', 'moving_mean', 'moving_var', 'min_data', 'max_data'),
          num_outputs=3, infer_params=_bn_q_infer,
          params={'eps': ('float', 1e-3), 'momentum': ('float', 0.9), 'fix_gamma': ('bool', True),
                  'use_global_stats': ('bool', False), 'output_mean_var': ('bool', False), 'axis': ('int', 1),
                  'cudnn_off': ('bool', False), 'min_calib_range': ('float?', None),
                  'max_calib_range': ('float?', None)})
def quantized_batch_norm(data, gamma, beta, moving_mean, moving_var, min_data, max_data, eps=1e-3, momentum=0.9,
                         fix_gamma=True, use_global_stats=False, output_mean_var=False, axis=1, cudnn_off=False,
                         min_calib_range=None, max_calib_range=None):
    """Inference BatchNorm on int8/uint8 data (reference quantized_batch_norm.cc): the input scale and
    the moving statistics fold into one per-channel affine map, the result is requantized to int8 with
    the calibrated output range (or the observed one)."""
    real = dequantize(data, min_data, max_data)
    nd_ = real.dim()
    ax = axis % nd_
    shape = [1] * nd_
    shape[ax] = real.shape[ax]
    g = torch.ones_like(gamma.float()) if fix_gamma else gamma.float()
    inv = torch.rsqrt(moving_var.float() + eps)
    scale = (g * inv).reshape(shape)
    shift = (beta.float() - moving_mean.float() * g * inv).reshape(shape)
    y = real * scale + shift
    if min_calib_range is not None and max_calib_range is not None:
        r = torch.tensor(max(abs(min_calib_range), abs(max_calib_range)), device=y.device)
    else:
        r = torch.maximum(y.min().abs(), y.max().abs())
    return _quantize_int8(y, -r, r)


def _qmul_nout(a):
    return 1 if str(a.get('enable_float_output', False)) in ('True', 'true', '1') else 3


@register('_contrib_quantized_elemwise_mul',
          arg_names=('lhs', 'rhs', 'lhs_min', 'lhs_max', 'rhs_min', 'rhs_max'), num_outputs=_qmul_nout,
          params={'min_calib_range': ('float?', None), 'max_calib_range': ('float?', None),
                  'enable_float_output': ('bool', False)})
def quantized_elemwise_mul(lhs, rhs, lhs_min, lhs_max, rhs_min, rhs_max, min_calib_range=None,
                           max_calib_range=None, enable_float_output=False):
    """int8 x int8 elementwise product (reference quantized_elemwise_mul.cc).  Output: fp32 real values
    (enable_float_output), int8 in the calibrated range, or int32 carrying a*b*scale_l*scale_r with
    the int32 range of an s8 x s8 product."""
    sl = _maxabs(lhs_min, lhs_max) / INT8_MAX
    sr = _maxabs(rhs_min, rhs_max) / INT8_MAX
    prod = lhs.to(torch.int32).to(torch.float64) * rhs.to(torch.int32).to(torch.float64)
    if enable_float_output:
        return (prod * (sl * sr).double()).float()
    if min_calib_range is not None and max_calib_range is not None:
        r = max(abs(min_calib_range), abs(max_calib_range))
        out_scale = (INT8_MAX / r) * (sl * sr).double()
        q = torch.clamp(torch.trunc(prod * out_scale), -INT8_MAX, INT8_MAX).to(torch.int8)
        t = torch.tensor([r], dtype=torch.float32, device=lhs.device)
        return q, -t, t
    out = torch.trunc(prod * (sl * sr).double()).to(torch.int32)
    r = (sl * sr * INT32_MAX).reshape(1).float()
    return out, -r, r


@register('_contrib_quantized_embedding', arg_names=('data', 'weight', 'min_weight', 'max_weight'),
          num_outputs=3, infer_params=lambda s, a: {1: (a['input_dim'], a['output_dim']), 2: (1,), 3: (1,)},
          params={'input_dim': ('int', 0), 'output_dim': ('int', 0), 'dtype': ('str', 'float32'),
                  'sparse_grad': ('bool', False)})
def quantized_embedding(data, weight, min_weight, max_weight, input_dim=0, output_dim=0, dtype='float32',
                        sparse_grad=False):
    """Row gather of an int8 table (reference quantized_indexing_op.cc); the output keeps the
    weight's range.  Out-of-range indices are clipped, as Embedding does."""
    idx = torch.clamp(data.to(torch.int64), 0, weight.shape[0] - 1)
    return weight[idx], _range_scalar(min_weight).reshape(1), _range_scalar(max_weight).reshape(1)


def _qrnn_nout(a):
    so = str(a.get('state_outputs', False)) in ('True', 'true', '1')
    return 3 if so else 1


@register('_contrib_quantized_rnn',
          arg_names=('data', 'parameters', 'state', 'state_cell', 'min_data', 'max_data'),
          num_outputs=_qrnn_nout,
          params={'state_size': ('int', 0), 'num_layers': ('int', 1), 'bidirectional': ('bool', False),
                  'mode': ('str', 'lstm'), 'p': ('float', 0.0), 'state_outputs': ('bool', False),
                  'projection_size': ('int?', None), 'lstm_state_clip_min': ('float?', None),
                  'lstm_state_clip_max': ('float?', None), 'lstm_state_clip_nan': ('bool', False),
                  'use_sequence_length': ('bool', False)})
def quantized_rnn(data, parameters, state, state_cell, min_data, max_data, state_size=0, num_layers=1,
                  bidirectional=False, mode='lstm', p=0.0, state_outputs=False, projection_size=None,
                  lstm_state_clip_min=None, lstm_state_clip_max=None, lstm_state_clip_nan=False,
                  use_sequence_length=False):
    """LSTM on uint8 data (reference quantized_rnn.cc).  As in the reference, the last two inputs carry
    the asymmetric data scale and shift of quantize_asym: real = (q - shift) / scale.  The recurrence
    then runs in fp32 (at least as accurate as the reference's int8-weight GEMMs)."""
    if mode != 'lstm':
        raise ValueError('quantized_rnn supports mode=lstm only')
    from .nn import rnn
    scale = _range_scalar(min_data)
    shift = _range_scalar(max_data)
    real = (data.float() - shift) / scale
    return rnn(real, parameters.float(), state.float(), state_cell.float(), state_size=state_size,
               num_layers=num_layers, bidirectional=bidirectional, mode='lstm', p=0.0,
               state_outputs=state_outputs, projection_size=projection_size,
               lstm_state_clip_min=lstm_state_clip_min, lstm_state_clip_max=lstm_state_clip_max,
               lstm_state_clip_nan=lstm_state_clip_nan)


@register('_contrib_quantize_asym', aliases=('quantize_asym',), num_outputs=3,
          params={'min_calib_range': ('float?', None), 'max_calib_range': ('float?', None)})
def quantize_asym(data, min_calib_range=None, max_calib_range=None):
    """Asymmetric uint8 quantization (reference quantize_asym-inl.h): q = x * scale + shift + 0.5 with
    scale = 255 / (max - min), shift = 255 - max * scale; int8 input is re-centred (+128), uint8 passes.
    Outputs (q, scale, shift)."""
    dev = data.device
    if data.dtype == torch.uint8:
        return data.clone(), torch.ones(1, device=dev), torch.zeros(1, device=dev)
    if data.dtype == torch.int8:
        q = (data.to(torch.int16) + 128).to(torch.uint8)
        return q, torch.ones(1, device=dev), torch.full((1,), 128.0, device=dev)
    x = data.float()
    if min_calib_range is not None and max_calib_range is not None:
        mn = torch.tensor(float(min_calib_range), device=dev)
        mx = torch.tensor(float(max_calib_range), device=dev)
    else:
        mn, mx = x.min(), x.max()
    scale = UINT8_MAX / (mx - mn)
    shift = UINT8_MAX - mx * scale
    q = torch.clamp(torch.floor(x * scale + shift + 0.5), 0, UINT8_MAX).to(torch.uint8)
    return q, scale.reshape(1), shift.reshape(1)


# ---------------------------------------------------------------------------
# intgemm (reference src/operator/contrib/intgemm/*): int8 GEMM with -128 banned.
# The "prepared weight" format of this framework is the plain row-major int8 [rows, inner]
# matrix the gfx950 i8 MFMA kernel consumes (the reference's is CPU-layout dependent; its tests
# only check consistency between the prepare / take / multiply routes).
# ---------------------------------------------------------------------------

@register('_contrib_intgemm_maxabsolute', aliases=('_npx_intgemm_maxabsolute',))
def intgemm_maxabsolute(data):
    return data.float().abs().max().reshape(1)


def _intgemm_quant(x, maxabs):
    m = _range_scalar(maxabs)
    q = torch.round(x.float() * (INT8_MAX / m))
    return torch.clamp(q, -INT8_MAX, INT8_MAX).to(torch.int8)


@register('_contrib_intgemm_prepare_data', aliases=('_npx_intgemm_prepare_data',),
          arg_names=('data', 'maxabs'))
def intgemm_prepare_data(data, maxabs):
    """int8 quantisation with maxabs -> 127 and -128 banned (values clipped to [-127, 127])."""
    return _intgemm_quant(data, maxabs)


def _pw_args(a):
    return ['weight'] if str(a.get('already_quantized', False)) in ('True', 'true', '1') else ['weight', 'maxabs']


@register('_contrib_intgemm_prepare_weight', aliases=('_npx_intgemm_prepare_weight',), arg_names=_pw_args,
          params={'already_quantized': ('bool', False)})
def intgemm_prepare_weight(weight, maxabs=None, already_quantized=False):
    if already_quantized:
        if weight.dtype != torch.int8:
            raise ValueError('intgemm_prepare_weight: already_quantized weight must be int8')
        return torch.clamp(weight, -127, 127).contiguous()
    return _intgemm_quant(weight, maxabs).contiguous()


@register('_contrib_intgemm_take_weight', aliases=('_npx_intgemm_take_weight',), arg_names=('weight', 'indices'))
def intgemm_take_weight(weight, indices):
    return weight[indices.to(torch.int64)].contiguous()


def _ifc_args(a):
    names = ['data', 'weight']
    if str(a.get('out_type', 'float32')) == 'float32':
        names.append('scaling')
    if not (str(a.get('no_bias', False)) in ('True', 'true', '1')):
        names.append('bias')
    return names


@register('_contrib_intgemm_fully_connected', aliases=('_npx_intgemm_fully_connected',), arg_names=_ifc_args,
          params={'num_hidden': ('int', 1), 'no_bias': ('bool', False), 'flatten': ('bool', True),
                  'out_type': ('str', 'float32')})
def intgemm_fully_connected(data, weight, *rest, num_hidden=1, no_bias=False, flatten=True, out_type='float32'):
    """C = data . weight^T on int8 operands (the gfx950 i8 MFMA GEMM on a GPU).  fp32 data is quantised on
    the fly with its own max-abs (the scaling is divided by that scale); ``scaling`` multiplies the int32
    result before the (unscaled) bias is added; out_type int32 skips the scaling."""
    rest = list(rest)
    scaling = rest.pop(0) if out_type == 'float32' else None
    bias = None if no_bias else rest.pop(0)
    x = data.reshape(data.shape[0], -1) if flatten else data
    lead = x.shape[:-1]
    x2 = x.reshape(-1, x.shape[-1])
    mult = None
    if x2.dtype != torch.int8:
        m = x2.float().abs().max()
        x2 = _intgemm_quant(x2, m.reshape(1))
        mult = m / INT8_MAX
    acc = _int8_matmul(x2, weight.reshape(weight.shape[0], -1))
    if out_type == 'int32':
        out = acc
        if bias is not None:
            out = out + bias.to(torch.int32)
    else:
        s = _range_scalar(scaling)
        if mult is not None:
            s = s * mult
        out = acc.double() * s.double()
        if bias is not None:
            out = out + bias.double()
        out = out.float()
    return out.reshape(*lead, weight.shape[0])


def _smooth_or_none(p, eps=0.0001):
    """Move ``eps`` of mass onto every zero bin, taken evenly off the non-zero bins; None when the
    distribution is all zeros or the correction would exceed a whole unit."""
    zeros = p == 0
    nz = p.size - int(zeros.sum())
    if nz == 0:
        return None
    eps1 = eps * float(zeros.sum()) / float(nz)
    if eps1 >= 1.0:
        return None
    return p + np.where(zeros, eps, -eps1)


def calibrate_entropy_host(hist, edges, num_quantized_bins=255):
    """(threshold, divergence): the symmetric clipping threshold whose int8 re-quantisation Q of the
    clipped histogram P has the smallest KL(P || Q) -- every candidate width from num_quantized_bins/2
    to half the histogram, as the reference's calibrate.cc:CalibrateComputeCPU evaluates it (the sliced
    counts are integral there, the clipped outliers are folded into the end bins of P)."""
    hist = np.asarray(hist, dtype=np.float32).reshape(-1)
    edges = np.asarray(edges, dtype=np.float32).reshape(-1)
    nb = hist.size
    if edges.size != nb + 1:
        raise MXNetError('_contrib_calibrate_entropy: hist_edges must have len(hist) + 1 entries')
    zero = nb // 2
    half_q = num_quantized_bins // 2
    cum = np.concatenate([[0.0], np.cumsum(hist, dtype=np.float64)])
    best_div, best_th = np.float32(np.finfo(np.float32).max), None
    for i in range(half_q, zero + 1):
        lo, hi = zero - i, zero + i + 1
        sliced = np.floor(hist[lo:hi]).astype(np.float64)          # the reference's size_t counts
        p = hist[lo:hi].astype(np.float64).copy()
        p[0] = cum[lo + 1]                                         # bins 0..lo folded into the first
        p[-1] = cum[nb] - cum[hi]                                  # bins hi.. folded into the last
        merged = sliced.size // num_quantized_bins
        qb = np.array([sliced[j * merged:(j + 1) * merged].sum() for j in range(num_quantized_bins)])
        qb[-1] += sliced[num_quantized_bins * merged:].sum()
        q = np.zeros(sliced.size)
        for j in range(num_quantized_bins):
            s0 = j * merged
            s1 = sliced.size if j == num_quantized_bins - 1 else (j + 1) * merged
            norm = int(np.count_nonzero(sliced[s0:s1]))
            if norm:
                seg = p[s0:s1] != 0
                q[s0:s1][seg] = qb[j] / norm
        ps, qs = _smooth_or_none(p), _smooth_or_none(q)
        if qs is None or ps is None:
            div = np.float32(np.inf)
        else:
            ps = ps / ps.sum()
            qs = qs / qs.sum()
            div = np.float32(np.sum(ps * np.log(ps / qs)))
        if best_th is None or div < best_div:
            best_div, best_th = div, edges[hi]
    return float(best_th), float(best_div)


@register('_contrib_calibrate_entropy', arg_names=('hist', 'hist_edges'), num_outputs=2,
          params={'num_quantized_bins': ('int', 255)})
def calibrate_entropy(hist, hist_edges, num_quantized_bins=255):
    """Calibrated threshold and its KL divergence for a histogram (reference:
    src/operator/quantization/calibrate.cc:193); a host computation over the small histogram."""
    th, div = calibrate_entropy_host(hist.detach().float().cpu().numpy(), hist_edges.detach().float().cpu().numpy(),
                                     int(num_quantized_bins))
    dev = hist.device
    return (torch.tensor([th], dtype=torch.float32, device=dev), torch.tensor([div], dtype=torch.float32, device=dev))
