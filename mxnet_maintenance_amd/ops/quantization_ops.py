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
import torch
import torch.nn.functional as F

from .registry import register

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
