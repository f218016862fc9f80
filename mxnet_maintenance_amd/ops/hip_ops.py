"""Dispatch layer between operator definitions and the gfx950 HIP kernels.

Every hot operator (FullyConnected, Convolution, BatchNorm(+ReLU/+add),
Pooling, ReLU/GELU, LayerNorm, softmax-cross-entropy) goes through a function
here. On an MI355X with the native extension loaded, the hand-written HIP
kernels in ``src/kernels/*.hip`` run (wrapped as ``torch.autograd.Function``
so they compose with the autograd tape); on the CPU the torch reference path
runs. On a GPU box a missing extension is an error, not a silent fallback
(set ``MXAMD_ALLOW_TORCH_FALLBACK=1`` to override while debugging).

Parity targets: src/operator/nn/{fully_connected,convolution,batch_norm,
pooling,activation,layer_norm,softmax}*.cu and the cuDNN wrappers in
src/operator/nn/cudnn/*.
"""
import os

import torch
import torch.nn.functional as F

from ..base import MXNetError
from . import kernels as _K

_ALLOW_FALLBACK = os.environ.get('MXAMD_ALLOW_TORCH_FALLBACK', '0') == '1'


def _acc(t):
    """Accumulation dtype: fp32 for fp16/bf16/fp32 inputs, fp64 stays fp64 (reference CPU semantics)."""
    return t if t.dtype == torch.float64 else t.float()


def _use_hip(t):
    """True when ``t`` lives on the GPU and the HIP kernels should run."""
    if not t.is_cuda:
        return False
    if _K.available():
        return _K.enabled()
    if _ALLOW_FALLBACK:
        return False
    raise MXNetError('HIP kernel extension not loaded on a GPU device: %s' % _K.load_error())


def _nd_to_ncx(x):
    nd = x.dim()
    return x.permute(0, nd - 1, *range(1, nd - 1))


def _ncx_to_nd(x):
    nd = x.dim()
    return x.permute(0, *range(2, nd), 1)


# ---------------------------------------------------------------------------
# GEMM-shaped ops
# ---------------------------------------------------------------------------

def linear(data, weight, bias):
    """y = data @ weight.T + bias (FullyConnected)."""
    if _use_hip(data) and _K.gemm_ok(data, weight):
        return _K.Linear.apply(data, weight, bias)
    if data.dim() == 2:
        return F.linear(data, weight, bias)
    return F.linear(data, weight, bias)


def embedding(data, weight):
    """Embedding lookup on the HIP gather / scatter-add kernels, or None (caller falls back)."""
    if _use_hip(weight) and _K.embedding_ok(data, weight):
        return _K.Embedding.apply(data, weight)
    return None


def _as_nhwc_view(t):
    """NHWC view of a 4-D NCHW-shaped tensor: free when its memory is channels-last (the output of a
    HIP conv/BN/pool below), one transpose copy otherwise (the network input)."""
    v = t.permute(0, 2, 3, 1)
    return v if v.is_contiguous() else v.contiguous()


def _nchw_on_hip(data):
    """The NCHW (default Gluon layout) fast path: HIP NHWC kernels over channels-last memory."""
    return (data.dim() == 4 and data.dtype in (torch.float16, torch.bfloat16) and _use_hip(data)
            and _NCHW_VIA_NHWC)


_NCHW_VIA_NHWC = os.environ.get('MXAMD_NCHW_VIA_NHWC', '1') == '1'


def _nhwc_weight(w):
    """KRSC layout of a KCRS weight for the channels-last kernels: a free view for 1x1 kernels, one
    permuted copy otherwise (ResNet-50: ~50 MB of the ~25 GB a training step moves).  Not cached: the
    optimizer kernels and replayed HIP graphs update weights without bumping tensor versions, so a
    cache could serve stale weights."""
    if w.shape[2] == 1 and w.shape[3] == 1 and w.is_contiguous():
        return w.view(w.shape[0], 1, 1, w.shape[1])
    return w.permute(0, 2, 3, 1).contiguous()


def conv(data, weight, bias, stride, pad, dilate, groups, channel_last):
    nsp = data.dim() - 2
    if groups > 1 and nsp == 2 and _use_hip(data):
        # depthwise (MobileNet): in-tree NHWC kernels, NCHW shapes through channels-last views
        from .conv_dw import dw_ok, ConvDwNHWC
        xl = data if channel_last else (_as_nhwc_view(data) if _nchw_on_hip(data) else None)
        if xl is not None and dw_ok(xl, weight, groups, dilate):
            rs = tuple(weight.shape[1:3]) if channel_last else tuple(weight.shape[2:4])
            y = ConvDwNHWC.apply(xl, weight, bias, rs, tuple(stride), tuple(pad), tuple(dilate))
            return y if channel_last else y.permute(0, 3, 1, 2)
    if not channel_last and nsp == 2 and _nchw_on_hip(data):
        # NCHW API, channels-last execution: activations stay NHWC in memory between HIP kernels
        # (NCHW-shaped permuted views), so the default layout runs on the same MFMA kernels
        xl = _as_nhwc_view(data)
        wl = _nhwc_weight(weight)
        if _K.conv_ok(xl, wl, stride, pad, dilate, groups):
            if _K.kpad_ok(xl, wl):
                return _K.conv_kpad(xl, wl, bias, stride, pad, dilate).permute(0, 3, 1, 2)
            return _K.ConvNHWC.apply(xl, wl, bias, tuple(stride), tuple(pad), tuple(dilate)).permute(0, 3, 1, 2)
    if channel_last and _use_hip(data) and _K.conv_ok(data, weight, stride, pad, dilate, groups):
        if _K.kpad_ok(data, weight):
            return _K.conv_kpad(data, weight, bias, stride, pad, dilate)
        return _K.ConvNHWC.apply(data, weight, bias, tuple(stride), tuple(pad), tuple(dilate))
    if nsp == 2 and groups == 1 and _use_hip(data) and tuple(dilate) != (1, 1):
        # dilated (atrous) 2-D convs: the big-tile / weight-gradient MFMA kernels with dilated taps
        xl = data if channel_last else (_as_nhwc_view(data) if _nchw_on_hip(data) else None)
        if xl is not None:
            wl = weight if channel_last else _nhwc_weight(weight)
            if _K.dil_ok(xl, wl, dilate):
                y = _K.ConvDilNHWC.apply(xl, wl, bias, tuple(stride), tuple(pad), tuple(dilate))
                return y if channel_last else y.permute(0, 3, 1, 2)
    if _use_hip(data):
        # grouped / dilated / 1-D / 3-D / fp32 / odd channel counts: the general in-tree MFMA kernel
        # (src/kernels/conv_gen.hip), chosen per shape against MIOpen by measured forward time
        from . import conv_gen
        y = conv_gen.conv(data, weight, bias, tuple(stride), tuple(pad), tuple(dilate), groups, channel_last)
        if y is not None:
            return y
    if channel_last:
        x = _nd_to_ncx(data)
        w = _nd_to_ncx(weight)
    else:
        x, w = data, weight
    fn = {1: F.conv1d, 2: F.conv2d, 3: F.conv3d}[nsp]
    y = fn(x, w, bias, stride=stride, padding=pad, dilation=dilate, groups=groups)
    return _ncx_to_nd(y) if channel_last else y


def conv_tee(data, weight, inplace_grad=False):
    """(conv1x1(data), data) with the identity-shortcut gradient fused into the dgrad GEMM."""
    if _use_hip(data) and hasattr(_K, 'ConvTeeNHWC') and _K.conv_tee_ok(data, weight):
        return _K.ConvTeeNHWC.apply(data, weight, bool(inplace_grad))
    return conv(data, weight, None, (1, 1), (0, 0), (1, 1), 1, True), data


# ---------------------------------------------------------------------------
# BatchNorm
# ---------------------------------------------------------------------------

def batch_norm_relu_maxpool(data, gamma, beta, moving_mean, moving_var, eps, momentum, fix_gamma, training,
                            axis, kernel, stride, pad, invstd_out=False):
    """max_pool(relu(BatchNorm(data))) -- the ResNet stem after its 7x7 conv. On channel-last HIP tensors
    one statistics pass and one pooling pass that applies the BatchNorm + ReLU to each window tap
    (kernel_fns.bnrelu_pool_ok); otherwise BatchNorm+ReLU followed by the pooling operator."""
    nd = data.dim()
    if (nd == 4 and axis % nd == 3 and _use_hip(data) and _K.bnrelu_pool_ok(data, kernel, stride, pad)):
        g = torch.ones_like(gamma) if fix_gamma else gamma
        return _K.BatchNormNHWC.apply(data, g, beta, None, eps, training, True, moving_mean, moving_var, momentum,
                                      invstd_out, (tuple(kernel), tuple(stride), tuple(pad)))
    out, m, v = batch_norm(data, gamma, beta, moving_mean, moving_var, eps, momentum, fix_gamma, training, axis,
                           'relu', invstd_out=invstd_out)
    return pool(out, 'max', tuple(kernel), tuple(stride), tuple(pad), 'valid', True, axis % nd == nd - 1), m, v


def batch_norm(data, gamma, beta, moving_mean, moving_var, eps, momentum, fix_gamma, training,
               axis, act_type, addend=None, invstd_out=False):
    """BatchNorm with MXNet semantics; returns (out, mean, var) -- (out, mean, 1/sqrt(var + eps)) in
    training mode with ``invstd_out`` (the reference's extra outputs, batch_norm.cc).

    ``moving_* = moving_* * momentum + batch_* * (1 - momentum)`` (biased
    variance, src/operator/nn/batch_norm.cc).  ``act_type='relu'`` fuses
    ReLU; ``addend`` fuses the residual add before the ReLU.
    """
    nd = data.dim()
    axis = axis % nd
    channel_last = (axis == nd - 1) and nd > 2
    g = torch.ones_like(gamma) if fix_gamma else gamma
    if axis == 1 and _nchw_on_hip(data) and data.permute(0, 2, 3, 1).is_contiguous():
        # channels-last memory behind an NCHW shape (a HIP conv's output): the NHWC kernel applies
        xl = data.permute(0, 2, 3, 1)
        al = _as_nhwc_view(addend) if addend is not None else None
        if _K.bn_ok(xl):
            out, m, v = _K.BatchNormNHWC.apply(xl, g, beta, al, eps, training, act_type == 'relu',
                                                moving_mean, moving_var, momentum, invstd_out)
            return out.permute(0, 3, 1, 2), m, v
    if channel_last and _use_hip(data) and _K.bn_ok(data):
        return _K.BatchNormNHWC.apply(data, g, beta, addend, eps, training, act_type == 'relu',
                                      moving_mean, moving_var, momentum, invstd_out)
    if channel_last:
        x = _nd_to_ncx(data)
    elif axis != 1:
        others = [i for i in range(nd) if i != axis]      # channel axis to position 1 (axis 0 included)
        perm = [others[0], axis] + others[1:]
        x = data.permute(*perm)
    else:
        x = data
    if training:
        out, smean, sinvstd = torch.ops.aten.native_batch_norm(x, g, beta, None, None, True, 0.0, eps)
        with torch.no_grad():
            var = (1.0 / (sinvstd.float() ** 2) - eps).clamp_(min=0.0) if sinvstd.numel() else sinvstd
            moving_mean.mul_(momentum).add_(smean.detach().to(moving_mean.dtype), alpha=1 - momentum)
            moving_var.mul_(momentum).add_(var.to(moving_var.dtype), alpha=1 - momentum)
        mean_out, var_out = smean, (sinvstd if invstd_out else var)
    else:
        out = F.batch_norm(x, moving_mean, moving_var, g, beta, False, 0.0, eps)
        mean_out, var_out = moving_mean, moving_var
    if channel_last:
        out = _ncx_to_nd(out)
    elif axis != 1:
        inv = [0] * nd
        others = [i for i in range(nd) if i != axis]
        perm = [others[0], axis] + others[1:]
        for i, p in enumerate(perm):
            inv[p] = i
        out = out.permute(*inv)
    if addend is not None:
        out = out + addend
    if act_type == 'relu':
        out = torch.relu(out)
    return out, mean_out, var_out


# ---------------------------------------------------------------------------
# Pooling
# ---------------------------------------------------------------------------

def global_pool(data, pool_type, channel_last):
    nsp = data.dim() - 2
    if not channel_last and pool_type == 'avg' and _nchw_on_hip(data) and data.permute(0, 2, 3, 1).is_contiguous():
        xl = data.permute(0, 2, 3, 1)
        if _K.gap_ok(xl):
            return _K.GlobalAvgPoolNHWC.apply(xl).permute(0, 3, 1, 2)
    if channel_last:
        if _use_hip(data) and nsp == 2 and pool_type == 'avg' and _K.gap_ok(data):
            return _K.GlobalAvgPoolNHWC.apply(data)
        dims = tuple(range(1, 1 + nsp))
    else:
        dims = tuple(range(2, 2 + nsp))
    if pool_type == 'max':
        return torch.amax(data, dim=dims, keepdim=True)
    if pool_type == 'sum':
        return torch.sum(data, dim=dims, keepdim=True)
    if pool_type == 'lp':
        return torch.sqrt(torch.sum(data * data, dim=dims, keepdim=True))
    return torch.mean(data, dim=dims, keepdim=True)


def _pool_out(n, k, s, p, conv):
    if conv == 'full':
        return int(-(-(n + 2 * p - k) // s)) + 1
    return (n + 2 * p - k) // s + 1


def pool(data, pool_type, kernel, stride, pad, convention, count_include_pad, channel_last, p_value=None):
    nsp = data.dim() - 2
    if not channel_last and nsp == 2 and pool_type in ('max', 'avg') and convention != 'same' \
            and _nchw_on_hip(data) and data.permute(0, 2, 3, 1).is_contiguous():
        xl = data.permute(0, 2, 3, 1)
        if _K.pool_ok(xl, kernel, stride, pad):
            return _K.PoolNHWC.apply(xl, pool_type, tuple(kernel), tuple(stride), tuple(pad),
                                     convention == 'full', bool(count_include_pad)).permute(0, 3, 1, 2)
    if channel_last and _use_hip(data) and nsp == 2 and pool_type in ('max', 'avg') \
            and _K.pool_ok(data, kernel, stride, pad):
        return _K.PoolNHWC.apply(data, pool_type, tuple(kernel), tuple(stride), tuple(pad),
                                 convention == 'full', bool(count_include_pad))
    x = _nd_to_ncx(data) if channel_last else data
    if channel_last and x.is_cuda and pool_type != 'max':
        # torch's channels_last avg-pool backward is wrong on ROCm (see tests/test_hip_kernels.py)
        x = x.contiguous()
    ceil = convention == 'full'
    pad_r = list(pad)
    if convention == 'same':
        ceil = False
        for i in range(nsp):
            n = x.shape[2 + i]
            out = -(-n // stride[i])
            tot = max((out - 1) * stride[i] + kernel[i] - n, 0)
            pad_r[i] = tot // 2
    if pool_type == 'max':
        fn = {1: F.max_pool1d, 2: F.max_pool2d, 3: F.max_pool3d}[nsp]
        y = fn(x, kernel, stride, pad_r, ceil_mode=ceil)
    elif pool_type == 'avg':
        fn = {1: F.avg_pool1d, 2: F.avg_pool2d, 3: F.avg_pool3d}[nsp]
        y = fn(x, kernel, stride, pad_r, ceil_mode=ceil, count_include_pad=count_include_pad)
    elif pool_type == 'sum':
        fn = {1: F.avg_pool1d, 2: F.avg_pool2d, 3: F.avg_pool3d}[nsp]
        y = fn(x, kernel, stride, pad_r, ceil_mode=ceil, count_include_pad=True) * float(torch.tensor(kernel).prod())
    elif pool_type == 'lp':
        pv = p_value or 2
        fn = {1: F.lp_pool1d, 2: F.lp_pool2d, 3: F.lp_pool3d}[nsp]
        if any(pad_r):
            x = F.pad(x, [q for pp in reversed(pad_r) for q in (pp, pp)])
        y = fn(x, pv, kernel, stride, ceil_mode=ceil)
    else:
        raise MXNetError('unknown pool_type %s' % pool_type)
    return _ncx_to_nd(y) if channel_last else y


# ---------------------------------------------------------------------------
# elementwise / normalisation
# ---------------------------------------------------------------------------

# MXAMD_HIP_ELEMWISE=0 sends relu and the broadcast binaries back to torch (A/B switch)
_HIP_ELEMWISE = os.environ.get('MXAMD_HIP_ELEMWISE', '1') == '1'


def relu(x):
    if _HIP_ELEMWISE and _use_hip(x) and _K.relu_ok(x):
        return _K.ReluHip.apply(x)
    return torch.relu(x)


def binary(op, a, b):
    """Broadcast add/sub/mul/div/maximum/minimum of two same-dtype GPU tensors on the in-tree
    kernel; None when the operands do not qualify (the caller runs the torch op)."""
    if (_HIP_ELEMWISE and isinstance(a, torch.Tensor) and isinstance(b, torch.Tensor) and _use_hip(a)
            and _K.binary_ok(a, b)):
        return _K.BinaryHip.apply(a, b, op)
    return None


def gelu(x):
    if _use_hip(x) and _K.ew_ok(x):
        return _K.GELU.apply(x)
    return F.gelu(x)


def layer_norm(data, gamma, beta, eps, want_stats=True):
    """LayerNorm over the last axis; returns (out, mean, std) (mean/std only meaningful with want_stats)."""
    if _use_hip(data) and _K.ln_ok(data):
        return _K.LayerNorm.apply(data, gamma, beta, eps, bool(want_stats))
    x = _acc(data)
    mean = x.mean(-1, keepdim=True)
    var = x.var(-1, keepdim=True, unbiased=False)
    std = torch.sqrt(var + eps)
    y = (x - mean) / std * _acc(gamma) + _acc(beta)
    return y.to(data.dtype), mean.to(data.dtype), std.to(data.dtype)


def add_dropout_layer_norm(x, h, gamma, beta, eps, p, handoff=False):
    """LayerNorm(x + dropout_p(h)) over the last axis: one HIP kernel each way on the GPU."""
    if (_use_hip(x) and x.dtype in (torch.float16, torch.bfloat16) and _K.ln_ok(x) and h.shape == x.shape
            and h.dtype == x.dtype and h.is_contiguous()
            and h.data_ptr() % 16 == 0 and 0.0 <= p < 1.0):
        return _K.AddDropoutLN.apply(x, h, gamma, beta, eps, p, bool(handoff))
    if p > 0:
        h = h * (torch.rand_like(h, dtype=torch.float32) >= p).to(h.dtype) / (1 - p)
    return layer_norm(x + h, gamma, beta, eps, False)[0]


def softmax(x, axis=-1, scale=1.0, log=False):
    """softmax / log_softmax of x*scale along ``axis``; None when the HIP kernel does not apply."""
    if _use_hip(x) and hasattr(_K, 'Softmax') and _K.softmax_ok(x, axis):
        return _K.Softmax.apply(x, scale, log)
    return None


def dropout(x, p):
    """(y, mask) Philox dropout on the GPU; None when the HIP kernel does not apply."""
    if _use_hip(x) and hasattr(_K, 'Dropout') and _K.ew_ok(x) and 0.0 < p < 1.0:
        return _K.Dropout.apply(x, p)
    return None


def softmax_ce(logits, label, reduction='none'):
    """Cross entropy of softmax(logits) against integer labels (fp32 accumulation).  Labels may be
    ``(N,)`` or ``(N, 1)`` (what NDArrayIter yields; the reference picks with keepdims, loss.py:390)."""
    if label.dim() > 1 and label.numel() == logits.shape[0]:
        label = label.reshape(-1)
    if _use_hip(logits) and _K.ce_ok(logits):
        loss = _K.SoftmaxCE.apply(logits, label)
    else:
        lg = logits.float() if logits.dtype in (torch.float16, torch.bfloat16) else logits
        loss = F.cross_entropy(lg, label.to(torch.int64), reduction='none')
    if reduction == 'sum':
        return loss.sum()
    if reduction == 'mean':
        return loss.mean()
    return loss
