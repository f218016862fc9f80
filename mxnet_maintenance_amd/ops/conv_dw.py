"""Depthwise (groups == channels) NHWC convolution on the in-tree gfx950 kernels (src/kernels/conv_dw.hip).

Parity: the depthwise path of src/operator/nn/depthwise_convolution-inl.h used by MobileNet v1/v2.
Forward / data-gradient are vector-memory gathers, the weight gradient is a fixed-order slab
reduction (deterministic).  ``dw_ok`` decides which convolutions take this path; the caller
(hip_ops.conv) falls back to MIOpen for everything else.
"""
import torch

from . import kernels as _K
from .kernel_fns import _DT, _stream

__all__ = ['dw_ok', 'ConvDwNHWC']


def dw_ok(x, w, groups, dilate):
    """NHWC x [N, H, W, C], weight [C, R, S, 1] (or [C, 1, R, S]) with groups == C == output channels."""
    if not (x.is_cuda and x.dim() == 4 and w.dim() == 4 and x.dtype in _DT and w.dtype == x.dtype):
        return False
    C = x.shape[3]
    taps = w.numel() // max(1, w.shape[0])
    return (groups == C and w.shape[0] == C and C % 8 == 0 and taps <= 25 and x.is_contiguous()
            and _K.available() and _K.enabled())


def _geom(x, R, S, stride, pad, dilate):
    N, H, W, C = x.shape
    Ho = (H + 2 * pad[0] - dilate[0] * (R - 1) - 1) // stride[0] + 1
    Wo = (W + 2 * pad[1] - dilate[1] * (S - 1) - 1) // stride[1] + 1
    return [N, H, W, C, Ho, Wo, R, S, stride[0], stride[1], pad[0], pad[1], dilate[0], dilate[1]]


class ConvDwNHWC(torch.autograd.Function):
    """y = depthwise_conv(x, w) (+ bias); ``rs`` = (R, S) of the kernel."""

    @staticmethod
    def forward(ctx, x, w, bias, rs, stride, pad, dilate):
        lib = _K.lib()
        R, S = rs
        g = _geom(x, R, S, stride, pad, dilate)
        C = g[3]
        wt = w.reshape(C, R * S).t().contiguous()                     # [R*S][C]: one 16-byte load per tap
        y = torch.empty((g[0], g[4], g[5], C), dtype=x.dtype, device=x.device)
        b32 = bias.float().contiguous() if bias is not None else None
        lib.conv_dw_fwd(_DT[x.dtype], x.data_ptr(), wt.data_ptr(), 0 if b32 is None else b32.data_ptr(),
                        y.data_ptr(), g, _stream())
        ctx.save_for_backward(x, wt)
        ctx.geom, ctx.wshape, ctx.has_bias = g, w.shape, bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _K.lib()
        x, wt = ctx.saved_tensors
        g = ctx.geom
        dy = dy.contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            lib.conv_dw_dgrad(_DT[x.dtype], dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), g, _stream())
        if ctx.needs_input_grad[1]:
            C, taps = g[3], g[6] * g[7]
            npos = g[0] * g[4] * g[5]
            nslice = max(1, min(npos, 65536 // (C // 8)))
            slab = torch.empty((nslice, taps, C), dtype=torch.float32, device=x.device)
            dw = torch.empty(ctx.wshape, dtype=x.dtype, device=x.device)
            lib.conv_dw_wgrad(_DT[x.dtype], x.data_ptr(), dy.data_ptr(), slab.data_ptr(), nslice, _DT[x.dtype],
                              dw.data_ptr(), 0, g, _stream())
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy.float().sum(dim=(0, 1, 2))
        return dx, dw, db, None, None, None, None
