"""General convolution / transposed convolution on the in-tree gfx950 kernel (src/kernels/conv_gen.hip).

Covers what the specialised NHWC kernels do not: grouped (non-depthwise) convolution, dilation,
1-D / 3-D, channel counts that are not multiples of 32/64, fp32, and Deconvolution (the data
gradient of a convolution, reference src/operator/nn/deconvolution-inl.h:207).

Tensors are channels-last 5-D inside (N, D, H, W, C; 1-D and 2-D get unit D / H), weights
[K][T][R][S][C/G].  ``conv_gen_fwd`` / ``conv_gen_dgrad`` / ``conv_gen_wgrad`` are the three GEMM
views; ``ConvGen`` and ``DeconvGen`` are their autograd pairings.  Per shape the first call times the
in-tree kernel against MIOpen (forward pass, numerics-checked, like every other conv choice in
kernel_fns) and keeps the faster; MXAMD_REQUIRE_HIP=1 pins the in-tree kernel.
"""
import os

import torch
import torch.nn.functional as F

from . import kernels as _K

_DT = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}


def _stream():
    return torch.cuda.current_stream().cuda_stream


def gen_ok(x, w):
    return (x.is_cuda and x.dtype in _DT and w.dtype == x.dtype and _K.available()
            and hasattr(_K.lib(), 'conv_gen'))


def _out_dim(n, k, s, p, d):
    return (n + 2 * p - d * (k - 1) - 1) // s + 1


def _geom(xshape, wshape, groups, stride, pad, dil, out_sp=None):
    """22-int geometry of conv_gen.hip from 5-D channels-last shapes."""
    N, D, H, W, C = xshape
    K, T, R, S, _cg = wshape
    if out_sp is None:
        out_sp = (_out_dim(D, T, stride[0], pad[0], dil[0]), _out_dim(H, R, stride[1], pad[1], dil[1]),
                  _out_dim(W, S, stride[2], pad[2], dil[2]))
    return [N, D, H, W, C, K, groups, T, R, S, out_sp[0], out_sp[1], out_sp[2],
            stride[0], stride[1], stride[2], pad[0], pad[1], pad[2], dil[0], dil[1], dil[2]]


def conv_gen_fwd(x, w, bias, groups, stride, pad, dil, out_sp=None):
    """y [N, Do, Ho, Wo, K] = conv(x [N, D, H, W, C], w [K, T, R, S, C/G]) (+ bias)."""
    x = x.contiguous()
    w = w.contiguous()
    g = _geom(x.shape, w.shape, groups, stride, pad, dil, out_sp)
    y = torch.empty((g[0], g[10], g[11], g[12], g[5]), dtype=x.dtype, device=x.device)
    b = bias.float().contiguous() if bias is not None else None
    _K.lib().conv_gen(_DT[x.dtype], 0, x.data_ptr(), w.data_ptr(), 0 if b is None else b.data_ptr(), y.data_ptr(),
                      g, 1, _stream())
    return y


def _w_transposed(w, groups):
    """[G*Cg][T][R][S][Kg] from [K][T][R][S][Cg] (the dgrad GEMM's contiguous-k weight rows)."""
    K, T, R, S, Cg = w.shape
    Kg = K // groups
    return w.reshape(groups, Kg, T * R * S, Cg).permute(0, 3, 2, 1).contiguous()


def conv_gen_dgrad(dy, w, xsp, groups, stride, pad, dil, bias=None):
    """dx [N, D, H, W, C] of a conv whose output gradient is dy [N, Do, Ho, Wo, K] (also the forward
    of a transposed convolution with input dy; ``bias`` then adds per output channel)."""
    dy = dy.contiguous()
    N = dy.shape[0]
    K = dy.shape[4]
    Cg = w.shape[4]
    C = Cg * groups
    g = _geom((N,) + tuple(xsp) + (C,), w.shape, groups, stride, pad, dil, out_sp=tuple(dy.shape[1:4]))
    wT = _w_transposed(w.contiguous(), groups)
    dx = torch.empty((N,) + tuple(xsp) + (C,), dtype=dy.dtype, device=dy.device)
    b = bias.float().contiguous() if bias is not None else None
    assert g[5] == K
    _K.lib().conv_gen(_DT[dy.dtype], 1, dy.data_ptr(), wT.data_ptr(), 0 if b is None else b.data_ptr(),
                      dx.data_ptr(), g, 1, _stream())
    return dx


def conv_gen_wgrad(x, dy, wshape, groups, stride, pad, dil):
    """dW [K, T, R, S, C/G] from x [N, D, H, W, C] and dy [N, Do, Ho, Wo, K] (split-K fp32 slabs summed
    in a fixed order: deterministic)."""
    x = x.contiguous()
    dy = dy.contiguous()
    g = _geom(x.shape, wshape, groups, stride, pad, dil, out_sp=tuple(dy.shape[1:4]))
    K, T, R, S, Cg = wshape
    Kg = K // groups
    cols = T * R * S * Cg
    pix = dy.shape[0] * dy.shape[1] * dy.shape[2] * dy.shape[3]
    tiles = ((Kg + 63) // 64) * ((cols + 63) // 64) * groups
    # enough workgroups to cover the chip, each reducing at least ~512 pixels
    splits = max(1, min(64, (512 + tiles - 1) // tiles, pix // 512 or 1))
    slab = torch.empty((splits, groups, Kg, cols), dtype=torch.float32, device=x.device)
    _K.lib().conv_gen(_DT[x.dtype], 2, dy.data_ptr(), x.data_ptr(), 0, slab.data_ptr(), g, splits, _stream())
    return slab.sum(0).reshape(K, T, R, S, Cg).to(x.dtype)


# ---- layout helpers: framework tensors <-> 5-D channels-last
def to5(t, channel_last):
    """5-D channels-last view/copy of a 3/4/5-D activation in NC* or N*C layout."""
    if not channel_last:
        t = t.movedim(1, -1)
    while t.dim() < 5:
        t = t.unsqueeze(1)
    return t.contiguous()


def from5(t, nsp, channel_last):
    while t.dim() > nsp + 2:
        t = t.squeeze(1)
    return t if channel_last else t.movedim(-1, 1)


def pad3(v, nsp, fill):
    v = tuple(v)
    return (fill,) * (3 - nsp) + v


class ConvGen(torch.autograd.Function):
    """Convolution on conv_gen.hip: forward, input gradient and weight gradient all in-tree."""

    @staticmethod
    def forward(ctx, x5, w5, bias, groups, stride, pad, dil):
        y = conv_gen_fwd(x5, w5, bias, groups, stride, pad, dil)
        ctx.save_for_backward(x5, w5)
        ctx.cfg = (groups, stride, pad, dil)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x5, w5 = ctx.saved_tensors
        groups, stride, pad, dil = ctx.cfg
        dy = dy.contiguous()
        dx = conv_gen_dgrad(dy, w5, x5.shape[1:4], groups, stride, pad, dil) if ctx.needs_input_grad[0] else None
        dw = conv_gen_wgrad(x5, dy, w5.shape, groups, stride, pad, dil) if ctx.needs_input_grad[1] else None
        db = dy.float().sum((0, 1, 2, 3)).to(dy.dtype) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return dx, dw, db, None, None, None, None


class DeconvGen(torch.autograd.Function):
    """Transposed convolution: y = conv^T(x, w) with w [Cin][T][R][S][Cout/G] (the conv weight of the
    conv whose input gradient this is); backward: dx = conv(dy, w), dW = wgrad(dy, x)."""

    @staticmethod
    def forward(ctx, x5, w5, bias, groups, stride, pad, dil, out_sp):
        y = conv_gen_dgrad(x5, w5, out_sp, groups, stride, pad, dil, bias=bias)
        ctx.save_for_backward(x5, w5)
        ctx.cfg = (groups, stride, pad, dil)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x5, w5 = ctx.saved_tensors
        groups, stride, pad, dil = ctx.cfg
        dy = dy.contiguous()
        dx = conv_gen_fwd(dy, w5, None, groups, stride, pad, dil, out_sp=tuple(x5.shape[1:4])) \
            if ctx.needs_input_grad[0] else None
        dw = conv_gen_wgrad(dy, x5, w5.shape, groups, stride, pad, dil) if ctx.needs_input_grad[1] else None
        db = dy.float().sum((0, 1, 2, 3)).to(dy.dtype) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return dx, dw, db, None, None, None, None, None


# ---- algorithm choice vs MIOpen (forward-timed, numerics-checked)
_CHOICE = {}


def _require_hip():
    return os.environ.get('MXAMD_REQUIRE_HIP', '0') == '1'


def choose(key, gen_fn, vendor_fn):
    """'gen' or 'vendor' for ``key``: the first call times both forward closures (under no_grad)."""
    if _require_hip():
        return 'gen'
    name = _CHOICE.get(key)
    if name is not None:
        return name
    from . import kernel_fns as KF
    if not KF._AUTOTUNE or torch.cuda.is_current_stream_capturing():
        return 'gen'
    with torch.no_grad():
        name, _ = KF._time_candidates([('miopen', vendor_fn), ('gen', gen_fn)], key=('convgen',) + key)
    name = 'gen' if name == 'gen' else 'vendor'
    _CHOICE[key] = name
    return name


def conv(data, weight, bias, stride, pad, dil, groups, channel_last):
    """Convolution of framework tensors on the generic kernel (or MIOpen when that measured faster);
    None when the kernel cannot take the operands."""
    if not gen_ok(data, weight):
        return None
    nsp = data.dim() - 2
    if nsp not in (1, 2, 3):
        return None
    x5 = to5(data, channel_last)
    w5 = to5(weight, channel_last)
    st, pd, dl = pad3(stride, nsp, 1), pad3(pad, nsp, 0), pad3(dil, nsp, 1)
    key = ('fwd', tuple(x5.shape), tuple(w5.shape), groups, st, pd, dl, x5.dtype, bias is not None)

    def vendor():
        fn = {1: F.conv1d, 2: F.conv2d, 3: F.conv3d}[nsp]
        xn = data if not channel_last else data.movedim(-1, 1)
        wn = weight if not channel_last else weight.movedim(-1, 1)
        return fn(xn, wn, bias, stride=tuple(stride), padding=tuple(pad), dilation=tuple(dil), groups=groups)

    def gen():
        return from5(conv_gen_fwd(x5, w5, bias, groups, st, pd, dl), nsp, False)

    if choose(key, gen, vendor) == 'vendor':
        y = vendor()
        return y.movedim(1, -1) if channel_last else y
    return from5(ConvGen.apply(x5, w5, bias, groups, st, pd, dl), nsp, channel_last)


def deconv(data, weight, bias, stride, pad, dil, adj, groups, channel_last):
    """Transposed convolution of framework tensors (MXNet Deconvolution; weight [Cin, Cout/G, k...]
    or channels-last [Cin, k..., Cout/G]); None when the kernel cannot take the operands."""
    if not gen_ok(data, weight):
        return None
    nsp = data.dim() - 2
    if nsp not in (1, 2, 3):
        return None
    x5 = to5(data, channel_last)
    w5 = to5(weight, channel_last)
    st, pd, dl, aj = pad3(stride, nsp, 1), pad3(pad, nsp, 0), pad3(dil, nsp, 1), pad3(adj, nsp, 0)
    T, R, S = w5.shape[1:4]
    out_sp = tuple((x5.shape[1 + i] - 1) * st[i] - 2 * pd[i] + dl[i] * ((T, R, S)[i] - 1) + 1 + aj[i]
                   for i in range(3))
    key = ('deconv', tuple(x5.shape), tuple(w5.shape), groups, st, pd, dl, aj, x5.dtype, bias is not None)

    def vendor():
        fn = {1: F.conv_transpose1d, 2: F.conv_transpose2d, 3: F.conv_transpose3d}[nsp]
        xn = data if not channel_last else data.movedim(-1, 1)
        wn = weight if not channel_last else weight.movedim(-1, 1)
        return fn(xn, wn, bias, stride=tuple(stride), padding=tuple(pad), output_padding=tuple(adj),
                  groups=groups, dilation=tuple(dil))

    def gen():
        return from5(conv_gen_dgrad(x5, w5, out_sp, groups, st, pd, dl, bias=bias), nsp, False)

    if choose(key, gen, vendor) == 'vendor':
        y = vendor()
        return y.movedim(1, -1) if channel_last else y
    return from5(DeconvGen.apply(x5, w5, bias, groups, st, pd, dl, out_sp), nsp, channel_last)
