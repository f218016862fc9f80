"""torch.autograd wrappers around the gfx950 HIP kernels.

Each wrapper validates shapes/dtypes/contiguity on the host (the kernels assume
them), allocates outputs with the torch caching allocator and launches on the
current HIP stream.  Numerics are checked against fp32 torch references in
tests/test_hip_kernels.py.
"""
import os

import torch

from . import kernels as _K
from .. import _state
from ..utils import env as _env

__all__ = ['BatchNormNHWC', 'SoftmaxCE', 'GlobalAvgPoolNHWC', 'flat_sgd']

_DT = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _p(t):
    return 0 if t is None else t.data_ptr()


def _f32(t):
    """fp32 view of a (small, per-channel) parameter: itself, its multi-precision fp32 master copy when
    the trainer's flat arena registered one (no conversion kernel), or a converted copy."""
    if t.dtype == torch.float32 and t.is_contiguous():
        return t
    m = getattr(t, '_mxamd_master', None)
    if m is not None and m[1] == t._version and m[0].shape == t.shape:
        return m[0]
    return t.float().contiguous()


# ---------------------------------------------------------------------------
# predicates (override the conservative defaults in kernels.py)
# ---------------------------------------------------------------------------

def bn_ok(x):
    C = x.shape[-1] if x.dim() else 0
    return (x.dtype in _DT and x.dim() >= 2 and x.is_contiguous() and C % 8 == 0
            and x.numel() > 0 and x.data_ptr() % 16 == 0)


def ce_ok(x):
    return x.dim() == 2 and x.dtype in _DT and x.is_contiguous()




def _leaf_grad(t, numel=None, dtype=torch.float32):
    """The .grad buffer of leaf ``t`` when a kernel may accumulate into it directly.

    Only inside mx.autograd.backward (not torch.autograd.grad, not create_graph),
    where .grad IS the destination: the buffer exists (our autograd
    zeroes grad_req='write' buffers before backward), is contiguous, of the
    expected dtype/size.  The caller then returns None for that input so
    torch's AccumulateGrad (a separate add kernel per parameter) never runs.
    """
    if t is None or _state.DIRECT_GRAD[0] <= 0 or torch.is_grad_enabled() or not t.is_leaf or not t.requires_grad:
        return None
    gb = t.grad
    if gb is None or gb.dtype != dtype or not gb.is_contiguous() or gb.shape != t.shape:
        return None
    if numel is not None and gb.numel() != numel:
        return None
    return gb


_RELU_FROM_X = [True]    # BN+ReLU backward recomputes the mask from x (debug switch)
_BN_BWD_FUSE = [os.environ.get('MXAMD_BN_BWD_FUSE', '1') != '0']   # BN-backward stats in dgrad epilogues
_BN_TAIL_DS = [os.environ.get('MXAMD_BN_TAIL_DS', '1') != '0']     # shortcut-BN stats in the tail backward
_BN_POOL_BWD = [True]    # stem BN+ReLU+pool backward as two gather passes (tests flip it for the A/B)
_ZEROS = {}


def _zeros_f32(n, dev):
    """A cached all-zero fp32 vector (statistics centre for conv-epilogue BN partials)."""
    z = _ZEROS.get((n, dev))
    if z is None:
        z = _ZEROS[(n, dev)] = torch.zeros(n, dtype=torch.float32, device=dev)
    return z


class _BnToken:
    """Identifies one BatchNorm call for the statistics / gradient hand-offs between fused kernels.
    ``lazy``: (dy, mask, version) when a residual tail handed this (shortcut) BatchNorm its incoming
    gradient as dy with the tail's ReLU mask still to apply."""
    __slots__ = ('lazy',)

    def __init__(self):
        self.lazy = None


class BatchNormNHWC(torch.autograd.Function):
    """BatchNorm over the last (channel) axis with optional fused residual add + ReLU."""

    @staticmethod
    def forward(ctx, x, gamma, beta, addend, eps, training, relu, moving_mean, moving_var, momentum=None,
                invstd_out=False, pool=None):
        # pool = ((kh, kw), (sh, sw), (ph, pw)): 3x3 max pooling of the BN + ReLU output in one pass
        # (pool_nhwc.hip's BatchNorm prologue; bnrelu_pool_ok) -- the normalised activation is never
        # materialised and the backward routes the pooled gradient first
        lib = _K.lib()
        C = x.shape[-1]
        R = x.numel() // C
        dev = x.device
        g = _f32(gamma)
        b = _f32(beta)
        mm = _f32(moving_mean)
        assert pool is None or (relu and addend is None)
        y = torch.empty_like(x) if pool is None else None
        if addend is not None:
            assert addend.shape == x.shape and addend.dtype == x.dtype
            addend = addend.contiguous()
        ext_nblk = 0
        center = mm
        if training:
            ext = getattr(x, '_mxamd_bn_part', None)
            if ext is not None and ext[0].numel() == 2 * C * ext[1] and ext[0].device == dev:
                # per-channel sum / sum-of-squares partials written by the producing conv's epilogue
                part, ext_nblk = ext
                center = _zeros_f32(C, dev)
            else:
                nblk = lib.bn_partials_rows(R, C)
                part = torch.empty(2 * nblk * C, dtype=torch.float32, device=dev)
            stats = torch.empty(5, C, dtype=torch.float32, device=dev)
            mean, invstd, var, scale, shift = stats.unbind(0)
        else:
            part = None
            mean = mm
            invstd = torch.rsqrt(_f32(moving_var) + eps)
            var = _f32(moving_var)
            scale = g * invstd
            shift = b - mean * scale
        # moving statistics are updated inside the finalize kernel when the
        # buffers are fp32 + contiguous (always true for Gluon BN params)
        upd = (training and momentum is not None and mm is moving_mean and moving_var.dtype == torch.float32
               and moving_var.is_contiguous())
        # residual tail (add + relu): the forward writes a 1-bit-per-element ReLU mask so the backward
        # never re-reads y (two full-tensor reads fewer per call)
        mask = (torch.empty(x.numel() // 8, dtype=torch.uint8, device=dev)
                if (addend is not None and relu and _RELU_FROM_X[0]) else None)
        lib.bn_nhwc_forward(_DT[x.dtype], x.data_ptr(), _p(addend), _p(y), _p(mask), g.data_ptr(),
                            b.data_ptr(),
                            center.data_ptr(), _p(part), mean.data_ptr(), invstd.data_ptr(), var.data_ptr(),
                            scale.data_ptr(), shift.data_ptr(), R, C, float(eps), int(bool(training)),
                            int(bool(relu)), 0, float(momentum or 0.0), moving_mean.data_ptr() if upd else 0,
                            moving_var.data_ptr() if upd else 0, int(ext_nblk), _stream())
        if training and momentum is not None and not upd:
            with torch.no_grad():
                moving_mean.mul_(momentum).add_(mean.to(moving_mean.dtype), alpha=1 - momentum)
                moving_var.mul_(momentum).add_(var.to(moving_var.dtype), alpha=1 - momentum)
        ctx.pool = None
        if pool is not None:
            (kh, kw), (sh, sw), (ph, pw) = pool
            N, H, W = x.shape[:3]
            Ho, Wo = _pool_out(H, kh, sh, ph, False), _pool_out(W, kw, sw, pw, False)
            y = torch.empty((N, Ho, Wo, C), dtype=x.dtype, device=dev)
            arg = torch.empty((N, Ho, Wo, C), dtype=torch.uint8, device=dev)
            ctx.pool = (N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw, 1)
            lib.pool_nhwc_forward_bnrelu(_DT[x.dtype], x.data_ptr(), y.data_ptr(), arg.data_ptr(), *ctx.pool,
                                         _stream(), scale.data_ptr(), shift.data_ptr())
            mask = arg        # saved in the mask slot: relu_mode 2 recomputes the ReLU mask from x
        # ReLU mask in backward: recomputed from x*scale+shift for BN+ReLU (y not kept),
        # read from y only for the residual tail (its mask also depends on the addend)
        relu_mode = 0 if not relu else (1 if not _RELU_FROM_X[0] else (3 if addend is not None else 2))
        if pool is not None:
            relu_mode = 2
        ctx.save_for_backward(x, y if relu_mode == 1 else mask, g, mean, invstd,
                              scale if relu_mode == 2 else None, shift if relu_mode == 2 else None)
        ctx.cfg = (relu_mode, bool(training), addend is not None, gamma.dtype, beta.dtype)
        # the addend is a tee conv's passthrough: the shortcut gradient may be handed over lazily
        ctx.tee_key = getattr(addend, '_mxamd_tee_key', None) if (addend is not None and relu_mode == 3) else None
        ctx.bn_token = None
        if training and relu_mode in (0, 2, 3) and _BN_BWD_FUSE[0] and pool is None:
            # a consumer convolution's dgrad (big-tile kernel) may emit this BN's backward statistics
            # from its epilogue: it needs z (= x here), mean, the ReLU mask source, and a token that
            # identifies this BN call (checked in backward)
            ctx.bn_token = _BnToken()
            y._mxamd_bn_src = (x, mean, scale if relu_mode == 2 else None, shift if relu_mode == 2 else None,
                               mask if relu_mode == 3 else None, relu_mode, ctx.bn_token)
        ctx.refs = (gamma, beta)
        # residual tail fed by a projection shortcut's BatchNorm (no ReLU): the tail's backward apply
        # also reduces that BN's backward statistics (its incoming gradient is the tail's dz)
        ctx.add_src = None
        if relu_mode == 3 and training and _BN_BWD_FUSE[0] and _BN_TAIL_DS[0]:
            src = getattr(addend, '_mxamd_bn_src', None)
            if (src is not None and src[5] == 0 and tuple(src[0].shape) == tuple(x.shape)
                    and src[0].dtype == x.dtype and src[0].is_contiguous()):
                ctx.add_src = src
        # invstd_out: the third output is the batch 1/sqrt(var + eps) the kernel already wrote (the
        # reference's training-mode extra output) instead of the variance
        third = invstd if (invstd_out and training) else var
        ctx.mark_non_differentiable(mean, third)
        # mean/var never receive gradients: skip materialising two zero tensors per call
        ctx.set_materialize_grads(False)
        return y, mean, third

    @staticmethod
    def backward(ctx, gy, _gm, _gv):
        lib = _K.lib()
        x, y, g, mean, invstd, fscale, fshift = ctx.saved_tensors
        relu_mode, training, has_add, gdt, bdt = ctx.cfg
        gamma_ref, beta_ref = ctx.refs
        if gy is None:
            return (None,) * 12
        gy = gy.contiguous()
        C = x.shape[-1]
        R = x.numel() // C
        dev = x.device
        fused_pool = False
        if ctx.pool is not None:
            fused_pool = (x.dtype in (torch.float16, torch.bfloat16) and 256 % (C // 8) == 0
                          and hasattr(lib, 'bn_pool_backward') and _BN_POOL_BWD[0])
            if not fused_pool:
                # the pooled gradient routed back to the BN output's shape first (argmax gather)
                gyd = torch.empty_like(x)
                lib.pool_nhwc_backward(_DT[x.dtype], 1, gy.data_ptr(), y.data_ptr(), gyd.data_ptr(), *ctx.pool,
                                       _stream())
                gy, y = gyd, None
        # a residual tail handed this (shortcut) BatchNorm its gradient lazily: gy is the tail's dy and the
        # tail's ReLU mask is applied in this backward's passes (unless autograd summed other gradients in)
        lazy_mask = None
        tok = ctx.bn_token
        if tok is not None and tok.lazy is not None:
            dy_l, mask_l, ver_l = tok.lazy
            tok.lazy = None
            if gy is dy_l and gy._version == ver_l and relu_mode == 0 and not has_add and ctx.pool is None:
                lazy_mask = mask_l
            else:
                gy = (gy - dy_l + _materialize_dz(dy_l, mask_l)).contiguous()
        dx = torch.empty_like(x)
        dz = torch.empty_like(x) if has_add else None
        ext = getattr(gy, '_mxamd_bn_bwd', None)
        ext_nblk = 0
        if (ext is not None and ctx.bn_token is not None and ext[2] is ctx.bn_token
                and ext[3] == gy._version):
            part, ext_nblk = ext[0], ext[1]      # statistics from the producing dgrad's epilogue
        else:
            nblk = lib.bn_partials_rows(R, C)
            part = torch.empty(2 * nblk * C, dtype=torch.float32, device=dev)
        out = torch.empty(5, C, dtype=torch.float32, device=dev)
        need_g, need_b = ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        # accumulate dgamma/dbeta straight into the parameters' fp32 grad buffers (arena views)
        tg = _leaf_grad(gamma_ref, C) if need_g else None
        tb = _leaf_grad(beta_ref, C) if need_b else None
        direct = tb is not None and (tg is not None or not need_g) and (tg is not None or tb is not None)
        if direct:
            dg_buf = tg if tg is not None else torch.zeros(C, dtype=torch.float32, device=dev)
            dg_ptr, db_ptr, accum = dg_buf.data_ptr(), tb.data_ptr(), 1
        else:
            dg_ptr, db_ptr, accum = out[0].data_ptr(), out[1].data_ptr(), 0
        if fused_pool:
            # statistics and dx straight from the pooled gradient (two gather passes, pool_nhwc.hip): the
            # routed full-resolution gradient is never materialised
            N_, H_, W_, C_, Ho_, Wo_, kh, kw, sh, sw, ph, pw, _ = ctx.pool
            ppart = torch.empty(2 * lib.bn_pool_bwd_blocks() * C, dtype=torch.float32, device=dev)
            lib.bn_pool_backward(_DT[x.dtype], x.data_ptr(), gy.data_ptr(), y.data_ptr(), dx.data_ptr(), g.data_ptr(),
                                 mean.data_ptr(), invstd.data_ptr(), fscale.data_ptr(), fshift.data_ptr(),
                                 ppart.data_ptr(), dg_ptr, db_ptr, out[2].data_ptr(), N_, H_, W_, C_, Ho_, Wo_, kh, kw,
                                 sh, sw, ph, pw, 0, int(training), accum, _stream())
            if direct:
                return dx, None, None, None, None, None, None, None, None, None, None, None
            return (dx, out[0].to(gdt) if need_g else None, out[1].to(bdt) if need_b else None,
                    None, None, None, None, None, None, None, None, None)
        ymask = y if relu_mode == 3 else None
        y = y if relu_mode == 1 else None
        ds = ctx.add_src if dz is not None else None
        # identity shortcut into a tee data gradient that takes a masked addend: d_addend = gy * mask is
        # not written here; gy goes back with the mask attached (ConvTeeNHWC._tee_dgrad multiplies it in)
        lazy = (dz is not None and ds is None and ymask is not None and ctx.tee_key is not None
                and lazy_shortcut_ok(ctx.tee_key))
        # projection shortcut: its BatchNorm takes dy + this mask directly (relu-from-mask apply)
        lazy_ds = (dz is not None and ds is not None and ymask is not None and _LAZY_DZ[0]
                   and isinstance(ds[6], _BnToken))
        if lazy or lazy_ds:
            dz = None
        kmode = relu_mode
        if lazy_mask is not None:
            kmode, ymask = 3, lazy_mask
        dkw = {}
        if ds is not None:
            ds_nblk = lib.bn_tail_ds_rows(R, C)
            ds_part = torch.empty(2 * ds_nblk * C, dtype=torch.float32, device=dev)
            dkw = dict(ds_z=ds[0].data_ptr(), ds_mean=ds[1].data_ptr(), ds_part=ds_part.data_ptr())
        lib.bn_nhwc_backward(_DT[x.dtype], x.data_ptr(), gy.data_ptr(), _p(y), _p(ymask), dx.data_ptr(), _p(dz),
                             g.data_ptr(),
                             mean.data_ptr(), invstd.data_ptr(), _p(fscale), _p(fshift), part.data_ptr(), dg_ptr,
                             db_ptr, out[2].data_ptr(), R, C, kmode, 0, int(training), accum, _stream(),
                             ext_nblk, **dkw)
        if ds is not None:
            # consumed by the shortcut BN's backward (token + version checked there)
            if lazy_ds:
                gy._mxamd_bn_bwd = (ds_part, ds_nblk, ds[6], gy._version)
                ds[6].lazy = (gy, ymask, gy._version)
                dz = gy
            else:
                dz._mxamd_bn_bwd = (ds_part, ds_nblk, ds[6], dz._version)
        if lazy:
            gy._mxamd_lazy_mask = (ymask, gy._version)
            dz = gy
        if direct:
            # returning None: torch still runs the leaves' AccumulateGrad node with an undefined
            # gradient, which fires their post-accumulate hooks (bucketed all-reduce readiness)
            dgamma = None
            dbeta = None
        else:
            dgamma = out[0].to(gdt) if need_g else None
            dbeta = out[1].to(bdt) if need_b else None
        return dx, dgamma, dbeta, dz, None, None, None, None, None, None, None, None


def bnrelu_pool_ok(x, kernel, stride, pad):
    """BatchNorm + ReLU + max pooling in one pass (BatchNormNHWC pool=): 3x3 windows, NHWC f16/bf16/f32
    with C % 8 == 0 and 32-bit element offsets (pool_nhwc.hip pool_fwd_max3_kernel<AFF>)."""
    return (bn_ok(x) and tuple(kernel) == (3, 3) and pool_ok(x, kernel, stride, pad)
            and x.numel() + 256 * 32 * 256 * 8 < 2 ** 31 and hasattr(_K.lib(), 'pool_nhwc_forward_bnrelu'))


class SoftmaxCE(torch.autograd.Function):
    """Per-row softmax cross-entropy with integer (or float-coded) labels; fp32 loss."""

    @staticmethod
    def forward(ctx, logits, label):
        lib = _K.lib()
        N, K = logits.shape
        lab = label.reshape(-1)
        is_int = not lab.is_floating_point()
        lab = lab.to(torch.int64).contiguous() if is_int else lab.float().contiguous()
        loss = torch.empty(N, dtype=torch.float32, device=logits.device)
        lse = torch.empty(N, dtype=torch.float32, device=logits.device)
        lib.softmax_ce_forward(_DT[logits.dtype], int(is_int), logits.data_ptr(), lab.data_ptr(), loss.data_ptr(),
                               lse.data_ptr(), N, K, _stream())
        ctx.save_for_backward(logits, lab, lse)
        ctx.is_int = is_int
        return loss

    @staticmethod
    def backward(ctx, gout):
        lib = _K.lib()
        logits, lab, lse = ctx.saved_tensors
        N, K = logits.shape
        g = gout.float().contiguous()
        dl = torch.empty_like(logits)
        lib.softmax_ce_backward(_DT[logits.dtype], int(ctx.is_int), logits.data_ptr(), lab.data_ptr(),
                                lse.data_ptr(), g.data_ptr(), dl.data_ptr(), N, K, _stream())
        return dl, None


class GlobalAvgPoolNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        lib = _K.lib()
        x = x.contiguous()
        N, C = x.shape[0], x.shape[-1]
        HW = x.numel() // (N * C)
        y = torch.empty((N,) + (1,) * (x.dim() - 2) + (C,), dtype=x.dtype, device=x.device)
        lib.gap_nhwc_forward(_DT[x.dtype], x.data_ptr(), y.data_ptr(), N, HW, C, _stream())
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, gy):
        lib = _K.lib()
        shape = ctx.shape
        N, C = shape[0], shape[-1]
        HW = int(torch.tensor(shape[1:-1]).prod())
        gy = gy.contiguous()
        dx = torch.empty(shape, dtype=gy.dtype, device=gy.device)
        lib.gap_nhwc_backward(_DT[gy.dtype], gy.data_ptr(), dx.data_ptr(), N, HW, C, _stream())
        return dx


def gap_ok(x):
    return x.dtype in _DT and x.is_contiguous() and x.shape[-1] % 8 == 0


# ---------------------------------------------------------------------------------- pointwise
class ReluHip(torch.autograd.Function):
    """relu / _backward_relu on src/kernels/pointwise.hip (16-byte vector lanes)."""

    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        y = torch.empty_like(x)
        _K.lib().relu_forward(_DT[x.dtype], x.data_ptr(), y.data_ptr(), x.numel(), _stream())
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, gy):
        y, = ctx.saved_tensors
        gy = gy.contiguous()
        dx = torch.empty_like(y)
        _K.lib().relu_backward(_DT[y.dtype], y.data_ptr(), gy.data_ptr(), dx.data_ptr(), y.numel(), _stream())
        return dx


def relu_ok(x):
    return x.dtype in _DT and x.is_cuda and x.numel() > 0 and x.data_ptr() % 16 == 0 and x.is_contiguous()


_PW_OPS = {'add': 0, 'sub': 1, 'mul': 2, 'div': 3, 'maximum': 4, 'minimum': 5}


def _bcast_strides(t, shape):
    """Element strides of ``t`` broadcast to ``shape`` (0 on broadcast axes)."""
    lead = len(shape) - t.dim()
    st = [0] * lead + list(t.stride())
    sz = [1] * lead + list(t.shape)
    return [0 if sz[d] == 1 and shape[d] != 1 else st[d] for d in range(len(shape))]


def _collapse(shape, sa, sb):
    """Merge adjacent dimensions that are contiguous for both operands (fewer index divisions)."""
    dims = [(n, a, b) for n, a, b in zip(shape, sa, sb) if n != 1] or [(1, 0, 0)]
    out = [list(dims[-1])]
    for n, a, b in reversed(dims[:-1]):
        pn, pa, pb = out[0]
        if a == pa * pn and b == pb * pn:
            out[0] = [n * pn, pa, pb]
        else:
            out.insert(0, [n, a, b])
    return [d[0] for d in out], [d[1] for d in out], [d[2] for d in out]


def _is_row(t, full):
    """``t`` equals the trailing dimensions of ``full`` (after dropping its leading size-1 axes)."""
    ts = tuple(t.shape)
    while ts and ts[0] == 1:
        ts = ts[1:]
    return len(ts) <= len(full) and ts == full[len(full) - len(ts):]


def binary_hip(op, a, b):
    """``a op b`` with NumPy broadcasting on src/kernels/pointwise.hip (same dtype operands).  Equal
    shapes and a row operand repeated along the leading axes run 16-byte vector lanes; any other
    broadcast runs the strided kernel."""
    shape = torch.broadcast_shapes(a.shape, b.shape)
    out = torch.empty(shape, dtype=a.dtype, device=a.device)
    n = out.numel()
    if n == 0:
        return out
    vec = 4 if a.dtype == torch.float32 else 8
    aligned = a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0
    mode, row = 3, 0
    full = tuple(shape)
    if aligned and a.is_contiguous() and b.is_contiguous():
        if tuple(a.shape) == full and tuple(b.shape) == full:
            mode = 0
        elif tuple(a.shape) == full and _is_row(b, full) and b.numel() % vec == 0:
            mode, row = 1, b.numel()
        elif tuple(b.shape) == full and _is_row(a, full) and a.numel() % vec == 0:
            mode, row = 2, a.numel()
    if mode == 3:
        shp, sa, sb = _collapse(list(shape), _bcast_strides(a, shape), _bcast_strides(b, shape))
        if len(shp) > 6:
            return {'add': torch.add, 'sub': torch.sub, 'mul': torch.mul, 'div': torch.div,
                    'maximum': torch.maximum, 'minimum': torch.minimum}[op](a, b)
    else:
        shp, sa, sb = [], [], []
    _K.lib().pointwise_binary(_DT[a.dtype], _PW_OPS[op], a.data_ptr(), b.data_ptr(), out.data_ptr(), n, mode, row,
                              shp, sa, sb, _stream())
    return out


def _sum_to(g, shape):
    if tuple(g.shape) == tuple(shape):
        return g
    return g.sum_to_size(shape) if len(shape) else g.sum()


class BinaryHip(torch.autograd.Function):
    """Broadcast add/sub/mul/div/maximum/minimum: forward and the element-wise parts of the backward
    on the in-tree kernel; broadcast axes of the gradients are reduced with sum_to_size."""

    @staticmethod
    def forward(ctx, a, b, op):
        ctx.op = op
        ctx.sa, ctx.sb = tuple(a.shape), tuple(b.shape)
        if op in ('mul', 'div', 'maximum', 'minimum'):
            ctx.save_for_backward(a, b)
        return binary_hip(op, a, b)

    @staticmethod
    def backward(ctx, g):
        op = ctx.op
        g = g.contiguous()
        if op == 'add':
            return _sum_to(g, ctx.sa), _sum_to(g, ctx.sb), None
        if op == 'sub':
            return _sum_to(g, ctx.sa), _sum_to(-g, ctx.sb), None
        a, b = ctx.saved_tensors
        if op == 'mul':
            return _sum_to(binary_hip('mul', g, b), ctx.sa), _sum_to(binary_hip('mul', g, a), ctx.sb), None
        if op == 'div':
            ga = binary_hip('div', g, b)
            gb = -binary_hip('div', binary_hip('mul', ga, a), b)
            return _sum_to(ga, ctx.sa), _sum_to(gb, ctx.sb), None
        take_a = (a >= b) if op == 'maximum' else (a <= b)
        ga = torch.where(take_a, g, torch.zeros_like(g))
        return _sum_to(ga, ctx.sa), _sum_to(g - ga, ctx.sb), None


def binary_ok(a, b):
    return (a.is_cuda and b.is_cuda and a.dtype == b.dtype and a.dtype in _DT and a.numel() > 0 and
            b.numel() > 0 and a.device == b.device)


__all__ += ['ReluHip', 'relu_ok', 'BinaryHip', 'binary_ok', 'binary_hip']




def flat_sgd(w, g, mom, w32, lr, wd, momentum, rescale, clip, hp=None):
    """Fused (mp-)SGD-momentum over flat arenas (numel % 8 == 0, 16-byte aligned); ``hp`` (optional
    device tensor): hp[0] replaces ``lr`` at run time (graph-captured steps)."""
    lib = _K.lib()
    n = w.numel()
    assert n % 8 == 0 and g.numel() == n and w.dtype == g.dtype and w.dtype in _DT
    assert mom is None or (mom.dtype == torch.float32 and mom.numel() == n)
    assert w32 is None or (w32.dtype == torch.float32 and w32.numel() == n)
    if momentum == 0.0:
        mom = None
    args = (_DT[w.dtype], w.data_ptr(), g.data_ptr(), _p(mom), _p(w32), n, float(lr), float(wd),
            float(momentum), float(rescale), float(clip), _stream())
    lib.flat_sgd(*args) if hp is None else lib.flat_sgd(*args, hp.data_ptr())


# ---------------------------------------------------------------------------
# NHWC implicit-GEMM convolution (src/kernels/conv_igemm.hip)
# ---------------------------------------------------------------------------

import os as _os

_CONV_HIP = _env.get('MXAMD_CONV_HIP') != 0


def conv_ok_shape(x, w, stride, pad, dilate=(1, 1), groups=1):
    """True when the HIP implicit-GEMM forward kernel handles this 2-D conv."""
    return (_CONV_HIP and x.dim() == 4 and w.dim() == 4 and groups == 1 and tuple(dilate) == (1, 1)
            and x.dtype in (torch.float16, torch.bfloat16) and w.dtype == x.dtype
            and x.is_contiguous() and w.is_contiguous() and x.shape[3] % 32 == 0 and w.shape[0] % 64 == 0
            and w.shape[3] == x.shape[3] and x.numel() < 2 ** 31 and x.data_ptr() % 16 == 0
            and w.data_ptr() % 16 == 0)


def stem_ok(x, w, stride, pad, bias=None):
    """True when the few-channel stride-2 stem kernel (src/kernels/conv_stem.hip) handles this conv:
    Cin <= 4, Cout = 64, kernel up to 8x8, stride 2, no bias."""
    return (_CONV_HIP and bias is None and x.dim() == 4 and w.dim() == 4 and x.dtype in (torch.float16, torch.bfloat16)
            and w.dtype == x.dtype and x.is_contiguous() and w.is_contiguous() and 1 <= x.shape[3] <= 4
            and w.shape[3] == x.shape[3] and w.shape[0] == 64 and w.shape[1] <= 8 and w.shape[2] <= 8
            and tuple(stride) == (2, 2) and all(0 <= p < 8 for p in pad) and _K.available()
            and hasattr(_K.lib(), 'conv_stem_fwd'))


def conv_stem_fwd(x, w, pad, bn_stats=False):
    """y[N,Ho,Wo,64] of a stride-2 stem conv on MFMA (conv_stem.hip); ``bn_stats``: also emit the
    BatchNorm sum / sum-of-squares partials of y (``y._mxamd_bn_part``)."""
    N, H, W, C = x.shape
    K, R, S, _ = w.shape
    Ho = (H + 2 * pad[0] - R) // 2 + 1
    Wo = (W + 2 * pad[1] - S) // 2 + 1
    y = torch.empty((N, Ho, Wo, K), dtype=x.dtype, device=x.device)
    lib = _K.lib()
    part, nparts = None, 0
    if bn_stats:
        nparts = 4 * lib.conv_stem_grid(N, H, W, R, S, pad[0], pad[1])
        part = torch.empty(2 * K * nparts, dtype=torch.float32, device=x.device)
    lib.conv_stem_fwd(_DT[x.dtype], x.data_ptr(), w.data_ptr(), y.data_ptr(), N, H, W, C, K, R, S, 2, 2, pad[0],
                      pad[1], _p(part), nparts, _stream())
    if part is not None:
        y._mxamd_bn_part = (part, nparts)
    return y


def conv_stem_wgrad(x, dy, wshape, pad, out=None, accum=False):
    """dW[64,R,S,C] of a stride-2 stem conv: per-workgroup fp32 slabs summed in a fixed order."""
    N, H, W, C = x.shape
    K, R, S, _ = wshape
    dy = dy.contiguous()
    lib = _K.lib()
    slab = torch.empty(lib.conv_stem_wgrad_workspace(N, H, W, R, S, pad[0], pad[1]), dtype=torch.float32,
                       device=x.device)
    if out is None:
        out = torch.empty((K, R, S, C), dtype=x.dtype, device=x.device)
        accum = False
    assert out.is_contiguous() and out.numel() == K * R * S * C and out.dtype in _DT
    lib.conv_stem_wgrad(_DT[x.dtype], x.data_ptr(), dy.data_ptr(), slab.data_ptr(), _DT[out.dtype], out.data_ptr(),
                        int(bool(accum)), N, H, W, C, K, R, S, 2, 2, pad[0], pad[1], _stream())
    return out


# 512-thread big-tile LDS-DMA kernel (conv_big.hip): variant -> (BCO, BPIX)
_BIG_VARIANTS = {10: (256, 256), 11: (128, 256), 12: (64, 512), 13: (256, 128), 14: (128, 256), 15: (256, 128),
                 # the 10..13 tiles on v_mfma_f32_32x32x16 (conv_big.hip MF = 32)
                 16: (256, 256), 17: (128, 256), 18: (64, 512), 19: (256, 128),
                 # 224 / 448-pixel tiles (FJ = 7): fill 7/8 of the CUs on the 14x14 / 28x28 layers
                 26: (256, 224), 27: (128, 448)}
# 14 / 15: the 11 / 13 tiles with a 128-VGPR budget, two workgroups per CU -- only for a single
# K-tile (reduction 64), where one LDS operand stage suffices and the epilogue's HBM streams dominate
_BIG_SKINNY = (14, 15)
# offered to the autotuner only with MXAMD_CONV_SKINNY=1: an A/B on the SSD-512 step measured the
# tree with them 15-20 % slower end to end, so they stay opt-in until that is understood
_SKINNY_ON = os.environ.get('MXAMD_CONV_SKINNY', '0') == '1'
# persistent LDS-DMA ring kernel (conv_ring.hip): variant -> (BCO, BPIX); no bias
_RING_VARIANTS = {20: (128, 128), 21: (256, 128), 22: (128, 256), 23: (64, 256), 24: (256, 256), 25: (64, 128)}


def conv_up2_ok(dy, w, stride, pad, xshape):
    """The 1x1 stride-2 data gradient as one big-tile GEMM pass writing the 2x-upsampled, zero-filled
    dX (conv_big.hip GeomB::up)."""
    K, R, S, C = w.shape
    return (_CONV_HIP and R == 1 and S == 1 and tuple(stride) == (2, 2) and tuple(pad) == (0, 0)
            and dy.dtype in (torch.float16, torch.bfloat16) and dy.is_cuda and dy.dim() == 4 and K % 64 == 0
            and xshape[1] == 2 * dy.shape[1] and xshape[2] == 2 * dy.shape[2] and xshape[3] == C)


def conv_dgrad_up2(dy, w, variant, bn_bwd=None):
    """dX of a 1x1 stride-2 conv: dY . W on the big-tile kernel, each result pixel stored at (2h, 2w) of
    dX and its three 2x2 siblings zeroed by the same epilogue."""
    wt = _dgrad_weight(w.contiguous())          # [C][1][1][K]: the 1x1 weight transposed
    return conv_fwd(dy.contiguous(), wt, (1, 1), (0, 0), None, variant, bn_bwd=bn_bwd, up=2)


def conv_fwd(x, w, stride, pad, bias=None, variant=0, bn_stats=False, addend=None, bn_bwd=None, up=0, dil=(1, 1)):
    """y[N,Ho,Wo,K] = conv(x[N,H,W,C], w[K,R,S,C]) on the MFMA implicit-GEMM kernel.

    ``variant``: 0 = heuristic tile, 1..4 = (BCO, BK) in (128,64) (128,32) (64,64) (64,32),
    5 / 6 = LDS-DMA pipelined kernel with a 128x128 / 64x256 tile (Cin % 64 == 0),
    10..13 = 512-thread LDS-DMA kernel with 256x256 / 128x256 / 64x512 / 256x128 tiles and a
    row-contiguous epilogue, 20..25 = persistent LDS-DMA ring kernel (see _RING_VARIANTS; no bias).
    ``bn_stats`` (big / ring kernels): also emit per-channel BatchNorm
    sum / sum-of-squares partials of y, attached to y as ``y._mxamd_bn_part``; ``addend`` (big kernel
    only, same shape/dtype as y): y = conv + addend.  ``bn_bwd`` (big kernel, or glds 5 / 6 when
    glds_bnb_ok; a BatchNorm's ``_mxamd_bn_src`` record): y is that BN's incoming gradient -- also emit
    its backward statistics (sum dz, sum dz*(z-mean)), attached to y as ``y._mxamd_bn_bwd``.
    ``dil`` (big kernel only, no fused epilogues): dilated taps."""
    N, H, W, C = x.shape
    K, R, S, _ = w.shape
    dil = tuple(dil)
    Ho = (H + 2 * pad[0] - dil[0] * (R - 1) - 1) // stride[0] + 1
    Wo = (W + 2 * pad[1] - dil[1] * (S - 1) - 1) // stride[1] + 1
    assert dil == (1, 1) or (variant in _BIG_VARIANTS and not bn_stats and bn_bwd is None and up == 0), \
        'conv_fwd: dilation runs on the big-tile kernel without fused epilogues'
    assert up in (0, 2) and (up == 0 or (variant in _BIG_VARIANTS and addend is None and not bn_stats))
    y = torch.empty((N, Ho * max(up, 1), Wo * max(up, 1), K), dtype=x.dtype, device=x.device)
    if N * Ho * Wo * K >= 2 ** 31:
        raise ValueError('conv_fwd: output too large for 32-bit indexing')
    b = _f32(bias) if bias is not None else None
    if addend is not None:
        assert variant in _BIG_VARIANTS and addend.shape == y.shape and addend.dtype == y.dtype
        addend = addend.contiguous()
    if variant in _RING_VARIANTS:
        assert bias is None and addend is None, 'conv ring kernel: no bias / addend'
        lib = _K.lib()
        v = variant - 20
        part, nparts = None, 0
        if bn_stats:
            nparts = lib.conv_nhwc_fwd_ring_nparts(N, H, W, R, S, stride[0], stride[1], pad[0], pad[1], v)
            part = torch.empty(2 * K * nparts, dtype=torch.float32, device=x.device)
        lib.conv_nhwc_fwd_ring(_DT[x.dtype], x.data_ptr(), w.data_ptr(), y.data_ptr(), _zero_page(x.device).data_ptr(),
                               N, H, W, C, K, R, S, stride[0], stride[1], pad[0], pad[1], v, _p(part), nparts,
                               _stream())
        if part is not None:
            y._mxamd_bn_part = (part, nparts)
        return y
    if variant in _BIG_VARIANTS:
        lib = _K.lib()
        v = variant - 10
        part, nparts = None, 0
        if bn_stats:
            nparts = lib.conv_nhwc_fwd_big_nparts(N, H, W, R, S, stride[0], stride[1], pad[0], pad[1], v)
            part = torch.empty(2 * K * nparts, dtype=torch.float32, device=x.device)
        bkw = {}
        if bn_bwd is not None:
            z, bmean, bscale, bshift, bmask, bmode, token = bn_bwd
            assert z.shape == y.shape and z.dtype == y.dtype and z.is_contiguous()
            bnp = lib.conv_nhwc_fwd_big_bwd_nparts(N, H, W, R, S, stride[0], stride[1], pad[0], pad[1], v)
            bpart = torch.empty(2 * K * bnp, dtype=torch.float32, device=x.device)
            bkw = dict(bn_z=z.data_ptr(), bn_mean=bmean.data_ptr(), bn_scale=_p(bscale), bn_shift=_p(bshift),
                       bn_mask=_p(bmask), bn_mode=int(bmode), bn_part=bpart.data_ptr(), bn_nparts=bnp)
        lib.conv_nhwc_fwd_big(_DT[x.dtype], x.data_ptr(), w.data_ptr(), _p(b), y.data_ptr(),
                              _zero_page(x.device).data_ptr(), N, H, W, C, K, R, S, stride[0], stride[1],
                              pad[0], pad[1], v, _p(part), nparts, _p(addend), _stream(), up=int(up), dh=dil[0],
                              dw=dil[1], **bkw)
        if bkw:
            # the version pins the statistics to exactly this gradient: when y has several consumers,
            # autograd may accumulate the others' gradients into this tensor in place (bumping its
            # version), and then the partials no longer describe it
            y._mxamd_bn_bwd = (bpart, bnp, bn_bwd[6], y._version)
        if part is not None:
            # consumed by a following BatchNormNHWC (training): its statistics pass over y is skipped
            y._mxamd_bn_part = (part, nparts)
        return y
    if variant in (5, 6):
        lib = _K.lib()
        bco = 128 if variant == 5 else 64
        bkw = _glds_bnb(bn_bwd, y, lib.conv_glds_bwd_nparts(N * Ho * Wo, bco))
        part = bkw.pop('_part', None)
        lib.conv_nhwc_fwd_glds(_DT[x.dtype], x.data_ptr(), w.data_ptr(), _p(b), y.data_ptr(),
                               _zero_page(x.device).data_ptr(), N, H, W, C, K, R, S, stride[0], stride[1],
                               pad[0], pad[1], bco, _stream(), **bkw)
        if part is not None:
            y._mxamd_bn_bwd = (part, bkw['bn_nparts'], bn_bwd[6], y._version)
        return y
    _K.lib().conv_nhwc_fwd(_DT[x.dtype], x.data_ptr(), w.data_ptr(), _p(b), y.data_ptr(), N, H, W, C, K, R, S,
                           stride[0], stride[1], pad[0], pad[1], int(variant), _stream())
    return y


def halo_ok(x, w, stride, pad):
    """True when the halo-tile 3x3 kernel (src/kernels/conv_halo.hip: C = K = 64, stride 1, pad 1)
    takes this NHWC conv."""
    K, R, S, C = w.shape
    return (_CONV_HIP and x.is_cuda and x.dtype in (torch.float16, torch.bfloat16) and x.dim() == 4
            and x.is_contiguous() and w.is_contiguous() and x.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0
            and hasattr(_K.lib(), 'conv3x3_halo')
            and bool(_K.lib().conv3x3_halo_ok(C, K, R, S, stride[0], stride[1], pad[0], pad[1], x.shape[2])))


def conv_halo(x, w, bn_stats=False, bn_bwd=None):
    """y = conv3x3(x, w) (stride 1, pad 1, C = K = 64) on the halo-tile kernel.  ``bn_stats``: BatchNorm
    sum / sum-of-squares partials attached as ``y._mxamd_bn_part`` (one per workgroup); ``bn_bwd`` (a
    BatchNorm's ``_mxamd_bn_src`` record with mode 0 / 2, y being that BN's incoming gradient): its
    backward statistics attached as ``y._mxamd_bn_bwd``."""
    N, H, W, C = x.shape
    K = w.shape[0]
    lib = _K.lib()
    y = torch.empty((N, H, W, K), dtype=x.dtype, device=x.device)
    nparts = lib.conv3x3_halo_nparts(N, H)
    part = torch.empty(2 * K * nparts, dtype=torch.float32, device=x.device) if (bn_stats or bn_bwd) else None
    kw = {}
    if bn_bwd is not None:
        z, bmean, bscale, bshift, _bmask, bmode, _token = bn_bwd
        assert int(bmode) in (0, 2) and z.shape == y.shape and z.dtype == y.dtype and z.is_contiguous()
        kw = dict(bn_z=z.data_ptr(), bn_mean=bmean.data_ptr(), bn_scale=_p(bscale), bn_shift=_p(bshift),
                  bn_mode=int(bmode), bn_part=part.data_ptr())
    lib.conv3x3_halo(_DT[x.dtype], x.data_ptr(), w.data_ptr(), y.data_ptr(), _zero_page(x.device).data_ptr(), N, H,
                     W, C, K, _p(part) if bn_bwd is None else 0, nparts if bn_bwd is None else 0, s=_stream(), **kw)
    if bn_bwd is not None:
        y._mxamd_bn_bwd = (part, nparts, bn_bwd[6], y._version)
    elif part is not None:
        y._mxamd_bn_part = (part, nparts)
    return y


def glds_bnb_ok(bn_src):
    """The LDS-DMA (glds / phase) kernels emit BN-backward statistics for a BN without ReLU or with
    the ReLU mask recomputed from z (modes 0 / 2), not from a stored mask bitmap."""
    return bn_src is not None and int(bn_src[5]) in (0, 2) and hasattr(_K.lib(), 'conv_glds_bwd_nparts')


def _glds_bnb(bn_bwd, y, nparts):
    """Launch keywords of the glds / phase kernels' BN-backward statistics epilogue (and '_part', the
    partials buffer, which the caller attaches to y)."""
    if bn_bwd is None:
        return {}
    z, bmean, bscale, bshift, _bmask, bmode, _token = bn_bwd
    assert int(bmode) in (0, 2) and z.shape == y.shape and z.dtype == y.dtype and z.is_contiguous()
    part = torch.empty(2 * y.shape[-1] * nparts, dtype=torch.float32, device=y.device)
    return dict(bn_z=z.data_ptr(), bn_mean=bmean.data_ptr(), bn_scale=_p(bscale), bn_shift=_p(bshift),
                bn_part=part.data_ptr(), bn_nparts=nparts, _part=part)


_ZERO = {}


def _zero_page(dev):
    """128+ bytes of zeros the LDS-DMA conv kernel reads for halo / out-of-range pixels."""
    z = _ZERO.get(dev)
    if z is None:
        z = _ZERO[dev] = torch.zeros(128, dtype=torch.float16, device=dev)
    return z


def _fwd_variants(C, K, bias=False, ktot=None):
    """Tile variants of conv_fwd valid for Cin=C, Cout=K (``ktot``: the reduction R*S*C).

    1..4: register-staged kernel (conv_igemm.hip) with (BCO, BK) = (128,64) (128,32) (64,64) (64,32);
    5, 6: LDS-DMA kernel (conv_glds.hip) with 128x128 / 64x256 tiles;
    10..15: 512-thread LDS-DMA kernel (conv_big.hip), see _BIG_VARIANTS (14 / 15 only when ktot == 64)."""
    v = []
    if C % 64 == 0 and not bias:
        v.extend(b for b, (bco, _bpix) in sorted(_RING_VARIANTS.items()) if K % bco == 0)
    if C % 64 == 0:
        v.extend(b for b, (bco, _bpix) in sorted(_BIG_VARIANTS.items())
                 if K % bco == 0 and (b not in _BIG_SKINNY or (_SKINNY_ON and ktot == 64)))
    if C % 64 == 0 and K % 128 == 0:
        v.append(5)
    if C % 64 == 0:
        v.append(6)
    if K % 128 == 0 and C % 64 == 0:
        v.append(1)
    if K % 128 == 0:
        v.append(2)
    if C % 64 == 0:
        v.append(3)
    v.append(4)
    return v


def conv_wgrad_ok(x, w):
    """True when the HIP MFMA weight-gradient kernel (src/kernels/conv_wgrad.hip) handles this conv."""
    return (_CONV_HIP and x.dim() == 4 and w.dim() == 4 and x.dtype in (torch.float16, torch.bfloat16)
            and x.is_contiguous() and x.shape[3] % 64 == 0 and w.shape[0] % 64 == 0 and w.shape[3] == x.shape[3]
            and x.numel() < 2 ** 31 and x.data_ptr() % 16 == 0)


def conv_wgrad(x, dy, wshape, stride, pad, out=None, accum=False, dma=True, ring=0, dil=(1, 1)):
    """dW[K,R,S,C] of an NHWC conv on MFMA (split-pixel fp32 slabs + reduce).

    ``out`` (optional, contiguous, f16/bf16/f32) receives the result; with
    ``accum`` the gradient is added to it (e.g. straight into a parameter's grad).
    ``ring`` 1..9: the LDS-DMA ring kernel with that tile (see conv_wgrad.hip), else the planned
    register-staged (``dma=False``) / LDS-DMA kernel.
    """
    N, H, W, C = x.shape
    K, R, S, _ = wshape
    dy = dy.contiguous()
    assert dy.dtype == x.dtype and dy.shape[0] == N and dy.shape[3] == K
    dh, dw = dil
    Ho = (H + 2 * pad[0] - dh * (R - 1) - 1) // stride[0] + 1
    Wo = (W + 2 * pad[1] - dw * (S - 1) - 1) // stride[1] + 1
    assert tuple(dy.shape[1:3]) == (Ho, Wo), 'conv_wgrad: dy shape does not match the conv geometry'
    assert dy.numel() < 2 ** 31 and dy.data_ptr() % 16 == 0
    lib = _K.lib()
    if ring:
        ws = lib.conv_nhwc_wgrad_ring_workspace(N, H, W, C, K, R, S, stride[0], stride[1], pad[0], pad[1], ring,
                                                dh=dh, dw=dw)
    else:
        ws = lib.conv_nhwc_wgrad_workspace(N, H, W, C, K, R, S, stride[0], stride[1], pad[0], pad[1], dh=dh, dw=dw)
    slab = torch.empty(ws, dtype=torch.float32, device=x.device)
    if out is None:
        out = torch.empty((K, R, S, C), dtype=x.dtype, device=x.device)
        accum = False
    assert out.is_contiguous() and out.numel() == K * R * S * C and out.dtype in _DT
    if ring:
        lib.conv_nhwc_wgrad_ring(_DT[x.dtype], x.data_ptr(), dy.data_ptr(), slab.data_ptr(), _DT[out.dtype],
                                 out.data_ptr(), int(bool(accum)), N, H, W, C, K, R, S, stride[0], stride[1], pad[0],
                                 pad[1], _zero_page(x.device).data_ptr(), int(ring), _stream(), dh=dh, dw=dw)
        return out
    lib.conv_nhwc_wgrad(_DT[x.dtype], x.data_ptr(), dy.data_ptr(), slab.data_ptr(), _DT[out.dtype], out.data_ptr(),
                        int(bool(accum)), N, H, W, C, K, R, S, stride[0], stride[1], pad[0], pad[1],
                        _zero_page(x.device).data_ptr() if dma else 0, _stream(), dh=dh, dw=dw)
    return out


def _taps_t(w, out, src, base, rstride):
    """out[base[z] + c*rstride[z] + k] = w[k, tap src[z], c] for every slot z, one launch
    (src/kernels/pointwise.hip weight_taps_t)."""
    K, R, S, C = w.shape
    for i in range(0, len(src), 32):
        _K.lib().weight_taps_t(w.element_size(), w.data_ptr(), out.data_ptr(), K, R * S, C, src[i:i + 32],
                               base[i:i + 32], rstride[i:i + 32], _stream())
    return out


def _dgrad_weight(w):
    """Weight of the equivalent forward conv computing dX from dY (stride 1): [Cin][R][S][Cout], flipped."""
    K, R, S, C = w.shape
    if not (w.is_cuda and w.is_contiguous() and w.element_size() in (2, 4) and _K.available()):
        return w.flip(1, 2).permute(3, 1, 2, 0).contiguous()
    T = R * S
    out = torch.empty((C, R, S, K), dtype=w.dtype, device=w.device)
    return _taps_t(w, out, [T - 1 - t for t in range(T)], [t * K for t in range(T)], [T * K] * T)


def transpose2d(w):
    """w^T of a 2-D [R][C] tensor, contiguous: the LDS-tiled tap-transpose kernel (pointwise.hip) for
    16-bit / fp32 CUDA tensors, else torch's strided copy (several us per weight-sized call on gfx950)."""
    R, C = w.shape
    if w.is_cuda and w.is_contiguous() and w.element_size() in (2, 4) and R % 8 == 0 and C % 8 == 0:
        return _dgrad_weight(w.view(R, 1, 1, C)).view(C, R)
    return w.t().contiguous()


def _phase_taps(R, P, s, ph):
    """Taps of kernel axis R (pad P, stride s) that reach dX positions s*a + ph: [(d, r)] with
    dX[s*a + ph] += dY[a + d] * W[r], d ascending."""
    return sorted(((ph + P - r) // s, r) for r in range(R) if (ph + P - r) % s == 0)


def conv_dgrad_strided_ok(dy, w, stride, pad, xshape, bco=128):
    K, R, S, C = w.shape
    s = tuple(stride)
    return (_CONV_HIP and s != (1, 1) and s[0] == s[1] and s[0] <= 2 and dy.dtype in (torch.float16, torch.bfloat16)
            and dy.dim() == 4 and K % 64 == 0 and C % bco == 0 and xshape[1] % s[0] == 0 and xshape[2] % s[1] == 0
            and dy.is_cuda and all(0 <= p < k for p, k in zip(pad, (R, S))))


_PHASE_PLANS = {}


def _phase_plan(wshape, stride, pad, device):
    """Per (weight shape, stride, pad): the phases with taps [(ph, pw, R_i, S_i, pad_h, pad_w, w_off)], the
    phases no tap reaches, and the tap-transpose table ([(tap, out offset, row stride)], total size) that
    builds every phase's weight slice ([C][R_i][S_i][K], concatenated) from W [K][R][S][C] in one launch."""
    key = (tuple(wshape), tuple(stride), tuple(pad), device)
    plan = _PHASE_PLANS.get(key)
    if plan is not None:
        return plan
    K, R, S, C = wshape
    st = stride[0]
    phases, empty, idx, off = [], [], [], 0
    for ph in range(st):
        th = _phase_taps(R, pad[0], st, ph)
        for pw in range(st):
            tw = _phase_taps(S, pad[1], st, pw)
            if not th or not tw:
                empty.append((ph, pw))
                continue
            dh = [d for d, _ in th]
            dw = [d for d, _ in tw]
            if dh != list(range(dh[0], dh[0] + len(dh))) or dw != list(range(dw[0], dw[0] + len(dw))):
                raise ValueError('conv_dgrad_strided: non-contiguous phase taps')
            # element (c, i, j, k) of the slice <- W[k, rr[i], ss[j], c]: one tap-transpose slot per (i, j)
            nt = len(th) * len(tw)
            for i, (_, r) in enumerate(th):
                for j, (_, c) in enumerate(tw):
                    idx.append((r * S + c, off + (i * len(tw) + j) * K, nt * K))
            phases.append((ph, pw, len(th), len(tw), -dh[0], -dw[0], off))
            off += C * nt * K
    plan = (phases, empty, (idx, off))
    _PHASE_PLANS[key] = plan
    return plan


def conv_dgrad_strided(dy, w, stride, pad, xshape, bco=128, bn_bwd=None):
    """Data gradient of a stride-s conv as s*s sub-pixel phases in one launch (src/kernels/conv_glds.hip
    conv_nhwc_dgrad_phases_glds): phase (ph, pw) of dX -- rows s*a + ph, columns s*b + pw -- is a
    stride-1 conv of dY with the taps of W that reach it, written in place; the first phase's
    epilogue also clears the phases no tap reaches (1x1 stride 2: 3 of 4).  No zero-stuffed dY and no
    scatter pass (cf. the reference's cuDNN backward-data, src/operator/nn/cudnn/cudnn_convolution-inl.h).
    ``bn_bwd`` (glds_bnb_ok): dX is the gradient of that BatchNorm's output -- the epilogue also emits
    its backward statistics, attached as ``dx._mxamd_bn_bwd``."""
    K, R, S, C = w.shape
    N, H, W, _ = xshape
    st = stride[0]
    Ho, Wo = H // st, W // st
    dy = dy.contiguous()
    phases, empty, gidx = _phase_plan(w.shape, stride, pad, w.device)
    if len(phases) > 4:
        raise ValueError('conv_dgrad_strided: at most 4 phases per launch')
    dx = torch.empty((N, H, W, C), dtype=dy.dtype, device=dy.device)
    if len(empty) > 3:
        raise ValueError('conv_dgrad_strided: at most 3 phases without taps')
    slots, total = gidx
    wsub = _taps_t(w.contiguous(), torch.empty(total, dtype=w.dtype, device=w.device), [t[0] for t in slots],
                   [t[1] for t in slots], [t[2] for t in slots])
    cols = list(zip(*phases))
    lib = _K.lib()
    bkw = _glds_bnb(bn_bwd, dx, len(phases) * lib.conv_glds_bwd_nparts(N * Ho * Wo, bco)) if bn_bwd else {}
    part = bkw.pop('_part', None)
    lib.conv_nhwc_dgrad_phases_glds(_DT[dy.dtype], dy.data_ptr(), wsub.data_ptr(), dx.data_ptr(),
                                    _zero_page(dy.device).data_ptr(), N, dy.shape[1], dy.shape[2], K, C, Ho, Wo,
                                    st, list(cols[0]), list(cols[1]), list(cols[2]), list(cols[3]),
                                    list(cols[4]), list(cols[5]), list(cols[6]), [e[0] for e in empty],
                                    [e[1] for e in empty], bco, _stream(), **bkw)
    if part is not None:
        dx._mxamd_bn_bwd = (part, bkw['bn_nparts'], bn_bwd[6], dx._version)
    return dx


def _conv_bwd_torch(dy, x, w, stride, pad, mask):
    xc = x.permute(0, 3, 1, 2)
    wc = w.permute(0, 3, 1, 2)
    dyc = dy.permute(0, 3, 1, 2)
    dx, dw, _ = torch.ops.aten.convolution_backward(dyc, xc, wc, None, list(stride), list(pad), [1, 1], False,
                                                    [0, 0], 1, [mask[0], mask[1], False])
    if dx is not None:
        dx = dx.permute(0, 2, 3, 1)
    if dw is not None:
        dw = dw.permute(0, 2, 3, 1)
    return dx, dw


# ---- algorithm selection (the MXNET_CUDNN_AUTOTUNE_DEFAULT analogue) -------------------------------
# Candidates per conv pass: the in-tree MFMA implicit-GEMM kernel, hipBLASLt
# (torch.mm on the NHWC tensor viewed as a matrix; only 1x1/stride-1, a plain
# library GEMM) and MIOpen.  With autotuning on (default) the first call of
# every (pass, shape, dtype) times each candidate on the live inputs and
# caches the fastest; during HIP-graph capture, or with autotuning off, a
# measured heuristic picks.

_AUTOTUNE = _env.get('MXNET_CUDNN_AUTOTUNE_DEFAULT') > 0
_ALGO = {}
_TIMES = {}   # key -> {candidate: ms per call} from the autotuning run


_REJECTED = {}   # key -> {candidate: relative error} of candidates that failed the numerics check


def _rel_err(a, b):
    a = a.float()
    b = b.float()
    return float((a - b).abs().max() / (b.abs().max() + 1e-6))


_VENDOR = ('mm', 'miopen')
# library candidates under other names: the split-K weight gradients ('splitk<n>' conv, 'sk<n>' FC) are
# hipBLASLt batched GEMMs
_VENDOR_PREFIX = ('splitk', 'blaslt', 'sk')
# near-ties go to the in-tree kernels: a library candidate must be this much faster to be picked
# (3 %: about the run-to-run spread of the timing; 8 % measured 2 % slower on BERT-base, where
# 7 %-slower in-tree weight gradients were picked over hipBLASLt)
_VENDOR_MARGIN = float(os.environ.get('MXAMD_VENDOR_MARGIN', '0.03'))


def _is_vendor(name):
    return name in _VENDOR or name.startswith(_VENDOR_PREFIX)
_TUNE_ROUNDS = int(os.environ.get('MXAMD_TUNE_ROUNDS', '2'))


def _time_candidates(cands, reps=3, key=None, tol=2e-2):
    """Time each candidate and return (fastest name, its output).

    Before timing, every in-tree candidate's output is compared with the vendor
    library's ('mm' / 'miopen', when present) on the live inputs; a candidate
    whose relative max error exceeds ``tol`` is rejected (recorded in
    ``_REJECTED``) so a wrong-but-fast kernel variant can never be selected.
    """
    ref = None
    ref_name = next((n for n, _ in cands if n in ('mm', 'miopen')), None)
    if ref_name is not None:
        ref = dict(cands)[ref_name]()
        if isinstance(ref, torch.Tensor):
            ref = ref.detach().clone()
        else:
            ref = None
    ok = []
    for name, fn in cands:
        if ref is not None and name != ref_name:
            r = fn()
            if isinstance(r, torch.Tensor) and r.shape == ref.shape:
                err = _rel_err(r, ref)
                if not err <= tol:      # also rejects NaN
                    _REJECTED.setdefault(key, {})[name] = err
                    continue
        ok.append((name, fn))
    # interleaved rounds, min per candidate: one slow sample (clock ramp, a neighbour's burst) does
    # not decide the choice
    times, outs = {}, {}
    for _ in range(_TUNE_ROUNDS):
        for name, fn in ok:
            fn()
            t, r = _measure(fn, reps)
            if name not in times or t < times[name]:
                times[name] = t
                outs[name] = r
    # data parallel: every rank must run the same kernels (the slowest rank sets the step time, and
    # ranks that disagree would differ numerically) -- agree on per-candidate times first
    names = [n for n, _ in cands]
    agreed = _agree_times([times.get(n, float('inf')) for n in names])
    best, best_t = None, None
    for name, t in zip(names, agreed):
        if t == float('inf'):
            continue
        if key is not None:
            _TIMES.setdefault(key, {})[name] = t / reps
        if _is_vendor(name):
            t *= 1.0 + _VENDOR_MARGIN     # near-ties (within timing noise) go to the in-tree kernels
        if best_t is None or t < best_t:
            best, best_t = name, t
    if best is not None and best not in outs:
        best = None                         # (cannot happen: a finite agreed time was timed here too)
    return best, (outs[best] if best is not None else None)


def _measure(fn, reps):
    """(ms for ``reps`` calls of ``fn``, last result): HIP events on a GPU, wall clock otherwise."""
    if torch.cuda.is_available():
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            r = fn()
        e.record()
        e.synchronize()
        return s.elapsed_time(e), r
    import time
    t0 = time.perf_counter()
    for _ in range(reps):
        r = fn()
    return (time.perf_counter() - t0) * 1e3, r


def _agree_times(vals):
    """Per-candidate times made identical on every rank: the MAX over ranks (a candidate rejected
    by the numerics check anywhere is out everywhere).  A CPU all-reduce over the gloo side group,
    so no GPU stream or RCCL communicator is touched; every rank autotunes the same keys in the same
    order (one model per rank), which keeps these collectives matched."""
    from ..parallel import dist
    if dist.world_size() <= 1 or not vals:
        return vals
    t = torch.tensor(vals, dtype=torch.float64)
    dist.all_reduce(t, op='max')
    return [float(v) for v in t.tolist()]


# ---- deterministic execution (MXNET_ENFORCE_DETERMINISM; reference: the cuDNN algorithm filter of
# src/operator/nn/cudnn/cudnn_convolution-inl.h:627 and cudnn_pooling-inl.h:53).  The in-tree kernels
# reduce in a fixed order (slab reductions, no float atomics); vendor candidates may pick split-K
# solutions that accumulate with atomics, so in this mode they are only used where no in-tree kernel
# can run, with torch's / MIOpen's deterministic algorithm selection switched on.
_DETERMINISTIC = [_env.get('MXNET_ENFORCE_DETERMINISM') != 0]
_NONDET = ('mm', 'miopen', 'sk', 'splitk', 'bmm', 'blaslt')


def _apply_torch_determinism(flag):
    torch.backends.cudnn.deterministic = bool(flag)
    if flag:
        torch.backends.cudnn.benchmark = False
    try:
        torch.use_deterministic_algorithms(bool(flag), warn_only=True)
    except Exception:   # pylint: disable=broad-except
        pass


def set_deterministic(flag):
    """Switch deterministic execution on or off at run time (the env knob sets the initial state).
    Algorithm choices are cached per mode, so switching does not reuse a nondeterministic choice."""
    _DETERMINISTIC[0] = bool(flag)
    _apply_torch_determinism(flag)


def deterministic():
    return _DETERMINISTIC[0]


if _DETERMINISTIC[0]:
    _apply_torch_determinism(True)


def _det_filter(cands):
    if not _DETERMINISTIC[0] or cands is None:
        return cands
    keep = [(n, f) for n, f in cands if not n.startswith(_NONDET)]
    return keep or cands


def _akey(key):
    """Algorithm-cache key: choices made in deterministic mode are kept apart."""
    return key + ('det',) if _DETERMINISTIC[0] else key


# Persisted tuning table (MXAMD_AUTOTUNE_FILE=path, JSON {repr(key): candidate}): read by every rank at
# first use, so a multi-GPU job whose ranks all load the same file runs identical kernels without
# timing anything; new choices are appended by rank 0.
_FILE_ALGO = {}
_FILE_STATE = {'loaded': False}


def _tuning_file():
    return os.environ.get('MXAMD_AUTOTUNE_FILE', '')


def _load_tuning_file():
    if _FILE_STATE['loaded']:
        return
    _FILE_STATE['loaded'] = True
    path = _tuning_file()
    if path and os.path.exists(path):
        import json
        try:
            with open(path) as f:
                _FILE_ALGO.update(json.load(f))
        except (OSError, ValueError):
            pass


def _save_tuning_file(key, name):
    path = _tuning_file()
    if not path or name is None:
        return
    from ..parallel import dist
    if dist.rank() != 0:
        return
    import json
    _FILE_ALGO[repr(key)] = name
    tmp = path + '.tmp'
    try:
        with open(tmp, 'w') as f:
            json.dump(_FILE_ALGO, f, indent=0, sort_keys=True)
        os.replace(tmp, path)
    except OSError:
        pass


def _select(key, cands, default, timing=None):
    """Run the cached / autotuned / default candidate and return its result.

    ``timing`` (optional, same names as ``cands``): the closures to time instead, e.g. with the
    cost of work a candidate leaves to the next operator included."""
    key = _akey(key)
    cands = _det_filter(cands)
    timing = _det_filter(timing)
    _load_tuning_file()
    name = _ALGO.get(key)
    if name is None:
        name = _FILE_ALGO.get(repr(key))
        if name is not None and name in dict(cands):
            _ALGO[key] = name
    if name is None:
        if _AUTOTUNE and not torch.cuda.is_current_stream_capturing() and len(cands) > 1:
            name, out = _time_candidates(timing or cands, key=key)
            _ALGO[key] = name
            _save_tuning_file(key, name)
            return out
        name = default
    table = dict(cands)
    return (table[name] if name in table else cands[0][1])()


_NCU = {}


def _num_cus(dev):
    n = _NCU.get(dev)
    if n is None:
        n = _NCU[dev] = torch.cuda.get_device_properties(dev).multi_processor_count
    return n


def pw_ok(x, kin, nout):
    """True when the streaming 1x1 kernel (src/kernels/conv_pw.hip) takes a Cin=kin -> Cout=nout conv of
    the NHWC activation ``x``."""
    return (_CONV_HIP and x.is_cuda and x.dtype in (torch.float16, torch.bfloat16) and x.is_contiguous()
            and x.data_ptr() % 16 == 0 and hasattr(_K.lib(), 'conv_pw_stream')
            and bool(_K.lib().conv_pw_stream_ok(int(kin), int(nout))))


def pw_bnb_ok(kin, nout, add, bn_src):
    """True when the streaming 1x1 kernel has a BatchNorm-backward statistics epilogue for this
    (Cin, Cout, addend) and the BN's ReLU mask source (2: from z, 3: forward mask bits)."""
    return (bn_src is not None and int(bn_src[5]) in (2, 3) and hasattr(_K.lib(), 'conv_pw_stream_bnb_ok')
            and bool(_K.lib().conv_pw_stream_bnb_ok(int(kin), int(nout), int(bool(add)), int(bn_src[5]))))


def conv_pw(x, w2, bn_stats=False, addend=None, bn_bwd=None, addend_mask=None):
    """y = x . w2^T (+ addend) for NHWC ``x`` [..., Cin] and ``w2`` [Cout, Cin] on the streaming 1x1
    kernel; ``bn_stats``: BatchNorm sum / sum-of-squares partials in ``y._mxamd_bn_part`` (one per
    workgroup); ``addend`` (the output's shape and dtype) is added in the epilogue.  ``bn_bwd`` (a
    BatchNorm's ``_mxamd_bn_src`` record, y being that BN's incoming gradient): its backward statistics
    (sum dz, sum dz*(z-mean)) from the epilogue, attached as ``y._mxamd_bn_bwd``."""
    C = x.shape[-1]
    K = w2.shape[0]
    M = x.numel() // C
    # a dgrad's w2 is the transpose of a contiguous [Cin][Cout] weight: the kernel transposes it while
    # loading its resident fragments (no per-call transposed copy)
    wt = int(w2.dim() == 2 and w2.stride() == (1, K) and not w2.is_contiguous() and w2.data_ptr() % 16 == 0
             and K % 8 == 0)
    if not wt:
        w2 = w2.contiguous()
    y = torch.empty(x.shape[:-1] + (K,), dtype=x.dtype, device=x.device)
    if addend is not None:
        addend = addend.contiguous()
        if tuple(addend.shape) != tuple(y.shape) or addend.dtype != y.dtype or addend.data_ptr() % 16:
            raise ValueError('conv_pw: addend must match the output (shape, dtype, 16-byte alignment)')
    lib = _K.lib()
    grid = lib.conv_pw_stream_grid(M, C, K, _num_cus(x.device), int(addend is not None or bn_bwd is not None))
    # BatchNorm partials: one per tile walker of a Cout slice (grid / slices per channel)
    nparts = grid // max(1, lib.conv_pw_stream_slices(C, K))
    part = torch.empty(2 * K * nparts, dtype=torch.float32, device=x.device) if (bn_stats or bn_bwd) else None
    bkw = {}
    if bn_bwd is not None:
        assert not bn_stats, 'conv_pw: forward and backward statistics are exclusive'
        z, bmean, bscale, bshift, bmask, bmode, _token = bn_bwd
        assert z.shape == y.shape and z.dtype == y.dtype and z.is_contiguous() and z.data_ptr() % 16 == 0
        bkw = dict(bn_z=z.data_ptr(), bn_mask=_p(bmask), bn_mean=bmean.data_ptr(), bn_scale=_p(bscale),
                   bn_shift=_p(bshift), bn_mode=int(bmode))
    if addend_mask is not None:
        # addend = dy * ReLU bits of a residual tail (its d_addend never materialised: _tee_dgrad)
        assert bn_bwd is not None and addend is not None and addend_mask.dtype == torch.uint8
        assert addend_mask.numel() * 8 == addend.numel() and addend_mask.is_contiguous()
        bkw['addend_mask'] = addend_mask.data_ptr()
    lib.conv_pw_stream(_DT[x.dtype], x.data_ptr(), w2.data_ptr(), y.data_ptr(), _zero_page(x.device).data_ptr(), M, C,
                       K, _p(part), grid, _stream(), _p(addend), wt, **bkw)
    if bn_bwd is not None:
        # pinned to this exact gradient tensor version (see conv_fwd)
        y._mxamd_bn_bwd = (part, nparts, bn_bwd[6], y._version)
    elif part is not None:
        y._mxamd_bn_part = (part, nparts)
    return y


def _fwd_candidates(x, w, stride, pad, bias):
    c = []
    K, R, S, C = w.shape
    if (R == 1 and S == 1 and tuple(stride) == (1, 1) and tuple(pad) == (0, 0) and bias is None
            and pw_ok(x, C, K)):
        c.append(('pw', lambda: conv_pw(x, w.reshape(K, C), bn_stats=bool(_state.STATE.training))))
    if stem_ok(x, w, stride, pad, bias):
        c.append(('stem', lambda: conv_stem_fwd(x, w, pad, bn_stats=bool(_state.STATE.training))))
    if bias is None and halo_ok(x, w, stride, pad):
        c.append(('halo', lambda: conv_halo(x, w, bn_stats=bool(_state.STATE.training))))
    if conv_ok_shape(x, w, stride, pad):
        c.append(('hip', lambda: conv_fwd(x, w, stride, pad, bias)))
        stats = bool(_state.STATE.training)
        for v in _fwd_variants(C, K, bias is not None, ktot=R * S * C):
            c.append(('hip%d' % v, lambda v=v: conv_fwd(x, w, stride, pad, bias, v, bn_stats=stats)))
    if R == 1 and S == 1 and tuple(stride) == (1, 1) and tuple(pad) == (0, 0):
        x2, w2 = x.reshape(-1, C), w.reshape(K, C)
        for name, fn in _gemm().candidates(x2, w2, bias=bias):
            c.append((name, lambda fn=fn: fn().view(x.shape[0], x.shape[1], x.shape[2], K)))

        def mm():
            y = torch.mm(x.reshape(-1, C), w.reshape(K, C).t())
            if bias is not None:
                y = y + bias.to(y.dtype)
            return y.view(x.shape[0], x.shape[1], x.shape[2], K)
        c.append(('mm', mm))

    def miopen():
        y = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), bias, tuple(stride), tuple(pad))
        return y.permute(0, 2, 3, 1).contiguous()
    c.append(('miopen', miopen))
    return c


_STATS_SCRATCH = {}


def _bn_stats_pass(y):
    """The BatchNorm statistics pass over ``y`` (what a following training-mode BN runs itself when
    the conv epilogue did not emit partials)."""
    C = y.shape[-1]
    R = y.numel() // C
    lib = _K.lib()
    n = 2 * lib.bn_partials_rows(R, C) * C
    buf = _STATS_SCRATCH.get(y.device)
    if buf is None or buf.numel() < n:
        buf = _STATS_SCRATCH[y.device] = torch.empty(n, dtype=torch.float32, device=y.device)
    lib.bn_nhwc_stats(_DT[y.dtype], y.data_ptr(), _zeros_f32(C, y.device).data_ptr(), buf.data_ptr(), R, C,
                      _stream())


def _fwd_timing(cands):
    """Timing closures for a training-mode conv feeding BatchNorm: candidates that do not emit BN
    partials from their epilogue are charged the statistics pass the BN then runs over their output."""
    if not _state.STATE.training:
        return None

    def charged(fn):
        def run():
            y = fn()
            if getattr(y, '_mxamd_bn_part', None) is None and y.shape[-1] % 8 == 0 and y.is_contiguous():
                _bn_stats_pass(y)
            return y
        return run
    return [(n, charged(fn)) for n, fn in cands]


def _fwd_default(x, w, stride):
    K, R, S, C = w.shape
    if C <= 4 and K == 64 and tuple(stride) == (2, 2) and R <= 8 and S <= 8:
        return 'stem'
    if R == 1 and S == 1 and tuple(stride) == (1, 1) and (K >= 256 or x.shape[1] * x.shape[2] <= 784):
        return 'mm'
    return 'hip'


def _dgrad_candidates(dy, x, w, stride, pad):
    c = []
    K, R, S, C = w.shape
    if R == 1 and S == 1 and tuple(stride) == (1, 1) and tuple(pad) == (0, 0):
        c.append(('mm', lambda: torch.mm(dy.reshape(-1, K), w.reshape(K, C)).view(x.shape)))
        if pw_ok(dy, K, C):
            c.append(('pw', lambda: conv_pw(dy, w.reshape(K, C).t())))
        c.extend(_gemm_dgrad_1x1(dy, w, x.shape))
    if (tuple(stride) == (1, 1) and C % 64 == 0 and K % 32 == 0 and 2 * pad[0] == R - 1 and 2 * pad[1] == S - 1
            and _CONV_HIP):
        c.append(('hip', lambda: conv_fwd(dy, _dgrad_weight(w), (1, 1), (R - 1 - pad[0], S - 1 - pad[1]))))
        for v in _fwd_variants(K, C, ktot=R * S * K):
            c.append(('hip%d' % v, lambda v=v: conv_fwd(dy, _dgrad_weight(w), (1, 1), (R - 1 - pad[0], S - 1 - pad[1]),
                                                        None, v)))
    for bco in (128, 64):
        if conv_dgrad_strided_ok(dy, w, stride, pad, x.shape, bco):
            c.append(('phase%d' % bco, lambda bco=bco: conv_dgrad_strided(dy, w, stride, pad, x.shape, bco)))
    if halo_ok(dy, w, stride, pad) and tuple(dy.shape) == tuple(x.shape[:3]) + (K,):
        c.append(('halo', lambda: conv_halo(dy, _dgrad_weight(w))))
    if conv_up2_ok(dy, w, stride, pad, x.shape):
        for v, (bco, _bpix) in sorted(_BIG_VARIANTS.items()):
            if C % bco == 0 and v not in _BIG_SKINNY:
                c.append(('up%d' % v, lambda v=v: conv_dgrad_up2(dy, w, v)))
    c.append(('miopen', lambda: _conv_bwd_torch(dy, x, w, stride, pad, (True, False))[0]))
    return c


def _gemm():
    from . import gemm
    return gemm


def _gemm_dgrad_1x1(dy, w, xshape, addend=None):
    """GEMM-kernel candidates for dX = dY . W of a 1x1 stride-1 conv (W^T materialised per call: a
    small copy next to the activation-sized GEMM), optionally + ``addend`` (beta = 1)."""
    K, C = w.shape[0], w.shape[3]
    G = _gemm()
    d2 = dy.reshape(-1, K)
    if not (K % 64 == 0 and C % 64 == 0 and d2.is_cuda and d2.dtype in G._DT and w.dtype == d2.dtype
            and d2.is_contiguous() and d2.data_ptr() % 16 == 0 and _K.available()):
        return []
    out = []
    for cfg in G.configs(d2.shape[0], C, K, G.AUTOTUNE_TILES):
        def run(cfg=cfg):
            add = addend.contiguous().view(-1, C) if addend is not None else None
            return G.gemm_nt(d2, transpose2d(w.reshape(K, C)), addend=add, cfg=cfg).view(xshape)
        out.append(('gemm%ds%d' % cfg, run))
    return out


def _big_algo(key):
    """The big-tile variant number autotuning picked for ``key``, else None."""
    algo = _ALGO.get(_akey(key))
    if algo and algo.startswith('hip') and algo[3:].isdigit() and int(algo[3:]) in _BIG_VARIANTS:
        return int(algo[3:])
    return None


def _bn_bwd_fusable(bn_src, out_shape):
    return bn_src is not None and _BN_BWD_FUSE[0] and tuple(bn_src[0].shape) == tuple(out_shape)


def _charge_bn_bwd(cands, z):
    """Timing closures for a dgrad whose output is the gradient of a BatchNorm(+ReLU) output: a
    candidate without the fused epilogue is charged the backward-statistics pass the BatchNorm then
    runs itself (one read of the gradient and one of the BN input z)."""
    def charged(fn):
        def run():
            r = fn()
            if isinstance(r, torch.Tensor) and r.shape[-1] % 8 == 0 and r.is_contiguous():
                _bn_stats_pass(r)
                _bn_stats_pass(z)
            return r
        return run
    return [(n, charged(fn)) for n, fn in cands]


def _dgrad_bn_candidates(dy, x, w, stride, pad, bn_src):
    """Dgrad candidates when a BatchNorm produced x: the plain candidates plus the kernels whose
    epilogue also emits that BatchNorm's backward statistics ('pw+bn', 'hipN+bn' for the big-tile and
    LDS-DMA stride-1 kernels, 'phaseN+bn' for the strided phase kernel).  Returns
    (candidates, timing closures): autotuning weighs the fused epilogue's extra cost against the
    reduction pass it saves."""
    cands = _dgrad_candidates(dy, x, w, stride, pad)
    K, R, S, C = w.shape
    fused = []
    if (R == 1 and S == 1 and tuple(stride) == (1, 1) and tuple(pad) == (0, 0) and pw_ok(dy, K, C)
            and pw_bnb_ok(K, C, False, bn_src)):
        fused.append(('pw+bn', lambda: conv_pw(dy, w.reshape(K, C).t(), bn_bwd=bn_src)))
    if (_CONV_HIP and tuple(stride) == (1, 1) and 2 * pad[0] == R - 1 and 2 * pad[1] == S - 1
            and K % 64 == 0):
        for v in _fwd_variants(K, C, ktot=R * S * K):
            if v in _BIG_VARIANTS or (v in (5, 6) and glds_bnb_ok(bn_src)):
                fused.append(('hip%d+bn' % v, lambda v=v: conv_fwd(dy, _dgrad_weight(w), (1, 1),
                                                                   (R - 1 - pad[0], S - 1 - pad[1]), None, v,
                                                                   bn_bwd=bn_src)))
    if conv_up2_ok(dy, w, stride, pad, x.shape):
        for v, (bco, _bpix) in sorted(_BIG_VARIANTS.items()):
            if C % bco == 0 and v not in _BIG_SKINNY:
                fused.append(('up%d+bn' % v, lambda v=v: conv_dgrad_up2(dy, w, v, bn_bwd=bn_src)))
    if glds_bnb_ok(bn_src) and halo_ok(dy, w, stride, pad) and tuple(dy.shape) == tuple(x.shape[:3]) + (K,):
        fused.append(('halo+bn', lambda: conv_halo(dy, _dgrad_weight(w), bn_bwd=bn_src)))
    if glds_bnb_ok(bn_src):
        for bco in (128, 64):
            if conv_dgrad_strided_ok(dy, w, stride, pad, x.shape, bco):
                fused.append(('phase%d+bn' % bco, lambda bco=bco: conv_dgrad_strided(dy, w, stride, pad, x.shape, bco,
                                                                                     bn_bwd=bn_src)))
    return cands + fused, _charge_bn_bwd(cands, bn_src[0]) + fused


def _dgrad_default(w, stride):
    K, R, S, C = w.shape
    if tuple(stride) != (1, 1):
        return 'miopen'
    if R == 1 and S == 1:
        return 'mm' if C >= 128 else 'miopen'
    return 'hip' if C >= 128 and C % 64 == 0 else 'miopen'


def _wgrad_candidates(dy, x, w, stride, pad):
    c = [('miopen', lambda: _conv_bwd_torch(dy, x, w, stride, pad, (False, True))[1])]
    K, R, S, C = w.shape
    if stem_ok(x, w, stride, pad):
        c.insert(0, ('stem', lambda: conv_stem_wgrad(x, dy, w.shape, pad)))
    if conv_wgrad_ok(x, w):
        c.insert(0, ('hip', lambda: conv_wgrad(x, dy, w.shape, stride, pad)))
        c.insert(1, ('hipreg', lambda: conv_wgrad(x, dy, w.shape, stride, pad, dma=False)))
        lib = _K.lib()
        for v in range(1, 10):
            if lib.conv_nhwc_wgrad_ring_ok(C, K, R, S, v):
                c.insert(2, ('ring%d' % v, lambda v=v: conv_wgrad(x, dy, w.shape, stride, pad, ring=v)))
    if R == 1 and S == 1 and tuple(stride) == (1, 1) and tuple(pad) == (0, 0):
        P = dy.numel() // K
        for chunks in (16, 64):
            if P % chunks == 0 and P // chunks >= 1024:
                def splitk(chunks=chunks):
                    # fp32 result: the caller accumulates it into the fp16 grad buffer (no cast pass)
                    return _splitk_wgrad(dy, x, chunks)
                c.append(('splitk%d' % chunks, splitk))
    return c


_BMM_OUT_DTYPE = [None]


def _splitk_wgrad(dy, x, chunks, out=None):
    """1x1 wgrad as a split-K batched GEMM (hipBLASLt): [chunks, K, P/chunks] x [chunks, P/chunks, C]
    with fp32 partial products, column-summed by the HIP slab reduce kernel — into a fresh fp32
    dW, or added straight into ``out`` (the weight's fp16/bf16 .grad buffer)."""
    K, C = dy.shape[-1], x.shape[-1]
    P = dy.numel() // K
    d3 = dy.reshape(chunks, P // chunks, K).transpose(1, 2)
    x3 = x.reshape(chunks, P // chunks, C)
    part = _bmm_f32(d3, x3)
    if not part.is_contiguous() or (K * C) % 4:
        r = part.sum(0).view(K, 1, 1, C)
        if out is not None:
            out.add_(r.view(out.shape))
            return None
        return r
    lib = _K.lib()
    if out is None:
        r = torch.empty(K, 1, 1, C, dtype=torch.float32, device=dy.device)
        lib.slab_reduce(0, part.data_ptr(), chunks, K * C, r.data_ptr(), 0, _stream())
        return r
    lib.slab_reduce(_DT[out.dtype], part.data_ptr(), chunks, K * C, out.data_ptr(), 1, _stream())
    return None


def _bmm_f32(a, b):
    """Batched GEMM with fp32 output (fp32 accumulation kept for the split-K sum)."""
    if _BMM_OUT_DTYPE[0] is not False:
        try:
            r = torch.bmm(a, b, out_dtype=torch.float32)
            _BMM_OUT_DTYPE[0] = True
            return r
        except (RuntimeError, TypeError):
            _BMM_OUT_DTYPE[0] = False
    return torch.bmm(a, b).float()


def _wgrad(dy, x, w, w_ref, stride, pad):
    """Weight gradient through the selected algorithm.

    Returns dW, or None when it was accumulated straight into the weight's
    .grad buffer (HIP kernel: its slab-reduce kernel adds into the buffer; the
    split-K GEMM candidates add their fp32 sum into it).
    """
    key = ('wgrad', tuple(x.shape), tuple(w.shape), tuple(stride), tuple(pad), x.dtype)
    algo = _ALGO.get(_akey(key))
    if algo == 'stem':
        tgt = _leaf_grad(w_ref, dtype=w.dtype)
        if tgt is not None:
            conv_stem_wgrad(x, dy, w.shape, pad, out=tgt, accum=True)
            return None
    if algo in ('hip', 'hipreg') or (algo or '').startswith('ring'):
        tgt = _leaf_grad(w_ref, dtype=w.dtype)
        if tgt is not None:
            conv_wgrad(x, dy, w.shape, stride, pad, out=tgt, accum=True, dma=algo == 'hip',
                       ring=int(algo[4:]) if algo.startswith('ring') else 0)
            return None
    elif algo is not None and algo.startswith('splitk'):
        tgt = _leaf_grad(w_ref, dtype=w.dtype)
        if tgt is not None:
            _splitk_wgrad(dy, x, int(algo[6:]), out=tgt)
            return None
    default = 'stem' if stem_ok(x, w, stride, pad) else ('hip' if conv_wgrad_ok(x, w) else 'miopen')
    dw = _select(key, _wgrad_candidates(dy, x, w, stride, pad), default)
    if dw.dtype != w.dtype:
        tgt = _leaf_grad(w_ref, dtype=w.dtype)
        if tgt is not None:
            tgt.add_(dw)          # fp32 split-K sum accumulated straight into the fp16/bf16 grad
            return None
        dw = dw.to(w.dtype)
    return dw


# ---------------------------------------------------------------- weight gradients on a side stream
# The backward of a conv layer is dgrad (feeds the previous BatchNorm's memory-bound backward) and wgrad
# (compute-bound, needed only by the optimizer).  With MXAMD_WGRAD_STREAM=1 the wgrad is issued on a
# per-device side stream forked from the caller's stream, so it runs under the following BatchNorm /
# dgrad kernels instead of in series with them.  Its operands stay referenced until the join, which
# happens at every host-visible point (engine.join_workers: Trainer / KVStore / asnumpy / dispatch),
# before a gradient bucket's all-reduce, and inside a captured HIP graph before the optimizer.
_WGRAD_SIDE = [os.environ.get('MXAMD_WGRAD_STREAM', '0') == '1']
_SIDE_STREAMS = {}
_SIDE_KEEP = []
_SIDE_DIRTY = set()


def join_side_streams():
    """Make each device's current stream wait for the side-stream weight gradients issued so far."""
    if not _SIDE_DIRTY:
        return
    for dev in list(_SIDE_DIRTY):
        torch.cuda.current_stream(dev).wait_stream(_SIDE_STREAMS[dev])
    _SIDE_DIRTY.clear()
    del _SIDE_KEEP[:]


def _wgrad_maybe_side(dy, x, w, w_ref, stride, pad):
    if not (_WGRAD_SIDE[0] and dy.is_cuda):
        return _wgrad(dy, x, w, w_ref, stride, pad)
    dev = dy.device.index
    side = _SIDE_STREAMS.get(dev)
    if side is None:
        side = _SIDE_STREAMS[dev] = torch.cuda.Stream(device=dev)
        from .. import engine
        engine.add_join_hook(join_side_streams)
    main = torch.cuda.current_stream(dev)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        dw = _wgrad(dy, x, w, w_ref, stride, pad)
    _SIDE_KEEP.append((dy, x))
    _SIDE_DIRTY.add(dev)
    if dw is not None:
        # returned to autograd, which consumes it on the caller's stream
        main.wait_stream(side)
        dw.record_stream(main)
    return dw


class ConvNHWC(torch.autograd.Function):
    """2-D NHWC convolution with per-shape algorithm selection (HIP MFMA kernel / hipBLASLt / MIOpen)."""

    @staticmethod
    def forward(ctx, x, w, bias, stride, pad, dilate):
        key = ('fwd', tuple(x.shape), tuple(w.shape), tuple(stride), tuple(pad), x.dtype, bias is not None)
        cands = _fwd_candidates(x, w, stride, pad, bias)
        y = _select(key, cands, _fwd_default(x, w, stride), timing=_fwd_timing(cands))
        ctx.save_for_backward(x, w)
        ctx.stride, ctx.pad = stride, pad
        ctx.has_bias = bias is not None
        ctx.b_ref = bias
        ctx.w_ref = w
        ctx.bn_src = getattr(x, '_mxamd_bn_src', None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        stride, pad = ctx.stride, ctx.pad
        dx = dw = db = None
        if ctx.needs_input_grad[1] and _WGRAD_SIDE[0]:
            # first, so that it overlaps the dgrad and what follows it
            dw = _wgrad_maybe_side(dy, x, w, ctx.w_ref, stride, pad)
        if ctx.needs_input_grad[0]:
            key = ('dgrad', tuple(x.shape), tuple(w.shape), tuple(stride), tuple(pad), x.dtype)
            if _bn_bwd_fusable(ctx.bn_src, x.shape):
                cands, timing = _dgrad_bn_candidates(dy, x, w, stride, pad, ctx.bn_src)
                dx = _select(key + ('bnbwd',), cands, _dgrad_default(w, stride), timing=timing)
            else:
                dx = _select(key, _dgrad_candidates(dy, x, w, stride, pad), _dgrad_default(w, stride))
        if ctx.needs_input_grad[1] and not _WGRAD_SIDE[0]:
            dw = _wgrad(dy, x, w, ctx.w_ref, stride, pad)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = _conv_bias_grad(dy, ctx.b_ref)
        return dx, dw, db, None, None, None


def _conv_bias_grad(dy, b_ref):
    """Bias gradient of an NHWC conv: column sums of dY [N*H*W, K] on the HIP reduce kernels, straight into
    the bias's .grad buffer when it is a leaf (None returned then) -- no fp32 copy of dY."""
    from .nlp_fns import bias_grad
    return bias_grad(dy.reshape(-1, dy.shape[-1]), b_ref, b_ref.dtype)


class ConvTeeNHWC(torch.autograd.Function):
    """1x1 stride-1 NHWC conv whose input also feeds an identity shortcut.

    Returns ``(y, x_passthrough)``.  The shortcut's gradient arrives here with
    the conv's, so dX = dY·W + dShortcut is ONE hipBLASLt GEMM with beta = 1
    (the residual gradient rides in as the C matrix) instead of a dgrad GEMM
    followed by a separate 3-pass elementwise add of two activation-sized
    tensors (what autograd's input-buffer accumulation would launch).
    """

    @staticmethod
    def forward(ctx, x, w, inplace_grad=False):
        stride, pad = (1, 1), (0, 0)
        key = ('fwd', tuple(x.shape), tuple(w.shape), stride, pad, x.dtype, False)
        cands = _fwd_candidates(x, w, stride, pad, None)
        y = _select(key, cands, _fwd_default(x, w, stride), timing=_fwd_timing(cands))
        ctx.save_for_backward(x, w)
        ctx.w_ref = w
        ctx.inplace_grad = inplace_grad
        ctx.bn_src = getattr(x, '_mxamd_bn_src', None)
        xp = x.view_as(x)
        # the passthrough feeds the block's residual tail: its gradient (the tail's dy * ReLU mask) may
        # arrive unmaterialised when this data gradient runs the masked-addend streaming kernel
        xp._mxamd_tee_key = _tee_key(x, w, ctx.bn_src)
        return y, xp

    @staticmethod
    def backward(ctx, gy, gpass):
        x, w = ctx.saved_tensors
        K, C = w.shape[0], w.shape[3]
        dx = dw = None
        if gy is None:
            return gpass, None, None
        gy = gy.contiguous()
        if ctx.needs_input_grad[1] and _WGRAD_SIDE[0]:
            dw = _wgrad_maybe_side(gy, x, w, ctx.w_ref, (1, 1), (0, 0))
        if ctx.needs_input_grad[0]:
            dx = _tee_dgrad(gy, x, w, gpass, ctx.inplace_grad, ctx.bn_src)
        if ctx.needs_input_grad[1] and not _WGRAD_SIDE[0]:
            dw = _wgrad(gy, x, w, ctx.w_ref, (1, 1), (0, 0))
        return dx, dw, None


def _tee_key(x, w, bn_src):
    return ('teedgrad', tuple(x.shape), tuple(w.shape), x.dtype) + (('bnbwd',) if _bn_bwd_fusable(bn_src, x.shape)
                                                                     else ())


_LAZY_DZ = [os.environ.get('MXAMD_LAZY_SHORTCUT_GRAD', '1') != '0']
_LAZY_USED = [0]    # tee data gradients that consumed a lazy shortcut gradient (tests)


def lazy_shortcut_ok(tee_key):
    """Whether a residual tail may hand its shortcut gradient dz = dy * mask to the tee data gradient
    unmaterialised: only once that data gradient is known to run the masked-addend streaming kernel."""
    return _LAZY_DZ[0] and tee_key is not None and _ALGO.get(_akey(tee_key)) == 'pw+bn'


def _unpack_lazy_dz(gpass):
    """(dy, mask) of a lazy shortcut gradient (see BatchNormNHWC.backward), or None."""
    lz = getattr(gpass, '_mxamd_lazy_mask', None) if gpass is not None else None
    if lz is None or lz[1] != gpass._version:
        return None
    return lz[0]


def _materialize_dz(gpass, mask):
    """dy * mask bits (the fallback when the chosen data gradient cannot take the masked addend)."""
    bits = (mask.view(-1, 1) >> torch.arange(8, device=mask.device, dtype=torch.uint8)) & 1
    return gpass * bits.view(gpass.shape).to(gpass.dtype)


def _tee_dgrad(gy, x, w, gpass, inplace, bn_src=None):
    """dX = dY . W (+ dShortcut) of a 1x1 stride-1 conv: the in-tree big-tile MFMA kernel with the
    shortcut gradient read in its epilogue (beta = 1), or hipBLASLt addmm -- autotuned per shape.
    A lazy dShortcut (the residual tail's dy with its ReLU mask, never multiplied out) goes to the
    streaming kernel's masked-addend stage."""
    K, C = w.shape[0], w.shape[3]
    g2 = gy.reshape(-1, K)
    w2 = w.reshape(K, C)
    amask = _unpack_lazy_dz(gpass)
    if amask is not None:
        key = _tee_key(x, w, bn_src)
        if (_ALGO.get(_akey(key)) == 'pw+bn' and _bn_bwd_fusable(bn_src, x.shape) and pw_ok(gy, K, C)
                and pw_bnb_ok(K, C, True, bn_src) and gpass.is_contiguous() and gpass.data_ptr() % 16 == 0):
            _LAZY_USED[0] += 1
            return conv_pw(gy, w2.t(), addend=gpass, bn_bwd=bn_src, addend_mask=amask)
        gpass, inplace = _materialize_dz(gpass, amask), True

    def mm():
        if gpass is not None and inplace and gpass.is_contiguous():
            # the shortcut's gradient buffer is private to this edge (the fused residual tail
            # returns a fresh d_addend): accumulate the GEMM into it, beta = 1, no copy
            return gpass.view(-1, C).addmm_(g2, w2).view(x.shape)
        if gpass is not None:
            return torch.addmm(gpass.contiguous().reshape(-1, C), g2, w2).view(x.shape)
        return torch.mm(g2, w2).view(x.shape)

    cands = []
    fused = []
    fuse_bn = _bn_bwd_fusable(bn_src, x.shape)
    if _CONV_HIP and K % 64 == 0 and gy.dtype in (torch.float16, torch.bfloat16) and gy.numel() < 2 ** 31:
        wt = None
        for v, (bco, _bpix) in sorted(_BIG_VARIANTS.items()):
            if C % bco or (v in _BIG_SKINNY and not (_SKINNY_ON and K == 64)):
                continue
            if wt is None:
                # W^T [C][1][1][K] on the LDS-tiled tap-transpose kernel (torch's strided transpose copy
                # cost ~6 us per call here)
                wt = _dgrad_weight(w.contiguous())

            def big(v=v, wt=wt, bn=None):
                add = gpass.contiguous() if gpass is not None else None
                return conv_fwd(gy, wt, (1, 1), (0, 0), None, v, addend=add, bn_bwd=bn)
            cands.append(('hip%d' % v, big))
            if fuse_bn:
                # the block input's BatchNorm (the previous block's residual tail) gets its backward
                # statistics from this dgrad's epilogue
                fused.append(('hip%d+bn' % v, lambda big=big: big(bn=bn_src)))
    cands.extend(_gemm_dgrad_1x1(gy, w, x.shape, addend=gpass))
    if pw_ok(gy, K, C) and (gpass is None or (gpass.is_contiguous() and gpass.data_ptr() % 16 == 0)):
        # streaming 1x1 kernel: small reductions (K <= 512) are memory-bound; the shortcut gradient
        # is added in its epilogue
        cands.append(('pw', lambda: conv_pw(gy, w2.t(), addend=gpass)))
        if fuse_bn and gpass is not None and pw_bnb_ok(K, C, True, bn_src):
            fused.append(('pw+bn', lambda: conv_pw(gy, w2.t(), addend=gpass, bn_bwd=bn_src)))
    # autotuning runs every candidate: use an out-of-place GEMM there (the in-place one would
    # accumulate into gpass once per timing repetition)
    cands.append(('mm', lambda: mm() if not (gpass is not None and inplace) else
                  torch.addmm(gpass.reshape(-1, C), g2, w2).view(x.shape)))
    key = ('teedgrad', tuple(x.shape), tuple(w.shape), x.dtype) + (('bnbwd',) if fuse_bn else ())
    if _ALGO.get(_akey(key)) == 'mm':
        return mm()
    if fuse_bn:
        return _select(key, cands + fused, 'mm', timing=_charge_bn_bwd(cands, bn_src[0]) + fused)
    return _select(key, cands, 'mm')


def conv_tee_ok(x, w):
    return (conv_ok(x, w, (1, 1), (0, 0), (1, 1), 1) and w.shape[1] == 1 and w.shape[2] == 1
            and x.shape[3] == w.shape[3])




def conv_algos():
    """The algorithm chosen for every (pass, shape) seen so far."""
    return dict(_ALGO)


def conv_algo_times():
    """Autotuning measurements: (pass, shape...) -> {candidate: ms}."""
    return {k: dict(v) for k, v in _TIMES.items()}


def _conv_bwd_dil_torch(dy, x, w, stride, pad, dil, mask):
    """MIOpen (through aten) gradients of a dilated NHWC conv: (dx, dw) per ``mask``."""
    r = torch.ops.aten.convolution_backward(dy.permute(0, 3, 1, 2), x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2),
                                            None, tuple(stride), tuple(pad), tuple(dil), False, (0, 0), 1,
                                            (mask[0], mask[1], False))
    return (r[0].permute(0, 2, 3, 1).contiguous() if mask[0] else None,
            r[1].permute(0, 2, 3, 1).contiguous() if mask[1] else None)


def dil_ok(x, w, dilate):
    """Dilated NHWC convs (DeepLab atrous layers) on the big-tile forward / data-gradient kernels and
    the MFMA weight-gradient kernels."""
    K, R, S, C = w.shape
    return (_CONV_HIP and tuple(dilate) != (1, 1) and C % 64 == 0 and K % 64 == 0 and x.is_contiguous()
            and x.dtype in (torch.float16, torch.bfloat16) and x.numel() < 2 ** 31)


class ConvDilNHWC(torch.autograd.Function):
    """Dilated 2-D NHWC convolution: forward on conv_big.hip with dilated taps; data gradient (stride 1)
    = the same kernel over dY with the flipped weight, dilation d and padding d*(R-1) - p; weight
    gradient on conv_wgrad.hip with dilated taps; each pass timed against MIOpen per shape (reference:
    the dilate parameter of src/operator/nn/convolution-inl.h)."""

    @staticmethod
    def forward(ctx, x, w, bias, stride, pad, dilate):
        K, R, S, C = w.shape
        key = ('fwd-dil', tuple(x.shape), tuple(w.shape), tuple(stride), tuple(pad), tuple(dilate), x.dtype,
               bias is not None)
        cands = [('hip%d' % v, lambda v=v: conv_fwd(x, w, stride, pad, bias, v, dil=dilate))
                 for v, (bco, _bpix) in sorted(_BIG_VARIANTS.items()) if K % bco == 0 and v not in _BIG_SKINNY]

        def miopen():
            y = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), bias, tuple(stride),
                                           tuple(pad), tuple(dilate))
            return y.permute(0, 2, 3, 1).contiguous()
        cands.append(('miopen', miopen))
        y = _select(key, cands, cands[0][0])
        ctx.save_for_backward(x, w)
        ctx.cfg = (tuple(stride), tuple(pad), tuple(dilate))
        ctx.has_bias = bias is not None
        ctx.b_ref = bias
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        stride, pad, dil = ctx.cfg
        dy = dy.contiguous()
        K, R, S, C = w.shape
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            key = ('dgrad-dil', tuple(x.shape), tuple(w.shape), stride, pad, dil, x.dtype)
            cands = []
            pp = (dil[0] * (R - 1) - pad[0], dil[1] * (S - 1) - pad[1])
            if stride == (1, 1) and pp[0] >= 0 and pp[1] >= 0:
                cands = [('hip%d' % v, lambda v=v: conv_fwd(dy, _dgrad_weight(w), (1, 1), pp, None, v, dil=dil))
                         for v, (bco, _bpix) in sorted(_BIG_VARIANTS.items())
                         if C % bco == 0 and v not in _BIG_SKINNY]
            cands.append(('miopen', lambda: _conv_bwd_dil_torch(dy, x, w, stride, pad, dil, (True, False))[0]))
            dx = _select(key, cands, cands[0][0])
        if ctx.needs_input_grad[1]:
            key = ('wgrad-dil', tuple(x.shape), tuple(w.shape), stride, pad, dil, x.dtype)
            cands = []
            if conv_wgrad_ok(x, w):
                cands.append(('hip', lambda: conv_wgrad(x, dy, w.shape, stride, pad, dil=dil)))
                lib = _K.lib()
                for v in range(1, 10):
                    if lib.conv_nhwc_wgrad_ring_ok(C, K, R, S, v):
                        cands.append(('ring%d' % v, lambda v=v: conv_wgrad(x, dy, w.shape, stride, pad, ring=v,
                                                                          dil=dil)))
            cands.append(('miopen', lambda: _conv_bwd_dil_torch(dy, x, w, stride, pad, dil, (False, True))[1]))
            dw = _select(key, cands, cands[0][0]).to(w.dtype)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = _conv_bias_grad(dy, ctx.b_ref)
        return dx, dw, db, None, None, None


_KPAD = _os.environ.get('MXAMD_CONV_KPAD', '1') == '1'


def kpad_ok(x, w):
    """Output channels that do not tile the MFMA kernels (detection heads: anchors x (classes + 1),
    deformable offsets: 2 x taps) with input channels that do."""
    return _KPAD and w.shape[0] % 64 != 0 and w.shape[3] % 64 == 0 and w.shape[0] >= 8


def conv_kpad(x, w, bias, stride, pad, dilate):
    """NHWC conv with the output channels zero-padded to a multiple of 64, so the forward, data and
    weight gradients run on the in-tree MFMA kernels instead of MIOpen; the result is the first
    ``K`` channels (a strided view), the padding's gradients are dropped by autograd."""
    K = w.shape[0]
    Kp = (K + 63) // 64 * 64
    wp = torch.nn.functional.pad(w, (0, 0, 0, 0, 0, 0, 0, Kp - K))
    bp = None if bias is None else torch.nn.functional.pad(bias, (0, Kp - K))
    return ConvNHWC.apply(x, wp, bp, tuple(stride), tuple(pad), tuple(dilate))[..., :K]


def conv_ok(x, w, stride, pad, dilate, groups):
    # any 2-D fp16/bf16 NHWC conv goes through ConvNHWC's algorithm selection
    return (len(stride) == 2 and x.dim() == 4 and groups == 1 and tuple(dilate) == (1, 1) and x.is_contiguous()
            and w.is_contiguous() and x.dtype in (torch.float16, torch.bfloat16) and w.dtype == x.dtype)


__all__ += ['ConvNHWC', 'ConvTeeNHWC', 'ConvDilNHWC', 'dil_ok', 'conv_kpad', 'kpad_ok', 'conv_fwd', 'conv_ok_shape', 'conv_wgrad', 'conv_wgrad_ok', 'stem_ok',
            'conv_stem_fwd', 'conv_stem_wgrad']


# ---------------------------------------------------------------------------
# NHWC pooling (src/kernels/pool_nhwc.hip)
# ---------------------------------------------------------------------------

def _pool_out(n, k, s, p, full):
    # MXNet: valid = floor, full = ceil (src/operator/nn/pooling-inl.h), no window clipping
    if full:
        return -(-(n + 2 * p - k) // s) + 1
    return (n + 2 * p - k) // s + 1


def pool_ok(x, kernel, stride, pad):
    return (x.dim() == 4 and x.dtype in _DT and x.is_contiguous() and x.shape[3] % 8 == 0 and x.numel() > 0
            and min(x.shape[1] + 2 * pad[0] - kernel[0], x.shape[2] + 2 * pad[1] - kernel[1]) >= 0
            and len(kernel) == 2 and kernel[0] * kernel[1] <= 256 and x.data_ptr() % 16 == 0
            and all(p < k for p, k in zip(pad, kernel)))


class PoolNHWC(torch.autograd.Function):
    """Max/avg 2-D pooling on NHWC tensors (max keeps a uint8 argmax per element)."""

    @staticmethod
    def forward(ctx, x, pool_type, kernel, stride, pad, full, count_include_pad):
        N, H, W, C = x.shape
        Ho = _pool_out(H, kernel[0], stride[0], pad[0], full)
        Wo = _pool_out(W, kernel[1], stride[1], pad[1], full)
        is_max = pool_type == 'max'
        y = torch.empty((N, Ho, Wo, C), dtype=x.dtype, device=x.device)
        arg = torch.empty((N, Ho, Wo, C), dtype=torch.uint8, device=x.device) if is_max else None
        geo = (N, H, W, C, Ho, Wo, kernel[0], kernel[1], stride[0], stride[1], pad[0], pad[1],
               int(bool(count_include_pad)))
        _K.lib().pool_nhwc_forward(_DT[x.dtype], int(is_max), x.data_ptr(), y.data_ptr(), _p(arg), *geo, _stream())
        ctx.geo, ctx.is_max, ctx.dt = geo, is_max, x.dtype
        if is_max:
            ctx.save_for_backward(arg)
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        geo = ctx.geo
        arg = ctx.saved_tensors[0] if ctx.is_max else None
        dx = torch.empty((geo[0], geo[1], geo[2], geo[3]), dtype=ctx.dt, device=dy.device)
        _K.lib().pool_nhwc_backward(_DT[ctx.dt], int(ctx.is_max), dy.data_ptr(), _p(arg), dx.data_ptr(), *geo,
                                    _stream())
        return dx, None, None, None, None, None, None


__all__ += ['PoolNHWC']
