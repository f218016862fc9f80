"""torch.autograd wrappers around the gfx950 HIP kernels.

Each wrapper validates shapes/dtypes/contiguity on the host (the kernels assume
them), allocates outputs with the torch caching allocator and launches on the
current HIP stream.  Numerics are checked against fp32 torch references in
tests/test_hip_kernels.py.
"""
import torch

from . import kernels as _K

__all__ = ['BatchNormNHWC', 'SoftmaxCE', 'GlobalAvgPoolNHWC', 'flat_sgd']

_DT = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _p(t):
    return 0 if t is None else t.data_ptr()


def _f32(t):
    return t if t.dtype == torch.float32 and t.is_contiguous() else t.float().contiguous()


# ---------------------------------------------------------------------------
# predicates (override the conservative defaults in kernels.py)
# ---------------------------------------------------------------------------

def bn_ok(x):
    return (x.dtype in _DT and x.dim() >= 2 and x.is_contiguous() and x.shape[-1] % 8 == 0
            and x.numel() > 0 and x.data_ptr() % 16 == 0)


def ce_ok(x):
    return x.dim() == 2 and x.dtype in _DT and x.is_contiguous()


_K.bn_ok = bn_ok
_K.ce_ok = ce_ok


class BatchNormNHWC(torch.autograd.Function):
    """BatchNorm over the last (channel) axis with optional fused residual add + ReLU."""

    @staticmethod
    def forward(ctx, x, gamma, beta, addend, eps, training, relu, moving_mean, moving_var, momentum=None):
        lib = _K.lib()
        C = x.shape[-1]
        R = x.numel() // C
        dev = x.device
        g = _f32(gamma)
        b = _f32(beta)
        mm = _f32(moving_mean)
        y = torch.empty_like(x)
        if addend is not None:
            assert addend.shape == x.shape and addend.dtype == x.dtype
            addend = addend.contiguous()
        if training:
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
        lib.bn_nhwc_forward(_DT[x.dtype], x.data_ptr(), _p(addend), y.data_ptr(), g.data_ptr(), b.data_ptr(),
                            mm.data_ptr(), _p(part), mean.data_ptr(), invstd.data_ptr(), var.data_ptr(),
                            scale.data_ptr(), shift.data_ptr(), R, C, float(eps), int(bool(training)),
                            int(bool(relu)), 0, float(momentum or 0.0), moving_mean.data_ptr() if upd else 0,
                            moving_var.data_ptr() if upd else 0, _stream())
        if training and momentum is not None and not upd:
            with torch.no_grad():
                moving_mean.mul_(momentum).add_(mean.to(moving_mean.dtype), alpha=1 - momentum)
                moving_var.mul_(momentum).add_(var.to(moving_var.dtype), alpha=1 - momentum)
        ctx.save_for_backward(x, y if relu else None, g, mean, invstd)
        ctx.cfg = (bool(relu), bool(training), addend is not None, gamma.dtype, beta.dtype)
        ctx.mark_non_differentiable(mean, var)
        return y, mean, var

    @staticmethod
    def backward(ctx, gy, _gm, _gv):
        lib = _K.lib()
        x, y, g, mean, invstd = ctx.saved_tensors
        relu, training, has_add, gdt, bdt = ctx.cfg
        gy = gy.contiguous()
        C = x.shape[-1]
        R = x.numel() // C
        dev = x.device
        dx = torch.empty_like(x)
        dz = torch.empty_like(x) if has_add else None
        nblk = lib.bn_partials_rows(R, C)
        part = torch.empty(2 * nblk * C, dtype=torch.float32, device=dev)
        out = torch.empty(5, C, dtype=torch.float32, device=dev)
        lib.bn_nhwc_backward(_DT[x.dtype], x.data_ptr(), gy.data_ptr(), _p(y), dx.data_ptr(), _p(dz), g.data_ptr(),
                             mean.data_ptr(), invstd.data_ptr(), part.data_ptr(), out[0].data_ptr(),
                             out[1].data_ptr(), out[2].data_ptr(), R, C, int(relu), 0, int(training), _stream())
        dgamma = out[0].to(gdt) if ctx.needs_input_grad[1] else None
        dbeta = out[1].to(bdt) if ctx.needs_input_grad[2] else None
        return dx, dgamma, dbeta, dz, None, None, None, None, None, None


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


_K.gap_ok = gap_ok


def flat_sgd(w, g, mom, w32, lr, wd, momentum, rescale, clip):
    """Fused (mp-)SGD-momentum over flat arenas (numel % 8 == 0, 16-byte aligned)."""
    lib = _K.lib()
    n = w.numel()
    assert n % 8 == 0 and g.numel() == n and w.dtype == g.dtype and w.dtype in _DT
    assert mom is None or (mom.dtype == torch.float32 and mom.numel() == n)
    assert w32 is None or (w32.dtype == torch.float32 and w32.numel() == n)
    if momentum == 0.0:
        mom = None
    lib.flat_sgd(_DT[w.dtype], w.data_ptr(), g.data_ptr(), _p(mom), _p(w32), n, float(lr), float(wd),
                 float(momentum), float(rescale), float(clip), _stream())
