"""torch.autograd wrappers for the transformer-path gfx950 kernels (src/kernels/nlp_kernels.hip)
and the fused flat-arena optimizer kernels (src/kernels/optim_kernels.hip).

LayerNorm (fwd/bwd with dgamma/dbeta straight into the parameters' fp32 grad
buffers), erf-GELU, last-axis softmax / log_softmax (with temperature) and
Philox dropout with a 1-bit mask.  Numerics vs fp32 torch references:
tests/test_hip_kernels.py.
"""
import torch

from . import kernels as _K
from .. import _state
from .kernel_fns import _DT, _stream, _p, _f32, _leaf_grad

__all__ = ['LayerNorm', 'AddDropoutLN', 'GELU', 'Softmax', 'Dropout', 'ln_ok', 'ew_ok', 'softmax_ok',
           'flat_adam', 'lamb_update', 'seg_sumsq', 'all_finite', 'ChunkTable']


def _aligned(t):
    return t.is_contiguous() and t.data_ptr() % 16 == 0


def ln_ok(x):
    return x.dtype in _DT and x.dim() >= 2 and _aligned(x) and x.shape[-1] % 8 == 0 and 8 <= x.shape[-1] <= 4096


def ew_ok(x):
    return x.dtype in _DT and _aligned(x) and x.numel() % 8 == 0 and x.numel() > 0


def softmax_ok(x, axis):
    return (x.dtype in _DT and x.dim() >= 1 and axis % x.dim() == x.dim() - 1 and _aligned(x)
            and x.shape[-1] % 8 == 0 and 8 <= x.shape[-1] <= 8192 and x.numel() > 0)




class LayerNorm(torch.autograd.Function):
    """y = (x - mean) / sqrt(var + eps) * gamma + beta over the last axis; returns (y, mean, std)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, eps, want_stats=True):
        lib = _K.lib()
        D = x.shape[-1]
        M = x.numel() // D
        # gamma/beta in the activation dtype are read as they are (no conversion kernels per call)
        pt = int(gamma.dtype == x.dtype and beta.dtype == x.dtype and gamma.is_contiguous() and beta.is_contiguous()
                 and gamma.data_ptr() % 16 == 0 and beta.data_ptr() % 16 == 0)
        g = gamma if pt else _f32(gamma)
        b = beta if pt else _f32(beta)
        y = torch.empty_like(x)
        stats = torch.empty(2, M, dtype=torch.float32, device=x.device)
        mean, rstd = stats[0], stats[1]
        lib.layernorm_forward(_DT[x.dtype], x.data_ptr(), g.data_ptr(), b.data_ptr(), y.data_ptr(), mean.data_ptr(),
                              rstd.data_ptr(), M, D, float(eps), _stream(), pt=pt)
        ctx.save_for_backward(x, g, mean, rstd)
        ctx.pt = pt
        ctx.refs = (gamma, beta)
        shp = tuple(x.shape[:-1]) + (1,)
        if want_stats:
            m_out = mean.view(shp).to(x.dtype)
            s_out = torch.reciprocal(rstd).view(shp).to(x.dtype)     # std = sqrt(var + eps)
        else:
            # hidden outputs (output_mean_var=False): fp32 views, no conversion kernels
            m_out, s_out = mean.view(shp), rstd.view(shp)
        ctx.mark_non_differentiable(m_out, s_out)
        ctx.set_materialize_grads(False)
        return y, m_out, s_out

    @staticmethod
    def backward(ctx, gy, _gm, _gs):
        if gy is None:
            return None, None, None, None, None
        lib = _K.lib()
        x, g, mean, rstd = ctx.saved_tensors
        gamma, beta = ctx.refs
        gy = gy.contiguous()
        D = x.shape[-1]
        M = x.numel() // D
        dx = torch.empty_like(x)
        nb = lib.layernorm_bwd_partials(M)
        part = torch.empty(nb * 2 * D, dtype=torch.float32, device=x.device)
        need_g, need_b = ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        # accumulate straight into the parameters' gradient buffers, in their dtype (no conversion/add kernels)
        same = gamma.dtype == beta.dtype and gamma.dtype in _DT
        tg = _leaf_grad(gamma, D, dtype=gamma.dtype) if (need_g and same) else None
        tb = _leaf_grad(beta, D, dtype=beta.dtype) if (need_b and same) else None
        if tg is not None and tb is not None:
            dg, db, accum, gdt = tg, tb, 1, _DT[gamma.dtype]
        else:
            out = torch.empty(2, D, dtype=torch.float32, device=x.device)
            dg, db, accum, gdt = out[0], out[1], 0, _DT[torch.float32]
        lib.layernorm_backward(_DT[x.dtype], x.data_ptr(), gy.data_ptr(), g.data_ptr(), mean.data_ptr(),
                               rstd.data_ptr(), dx.data_ptr(), part.data_ptr(), dg.data_ptr(), db.data_ptr(), gdt,
                               accum, M, D, _stream(), pt=ctx.pt)
        if accum:
            return dx, None, None, None, None
        return (dx, dg.view(gamma.shape).to(gamma.dtype) if need_g else None,
                db.view(beta.shape).to(beta.dtype) if need_b else None, None, None)


# residual-gradient handoff to the Dense data gradient and bias gradients from the fused LayerNorm
# backward's partials (MXAMD_RESIDUAL_HANDOFF=0: autograd accumulation and separate column sums, for A/B)
_HANDOFF = __import__('os').environ.get('MXAMD_RESIDUAL_HANDOFF', '1') == '1'


class AddDropoutLN(torch.autograd.Function):
    """y = LayerNorm(x + dropout_p(h)) over the last axis in one kernel (the post-LN transformer
    sub-layer tail); backward: the residual gradient, the dropout-masked branch gradient and
    dgamma / dbeta in one kernel."""

    @staticmethod
    def forward(ctx, x, h, gamma, beta, eps, p, handoff=False):
        lib = _K.lib()
        D = x.shape[-1]
        M = x.numel() // D
        # handoff: x also feeds a FullyConnected (Linear below) whose backward runs after this one (a
        # transformer sub-layer: x -> Dense -> ... -> h); the residual gradient is then added by that
        # layer's data-gradient GEMM (addend) instead of by a separate autograd accumulation
        ctx.res_src = x if (handoff and _HANDOFF and getattr(x, '_mxamd_fc_input', False)) else None
        pt = int(gamma.dtype == x.dtype and beta.dtype == x.dtype and gamma.is_contiguous() and beta.is_contiguous()
                 and gamma.data_ptr() % 16 == 0 and beta.data_ptr() % 16 == 0)
        g = gamma if pt else _f32(gamma)
        b = beta if pt else _f32(beta)
        y = torch.empty_like(x)
        sm = torch.empty_like(x)
        stats = torch.empty(2, M, dtype=torch.float32, device=x.device)
        mask = torch.empty(x.numel() // 8, dtype=torch.uint8, device=x.device) if p > 0 else None
        ctr = _state.GRAPH_RNG[0]
        base = ctr.data_ptr() if (p > 0 and ctr is not None and torch.cuda.is_current_stream_capturing()) else 0
        lib.add_dropout_ln_forward(_DT[x.dtype], x.data_ptr(), h.data_ptr(), g.data_ptr(), b.data_ptr(), pt,
                                   y.data_ptr(), sm.data_ptr(), _p(mask), stats[0].data_ptr(), stats[1].data_ptr(),
                                   M, D, float(eps), float(p), _seed() if p > 0 else 0, base, _stream())
        ctx.save_for_backward(sm, g, stats, mask)
        ctx.cfg = (pt, float(p))
        ctx.refs = (gamma, beta)
        return y

    @staticmethod
    def backward(ctx, gy):
        lib = _K.lib()
        sm, g, stats, mask = ctx.saved_tensors
        pt, p = ctx.cfg
        gamma, beta = ctx.refs
        gy = gy.contiguous()
        D = sm.shape[-1]
        M = sm.numel() // D
        ds = torch.empty_like(sm)
        dh = torch.empty_like(sm)
        nb = lib.layernorm_bwd_partials(M)
        part = torch.empty(nb * 2 * D, dtype=torch.float32, device=sm.device)
        need_g, need_b = ctx.needs_input_grad[2], ctx.needs_input_grad[3]
        same = gamma.dtype == beta.dtype and gamma.dtype in _DT
        tg = _leaf_grad(gamma, D, dtype=gamma.dtype) if (need_g and same) else None
        tb = _leaf_grad(beta, D, dtype=beta.dtype) if (need_b and same) else None
        if tg is not None and tb is not None:
            dg, db, accum, gdt = tg, tb, 1, _DT[gamma.dtype]
        else:
            out = torch.empty(2, D, dtype=torch.float32, device=sm.device)
            dg, db, accum, gdt = out[0], out[1], 0, _DT[torch.float32]
        # column sums of dh (partials per block): the bias gradient of the Linear that produced h
        hpart = torch.empty(nb * D, dtype=torch.float32, device=sm.device)
        lib.add_dropout_ln_backward(_DT[sm.dtype], sm.data_ptr(), gy.data_ptr(), g.data_ptr(), pt,
                                    stats[0].data_ptr(), stats[1].data_ptr(), _p(mask), p, ds.data_ptr(),
                                    dh.data_ptr(), part.data_ptr(), hpart.data_ptr(), dg.data_ptr(), db.data_ptr(),
                                    gdt, accum, M, D, _stream())
        if _HANDOFF:
            dh._mxamd_bias_part = (hpart, nb, dh._version)
        dx = ds
        if ctx.res_src is not None and ctx.needs_input_grad[0]:
            ctx.res_src._mxamd_res_grad = ds
            dx = None
        ctx.res_src = None
        if accum:
            return dx, dh, None, None, None, None, None
        return (dx, dh, dg.view(gamma.shape).to(gamma.dtype) if need_g else None,
                db.view(beta.shape).to(beta.dtype) if need_b else None, None, None, None)


class GELU(torch.autograd.Function):
    """erf-GELU (MXNet LeakyReLU act_type='gelu')."""

    @staticmethod
    def forward(ctx, x):
        y = torch.empty_like(x)
        _K.lib().gelu_forward(_DT[x.dtype], x.data_ptr(), y.data_ptr(), x.numel(), _stream())
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, = ctx.saved_tensors
        gy = gy.contiguous()
        dx = torch.empty_like(x)
        lib = _K.lib()
        N = x.shape[-1] if x.dim() else 1
        if (x.dim() >= 2 and N % 8 == 0 and x.dtype in (torch.float16, torch.bfloat16) and x.is_contiguous()
                and hasattr(lib, "gelu_backward_colpart")):
            # the producing Dense's bias gradient rides along as column partials (consumed by
            # Linear.backward through dx._mxamd_bias_part, like the add_dropout_layernorm tail's)
            M = x.numel() // N
            nb = lib.gelu_colpart_blocks(M, N)
            part = torch.empty(nb, N, dtype=torch.float32, device=x.device)
            lib.gelu_backward_colpart(_DT[x.dtype], x.data_ptr(), gy.data_ptr(), dx.data_ptr(), part.data_ptr(), M, N,
                                      _stream())
            dx._mxamd_bias_part = (part, nb, dx._version)
            return dx
        lib.gelu_backward(_DT[x.dtype], x.data_ptr(), gy.data_ptr(), dx.data_ptr(), x.numel(), _stream())
        return dx


class Softmax(torch.autograd.Function):
    """softmax / log_softmax of (x * scale) over the last axis, one wave per row."""

    @staticmethod
    def forward(ctx, x, scale=1.0, log=False):
        L = x.shape[-1]
        M = x.numel() // L
        y = torch.empty_like(x)
        _K.lib().softmax_forward(_DT[x.dtype], int(bool(log)), x.data_ptr(), y.data_ptr(), M, L, float(scale),
                                 _stream())
        ctx.save_for_backward(y)
        ctx.cfg = (float(scale), bool(log))
        return y

    @staticmethod
    def backward(ctx, gy):
        y, = ctx.saved_tensors
        scale, log = ctx.cfg
        gy = gy.contiguous()
        L = y.shape[-1]
        M = y.numel() // L
        dx = torch.empty_like(y)
        _K.lib().softmax_backward(_DT[y.dtype], int(log), y.data_ptr(), gy.data_ptr(), dx.data_ptr(), M, L, scale,
                                  _stream())
        return dx, None, None


def _seed():
    # drawn from torch's default CPU generator, so mx.random.seed() makes the masks reproducible
    return int(torch.randint(0, 2 ** 62, (1,)).item())


class Dropout(torch.autograd.Function):
    """y = x * keep / (1 - p), keep ~ Bernoulli(1 - p) from Philox(seed, index); returns (y, bitmask)."""

    @staticmethod
    def forward(ctx, x, p):
        y = torch.empty_like(x)
        mask = torch.empty(x.numel() // 8, dtype=torch.uint8, device=x.device)
        ctr = _state.GRAPH_RNG[0]
        if ctr is not None and torch.cuda.is_current_stream_capturing():
            _K.lib().dropout_forward(_DT[x.dtype], x.data_ptr(), y.data_ptr(), mask.data_ptr(), x.numel(),
                                     float(p), _seed(), _stream(), ctr.data_ptr())
        else:
            _K.lib().dropout_forward(_DT[x.dtype], x.data_ptr(), y.data_ptr(), mask.data_ptr(), x.numel(),
                                     float(p), _seed(), _stream())
        ctx.save_for_backward(mask)
        ctx.p = float(p)
        ctx.mark_non_differentiable(mask)
        ctx.set_materialize_grads(False)      # no zero-filled gradient for the mask output
        return y, mask

    @staticmethod
    def backward(ctx, gy, _gm):
        if gy is None:
            return None, None
        mask, = ctx.saved_tensors
        gy = gy.contiguous()
        dx = torch.empty_like(gy)
        _K.lib().dropout_backward(_DT[gy.dtype], gy.data_ptr(), mask.data_ptr(), dx.data_ptr(), gy.numel(), ctx.p,
                                  _stream())
        return dx, None


# ---------------------------------------------------------------------------
# flat-arena optimizers
# ---------------------------------------------------------------------------

class ChunkTable:
    """Device table mapping <= chunk-element pieces of an arena to parameter segments.

    ``segments``: list of (offset, length) in elements (offsets 8-aligned).  Each
    entry is (int64 start, int32 len, int32 seg) = 16 bytes, the layout of
    ``struct Chunk`` in src/kernels/optim_kernels.hip.
    """

    def __init__(self, segments, device, chunk=2048 * 8):
        import numpy as np
        rows = []
        for seg, (off, n) in enumerate(segments):
            n8 = (n + 7) // 8 * 8
            for s in range(0, n8, chunk):
                rows.append((off + s, min(chunk, n8 - s), seg))
        arr = np.zeros(len(rows), dtype=[('start', '<i8'), ('len', '<i4'), ('seg', '<i4')])
        for i, r in enumerate(rows):
            arr[i] = r
        self.n = len(rows)
        self.nseg = len(segments)
        self.table = torch.from_numpy(arr.view(np.uint8).copy()).to(device)


def flat_adam(w, g, mean, var, w32, lr, beta1, beta2, eps, wd, rescale, clip, adamw=False, eta=1.0, hp=None):
    """``hp``: optional device float tensor; hp[0] replaces ``lr`` at run time (graph-captured steps)."""
    lib = _K.lib()
    n = w.numel()
    assert n % 8 == 0 and g.numel() == n and mean.numel() == n and var.numel() == n
    args = (_DT[w.dtype], int(bool(adamw)), w.data_ptr(), g.data_ptr(), mean.data_ptr(), var.data_ptr(), _p(w32),
            n, float(lr), float(beta1), float(beta2), float(eps), float(wd), float(eta), float(rescale),
            float(clip), _stream())
    lib.flat_adam(*args) if hp is None else lib.flat_adam(*args, hp.data_ptr())


def lamb_update(w, g, mean, var, w32, upd, table, nrm, lr, beta1, beta2, eps, t, bias_correction, wd, rescale, clip,
                lower_bound=-1.0, upper_bound=-1.0, hp=None):
    """``hp``: optional device float tensor {lr, bc1, bc2} read at run time (graph-captured steps).
    ``nrm``: 2 * (segments + chunks) floats -- the per-segment norms, then the per-chunk partials."""
    assert nrm.numel() >= 2 * (table.nseg + table.n), 'lamb_update: nrm needs 2*(nseg + nchunks) floats'
    bc1 = 1.0 - beta1 ** t if bias_correction else 1.0
    bc2 = 1.0 - beta2 ** t if bias_correction else 1.0
    args = (_DT[w.dtype], w.data_ptr(), g.data_ptr(), mean.data_ptr(), var.data_ptr(), _p(w32),
            upd.data_ptr(), table.table.data_ptr(), table.n, nrm.data_ptr(), table.nseg, float(lr),
            float(beta1), float(beta2), float(eps), float(bc1), float(bc2), float(wd), float(rescale),
            float(clip), float(lower_bound), float(upper_bound), _stream())
    _K.lib().lamb_update(*args) if hp is None else _K.lib().lamb_update(*args, hp.data_ptr())


def seg_sumsq(x, table):
    # per-segment sums followed by the per-chunk partials they are reduced from (workspace)
    out = torch.empty(table.nseg + table.n, dtype=torch.float32, device=x.device)
    _K.lib().seg_sumsq(_DT[x.dtype], x.data_ptr(), table.table.data_ptr(), table.n, out.data_ptr(), table.nseg,
                       _stream())
    return out[:table.nseg]


def all_finite(x, scale=1.0, flag=None):
    """int32 device flag: 1 when every element of x*scale is finite (x flat, numel % 8 == 0)."""
    init = flag is None
    if flag is None:
        flag = torch.empty(1, dtype=torch.int32, device=x.device)
    _K.lib().all_finite(_DT[x.dtype], x.data_ptr(), x.numel(), float(scale), flag.data_ptr(), int(init), _stream())
    return flag




# ---------------------------------------------------------------------------
# FullyConnected on MFMA: the NHWC implicit-GEMM kernels with a 1x1 "image"
# ---------------------------------------------------------------------------
# y[M,N] = x[M,K] W[N,K]^T + b is conv_nhwc_fwd on x viewed as [M,1,1,K] with the
# OHWI weight [N,1,1,K] (bias in the epilogue); dX = dY W is the same kernel with
# W^T; dW = dY^T X is the split-pixel MFMA wgrad kernel.  Per (pass, shape) the
# autotuner (kernel_fns._select) compares them with hipBLASLt (torch.mm) and
# keeps the faster.

from . import kernel_fns as _KF  # noqa: E402
from . import gemm as _G  # noqa: E402


def gemm_ok(x, w):
    return (x.is_cuda and x.dtype in (torch.float16, torch.bfloat16) and w.dtype == x.dtype and w.dim() == 2
            and x.shape[-1] == w.shape[1] and x.numel() > 0 and x.numel() // x.shape[-1] < 2 ** 31 // max(1, w.shape[0]))


def _fc_fwd_cands(x2, w, b):
    M, K = x2.shape
    N = w.shape[0]
    c = []
    if K % 32 == 0 and N % 64 == 0 and x2.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0:
        c.append(('hip', lambda: _KF.conv_fwd(x2.view(M, 1, 1, K), w.view(N, 1, 1, K), (1, 1), (0, 0),
                                              b).view(M, N)))
        # the conv kernels' large-tile LDS-DMA variants (big 256x256 / 128x256 tiles, persistent ring)
        # are GEMMs on a [M,1,1,K] view as well
        for v in _KF._fwd_variants(K, N, b is not None, ktot=K):
            if v >= 10:
                c.append(('hip%d' % v, lambda v=v: _KF.conv_fwd(x2.view(M, 1, 1, K), w.view(N, 1, 1, K), (1, 1),
                                                                (0, 0), b, v).view(M, N)))
    c.extend(_G.candidates(x2, w, bias=b))
    c.append(('mm', lambda: torch.nn.functional.linear(x2, w, None if b is None else b.to(x2.dtype))))
    return c


def _wt(w):
    """W^T ([in][out]) for the K-contiguous data-gradient GEMMs on the in-tree LDS-tiled transpose
    (kernel_fns.transpose2d): torch's strided transpose copy of a 768 x 3072 bf16 weight took ~15 us,
    enough to hand every BERT data gradient to hipBLASLt although the GEMM itself is faster in-tree
    (tools/bench_gemm.py)."""
    return _KF.transpose2d(w)


def _fc_dgrad_cands(dy2, w, addend=None):
    """dX = dY . W (+ addend: a residual gradient folded into the GEMM epilogue / beta = 1)."""
    M, N = dy2.shape
    K = w.shape[1]
    c = []
    if addend is not None:
        if N % 32 == 0 and K % 64 == 0 and dy2.data_ptr() % 16 == 0:
            for v in _KF._fwd_variants(N, K, False, ktot=N):
                if v in _KF._BIG_VARIANTS and v not in _KF._BIG_SKINNY:
                    c.append(('hip%d' % v, lambda v=v: _KF.conv_fwd(dy2.view(M, 1, 1, N),
                                                                    _wt(w).view(K, 1, 1, N), (1, 1),
                                                                    (0, 0), None, v,
                                                                    addend=addend.view(M, 1, 1, K)).view(M, K)))
        if (N % 64 == 0 and K % 64 == 0 and dy2.is_cuda and dy2.dtype in _G._DT and w.dtype == dy2.dtype
                and dy2.is_contiguous() and dy2.data_ptr() % 16 == 0 and _K.available()):
            for cfg in _G.configs(M, K, N, _G.AUTOTUNE_TILES):
                c.append(('gemm%ds%d' % cfg, lambda cfg=cfg: _G.gemm_nt(dy2, _wt(w), addend=addend,
                                                                         cfg=cfg)))
        # the library GEMM plus one add: torch.addmm would first copy the addend into its output and
        # then run a beta = 1 GEMM, slower than both (measured in the BERT step)
        c.append(('mm', lambda: torch.mm(dy2, w).add_(addend)))
        return c
    if N % 32 == 0 and K % 64 == 0:
        c.append(('hip', lambda: _KF.conv_fwd(dy2.view(M, 1, 1, N), _wt(w).view(K, 1, 1, N), (1, 1),
                                              (0, 0)).view(M, K)))
        if dy2.data_ptr() % 16 == 0:
            for v in _KF._fwd_variants(N, K, False, ktot=N):
                if v >= 10:
                    c.append(('hip%d' % v, lambda v=v: _KF.conv_fwd(dy2.view(M, 1, 1, N),
                                                                    _wt(w).view(K, 1, 1, N), (1, 1),
                                                                    (0, 0), None, v).view(M, K)))
    # dX = dY . W = dY . (W^T)^T: the GEMM kernel on a fresh W^T (a small copy; the weight may
    # change in place between steps through the fused optimizer's raw pointers, so no caching)
    if (N % 64 == 0 and K % 64 == 0 and dy2.is_cuda and dy2.dtype in _G._DT and w.dtype == dy2.dtype
            and dy2.is_contiguous() and dy2.data_ptr() % 16 == 0 and _K.available()):
        for cfg in _G.configs(M, K, N, _G.AUTOTUNE_TILES):
            c.append(('gemm%ds%d' % cfg, lambda cfg=cfg: _G.gemm_nt(dy2, _wt(w), cfg=cfg)))
    c.append(('mm', lambda: torch.mm(dy2, w)))
    return c


def _splitk_wgrad(dy2, x2, splits, out, accum):
    """dW = dY^T X as ``splits`` batched GEMMs over row blocks of M (fp32 partials, so a small N x K
    output still covers all 256 CUs) summed -- and accumulated into ``out`` when ``accum`` -- by the
    in-tree slab_reduce kernel."""
    M, N = dy2.shape
    K = x2.shape[1]
    slab = torch.empty(splits, N, K, dtype=torch.float32, device=dy2.device)
    torch.bmm(dy2.view(splits, M // splits, N).transpose(1, 2), x2.view(splits, M // splits, K),
              out_dtype=torch.float32, out=slab)
    _K.lib().slab_reduce(_DT[out.dtype], slab.data_ptr(), splits, N * K, out.data_ptr(), int(accum), _stream())
    return out


def _fc_wgrad_cands(dy2, x2, w):
    M, N = dy2.shape
    K = x2.shape[1]
    c = []
    if (N * K) % 4 == 0 and dy2.is_contiguous() and x2.is_contiguous():
        for S in (2, 4):
            if M % S == 0 and (M // S) >= 256:
                c.append(('sk%d' % S, lambda S=S: _splitk_wgrad(dy2, x2, S, torch.empty(N, K, dtype=w.dtype,
                                                                                         device=w.device), False)))
    if K % 64 == 0 and N % 64 == 0 and x2.data_ptr() % 16 == 0:
        c.append(('hip', lambda: _KF.conv_wgrad(x2.view(M, 1, 1, K), dy2.view(M, 1, 1, N), (N, 1, 1, K), (1, 1),
                                                (0, 0)).view(N, K)))
        # the persistent LDS-DMA ring weight-gradient kernels (conv_wgrad.hip), TN on a [M,1,1,*] view
        lib = _K.lib()
        for v in range(1, 10):
            if lib.conv_nhwc_wgrad_ring_ok(K, N, 1, 1, v):
                c.append(('ring%d' % v, lambda v=v: _KF.conv_wgrad(x2.view(M, 1, 1, K), dy2.view(M, 1, 1, N),
                                                                   (N, 1, 1, K), (1, 1), (0, 0), ring=v).view(N, K)))
    c.append(('mm', lambda: torch.mm(dy2.t(), x2)))
    return c


class Linear(torch.autograd.Function):
    """FullyConnected (flatten=False semantics on the last axis) with per-shape kernel selection."""

    @staticmethod
    def forward(ctx, x, w, b):
        K = x.shape[-1]
        x2 = x.reshape(-1, K).contiguous()
        key = ('fc_fwd', tuple(x2.shape), tuple(w.shape), x.dtype, b is not None)
        y = _KF._select(key, _fc_fwd_cands(x2, w.contiguous(), b), 'mm')
        ctx.save_for_backward(x2, w)
        ctx.has_b = b is not None
        ctx.bdt = b.dtype if b is not None else None
        ctx.xshape = x.shape
        ctx.refs = (w, b)
        # a residual gradient may be handed to this layer's data gradient (AddDropoutLN handoff)
        x._mxamd_fc_input = True
        ctx.x_src = x
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        w_ref, b_ref = ctx.refs
        N = w.shape[0]
        dy2 = dy.reshape(-1, N).contiguous()
        dx = dw = db = None
        res = getattr(ctx.x_src, '_mxamd_res_grad', None)
        if res is not None:
            del ctx.x_src._mxamd_res_grad
        ctx.x_src = None
        if ctx.needs_input_grad[0]:
            if res is not None:
                add = res.reshape(-1, w.shape[1]).contiguous()
                key = ('fc_dgrad_add', tuple(dy2.shape), tuple(w.shape), dy.dtype)
                dx = _KF._select(key, _fc_dgrad_cands(dy2, w.contiguous(), add), 'mm').view(ctx.xshape)
            else:
                key = ('fc_dgrad', tuple(dy2.shape), tuple(w.shape), dy.dtype)
                dx = _KF._select(key, _fc_dgrad_cands(dy2, w.contiguous()), 'mm').view(ctx.xshape)
        elif res is not None:
            dx = res
        if ctx.needs_input_grad[1]:
            dw = _fc_wgrad(dy2, x2, w, w_ref)
        if ctx.has_b and ctx.needs_input_grad[2]:
            bp = getattr(dy, '_mxamd_bias_part', None)
            if bp is not None and bp[2] == dy._version and dy.shape[-1] == N:
                db = _bias_from_partials(bp[0], bp[1], N, b_ref, ctx.bdt, dy.device)
            else:
                db = bias_grad(dy2, b_ref, ctx.bdt)
        return dx, dw, db


import os as _os                       # noqa: E402
_FC_DIRECT = _os.environ.get('MXAMD_FC_DIRECT', '1') == '1'


def _fc_wgrad(dy2, x2, w, w_ref):
    """dW = dY^T X; accumulated straight into the weight's .grad buffer when possible (GEMM with
    beta = 1 / the MFMA kernel's accumulating reduce) so no separate dW tensor and add kernel."""
    key = ('fc_wgrad', tuple(dy2.shape), tuple(x2.shape), dy2.dtype)
    algo = _KF._ALGO.get(_KF._akey(key))
    tgt = _leaf_grad(w_ref, dtype=w.dtype) if (algo is not None and _FC_DIRECT) else None
    if tgt is not None:
        N, K = w.shape
        if algo == 'hip' or algo.startswith('ring'):
            _KF.conv_wgrad(x2.view(-1, 1, 1, K), dy2.view(-1, 1, 1, N), (N, 1, 1, K), (1, 1), (0, 0),
                           out=tgt.view(N, 1, 1, K), accum=True, ring=int(algo[4:]) if algo != 'hip' else 0)
        elif algo.startswith('sk'):
            _splitk_wgrad(dy2, x2, int(algo[2:]), tgt.view(N, K), True)
        else:
            tgt.addmm_(dy2.t(), x2)
        return None
    return _KF._select(key, _fc_wgrad_cands(dy2, x2, w), 'mm').to(w.dtype)


_COLSUM_PART = {}


def bias_grad(dy2, b_ref, bdt):
    """db = column sums of dY [M, N] in fp32 on the HIP reduce kernels, accumulated into the bias's
    .grad buffer when possible (returns None then)."""
    M, N = dy2.shape
    if not (dy2.is_cuda and _K.available() and dy2.dtype in _DT and N % 8 == 0 and _aligned(dy2)):
        return torch.sum(dy2, 0, dtype=torch.float32).to(bdt)
    lib = _K.lib()
    n = lib.colsum_partials(M, N)
    # scratch per (device, stream): concurrent reductions on different streams must not share it
    skey = (dy2.device, torch.cuda.current_stream(dy2.device).cuda_stream)
    part = _COLSUM_PART.get(skey)
    if part is None or part.numel() < n:
        part = _COLSUM_PART[skey] = torch.empty(n, dtype=torch.float32, device=dy2.device)
    tgt = _leaf_grad(b_ref, N, dtype=bdt) if (bdt in _DT and _FC_DIRECT) else None
    # not accumulated in place: written in the bias dtype by the same kernel (fp32 sums), no conversion launch
    out = tgt if tgt is not None else torch.empty(N, dtype=bdt if bdt in _DT else torch.float32, device=dy2.device)
    # two launches (partial rows, then their sum); see bn_nhwc.hip on why not one
    lib.colsum_rows(_DT[dy2.dtype], dy2.data_ptr(), _KF._zeros_f32(N, dy2.device).data_ptr(), part.data_ptr(),
                    M, N, _DT[out.dtype], out.data_ptr(), int(tgt is not None), _stream())
    if tgt is not None:
        return None
    return out if out.dtype == bdt else out.to(bdt)


def _bias_from_partials(part, nb, N, b_ref, bdt, dev):
    """db from column partials an earlier kernel already reduced (add_dropout_ln backward): one small
    column-sum launch, accumulated straight into the bias's .grad buffer when possible."""
    tgt = _leaf_grad(b_ref, N, dtype=bdt) if (bdt in _DT and _FC_DIRECT) else None
    out = tgt if tgt is not None else torch.empty(N, dtype=bdt if bdt in _DT else torch.float32, device=dev)
    _K.lib().column_sum_partials(_DT[out.dtype], part.data_ptr(), nb, N, out.data_ptr(), int(tgt is not None),
                                 _stream())
    return None if tgt is not None else (out if out.dtype == bdt else out.to(bdt))


_IDX_T = {torch.float32: 0, torch.int64: 1, torch.int32: 2}
_EMB_DIRECT = _os.environ.get('MXAMD_EMB_DIRECT', '1') == '1'
_EMB_SCRATCH = {}


def embedding_ok(idx, w):
    return (_os.environ.get('MXAMD_EMB_HIP', '1') == '1' and w.is_cuda and w.dtype in _DT and w.dim() == 2 and w.shape[1] % 8 == 0 and _aligned(w)
            and idx.device == w.device and idx.numel() > 0 and w.shape[0] < 2 ** 31)


class Embedding(torch.autograd.Function):
    """Row gather ``y[..., :] = W[idx[...], :]`` (indices clamped to [0, V), any of float32 / int64 /
    int32) and its scatter-add backward on HIP kernels: fp32 hardware atomics into a persistent,
    always-zero [V, C] scratch, then one pass that adds the touched rows into the weight's .grad
    buffer (or a fresh gradient) and re-zeroes them.  No sort / unique, nothing data-dependent on
    the host, so the backward is HIP-graph capturable."""

    @staticmethod
    def forward(ctx, idx, w):
        if idx.dtype not in _IDX_T:
            idx = idx.to(torch.int64)
        idx = idx.contiguous()
        V, C = w.shape
        n = idx.numel()
        y = torch.empty(tuple(idx.shape) + (C,), dtype=w.dtype, device=w.device)
        _K.lib().embedding_forward(_DT[w.dtype], _IDX_T[idx.dtype], idx.data_ptr(), w.contiguous().data_ptr(),
                                   y.data_ptr(), n, V, C, _stream())
        ctx.save_for_backward(idx)
        ctx.w_ref = w
        ctx.vc = (V, C, w.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        idx, = ctx.saved_tensors
        V, C, wdt = ctx.vc
        dy = dy.contiguous()
        dev = dy.device
        if _KF.deterministic():
            # MXNET_ENFORCE_DETERMINISM: an ordered (sort-based) accumulation instead of float atomics
            rows = idx.reshape(-1).to(torch.int64).clamp(0, V - 1)
            acc = torch.zeros((V, C), dtype=torch.float32, device=dev)
            acc.index_put_((rows,), dy.reshape(-1, C).float(), accumulate=True)
            tgt = _leaf_grad(ctx.w_ref, V * C, dtype=wdt) if ctx.needs_input_grad[1] else None
            if tgt is not None:
                tgt.add_(acc.view(tgt.shape))
                return None, None
            return None, acc.to(wdt)
        key = (V, C, dev)
        sc = _EMB_SCRATCH.get(key)
        if sc is None:
            sc = _EMB_SCRATCH[key] = (torch.zeros(V * C, dtype=torch.float32, device=dev),
                                      torch.zeros(V, dtype=torch.uint8, device=dev))
        tgt = _leaf_grad(ctx.w_ref, V * C, dtype=wdt) if (ctx.needs_input_grad[1] and _EMB_DIRECT) else None
        out = tgt if tgt is not None else torch.empty((V, C), dtype=wdt, device=dev)
        _K.lib().embedding_backward(_DT[dy.dtype], _IDX_T[idx.dtype], idx.data_ptr(), dy.data_ptr(),
                                    sc[0].data_ptr(), sc[1].data_ptr(), _DT[out.dtype], out.data_ptr(),
                                    int(tgt is not None), idx.numel(), V, C, _stream())
        return None, (None if tgt is not None else out)


__all__ += ['Linear', 'gemm_ok', 'Embedding', 'embedding_ok']
