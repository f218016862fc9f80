"""contrib operators: deformable convolution (v1 / modulated v2), SyncBatchNorm, PixelShuffle helpers.

Parity: src/operator/contrib/deformable_convolution*, modulated_deformable_convolution*,
sync_batch_norm*.  On the GPU deformable convolution runs the in-tree gfx950 kernels of
src/kernels/deform_conv.hip: a deformable im2col (bilinear sampling at the offset taps, mask
applied) writing one K-contiguous column row per output pixel, contracted on the matrix cores by
the in-tree GEMMs (reference: deformable_convolution-inl.h:150-159 -- im2col + linalg_gemm per
group):
  forward      out[N*L, O]   = cols[N*L, C*K] . W[O, C*K]^T (+ bias)  gemm.hip NT, bias in the epilogue
  weight grad  dW[O, C*K]    = dout^T . cols                          conv_wgrad.hip TN (fp32 slabs)
  column grad  dcols[N*L,C*K] = dout . W  (fp32 out)                  gemm.hip NT on W^T
the output stays NHWC in memory (an NCHW view), and the backward runs col2im (data gradient, fp32
atomics) + col2im_coord (offset / mask gradients, register reductions) on the fp32 column
gradient.  fp32 operands keep the plane layout contracted by torch.matmul.  On the CPU the same math is one ``grid_sample`` per kernel tap (bilinear, zero outside)
followed by the grouped GEMM, differentiated by autograd.
"""
import torch
import torch.nn.functional as F

from .. import _state
from .registry import register


def _deform_columns(x, offset, mask, kernel, stride, pad, dilate, dg):
    """Sampled columns [N, C, K, Ho, Wo] for deformable convolution."""
    N, C, H, W = x.shape
    kh, kw = kernel
    sh, sw = stride
    ph, pw = pad
    dh, dw = dilate
    Ho, Wo = offset.shape[2], offset.shape[3]
    K = kh * kw
    dev, dt = x.device, x.dtype
    base_h = (torch.arange(Ho, device=dev, dtype=dt) * sh - ph).view(1, Ho, 1)
    base_w = (torch.arange(Wo, device=dev, dtype=dt) * sw - pw).view(1, 1, Wo)
    cpg = C // dg
    off = offset.reshape(N, dg, K, 2, Ho, Wo)
    cols = []
    for k in range(K):
        i, j = divmod(k, kw)
        hs = base_h + i * dh + off[:, :, k, 0]          # [N, dg, Ho, Wo]
        ws = base_w + j * dw + off[:, :, k, 1]
        gy = 2.0 * hs / max(H - 1, 1) - 1.0
        gx = 2.0 * ws / max(W - 1, 1) - 1.0
        grid = torch.stack([gx, gy], dim=-1).reshape(N * dg, Ho, Wo, 2)
        xs = x.reshape(N * dg, cpg, H, W)
        s = F.grid_sample(xs, grid, mode='bilinear', padding_mode='zeros', align_corners=True)
        s = s.reshape(N, dg, cpg, Ho, Wo)
        if mask is not None:
            s = s * mask.reshape(N, dg, K, Ho, Wo)[:, :, k].unsqueeze(2)
        cols.append(s.reshape(N, C, Ho, Wo))
    return torch.stack(cols, dim=2)                     # [N, C, K, Ho, Wo]


class _DeformConvHip(torch.autograd.Function):
    """Deformable conv on the HIP kernels: columns [N, g, C/g*K, L] -> GEMM with [g, O/g, C/g*K]."""

    @staticmethod
    def forward(ctx, x, offset, mask, weight, geom, num_group):
        from . import kernels as _K
        from .kernel_fns import _DT, _stream
        lib = _K.lib()
        N, C, H, W = x.shape
        O = weight.shape[0]
        Ho, Wo = geom[4], geom[5]
        K = geom[6] * geom[7]
        x, offset = x.contiguous(), offset.contiguous()
        mask = mask.contiguous() if mask is not None else None
        cols = torch.empty((N, C * K, Ho * Wo), dtype=x.dtype, device=x.device)
        lib.deform_im2col(_DT[x.dtype], x.data_ptr(), offset.data_ptr(), 0 if mask is None else mask.data_ptr(),
                          cols.data_ptr(), list(geom), _stream())
        g = num_group
        wmat = weight.reshape(g, O // g, (C // g) * K)
        out = torch.matmul(wmat, cols.view(N, g, (C // g) * K, Ho * Wo))        # [N, g, O/g, L]
        ctx.save_for_backward(x, offset, mask, weight, cols)
        ctx.geom, ctx.g = geom, g
        return out.reshape(N, O, Ho, Wo)

    @staticmethod
    def backward(ctx, gout):
        from . import kernels as _K
        from .kernel_fns import _DT, _stream
        lib = _K.lib()
        x, offset, mask, weight, cols = ctx.saved_tensors
        geom, g = ctx.geom, ctx.g
        N, C, H, W = x.shape
        O = weight.shape[0]
        L = geom[4] * geom[5]
        K = geom[6] * geom[7]
        go = gout.contiguous().view(N, g, O // g, L)
        wmat = weight.reshape(g, O // g, (C // g) * K)
        gw = torch.matmul(go.permute(1, 2, 0, 3).reshape(g, O // g, N * L),
                          cols.view(N, g, (C // g) * K, L).permute(1, 0, 3, 2).reshape(g, N * L, (C // g) * K))
        # fp32 column gradients: the offset gradient is a difference of products, bf16 columns lose it
        gcols = torch.matmul(wmat.transpose(1, 2).float(), go.float()).reshape(N, C * K, L).contiguous()
        gx32 = torch.zeros(x.shape, dtype=torch.float32, device=x.device)
        mptr = 0 if mask is None else mask.data_ptr()
        lib.deform_col2im(_DT[x.dtype], offset.data_ptr(), mptr, gcols.data_ptr(), gx32.data_ptr(), list(geom),
                          _stream())
        goff = torch.empty_like(offset)
        gmask = torch.empty_like(mask) if mask is not None else None
        lib.deform_col2im_coord(_DT[x.dtype], x.data_ptr(), offset.data_ptr(), mptr, gcols.data_ptr(),
                                goff.data_ptr(), 0 if gmask is None else gmask.data_ptr(), list(geom), _stream())
        return gx32.to(x.dtype), goff, gmask, gw.reshape(weight.shape).to(weight.dtype), None, None


DISPATCH = {'gemm': 0, 'plane': 0}


def _pick(key, cands, fallback):
    """Autotuned in-tree GEMM candidate for ``key``; ``fallback`` (torch) when none tiles the shape."""
    from .kernel_fns import _select
    if not cands:
        from .rnn_fns import _require_hip
        if _require_hip():
            from ..base import MXNetError
            raise MXNetError('deformable convolution: %r does not tile for the in-tree GEMM kernels' % (key,))
        return fallback()
    return _select(key, cands, cands[0][0])


def _pixel_rows(t):
    """[N, F, Ho, Wo] (NCHW-shaped) -> ([N, Ho, Wo, F] view with unit feature stride, row stride):
    free for channels-last memory, including a channel slice of a wider buffer (the output-channel
    padded offset conv), one copy otherwise."""
    v = t.permute(0, 2, 3, 1)
    N, Ho, Wo, F = v.shape
    ld = v.stride(2)
    if not (v.stride(3) == 1 and ld >= F and v.stride(1) == Wo * ld and v.stride(0) == Ho * Wo * ld
            and v.data_ptr() % 16 == 0):
        v = v.contiguous()
        ld = F
    return v, ld


def _nhwc_ok(x, weight, dg, kernel):
    C = x.shape[1]
    return (C // dg) % 64 == 0 and kernel[0] * kernel[1] <= 16


class _DeformConvRows(torch.autograd.Function):
    """Deformable conv (f16/bf16) with row columns [N*L, C*K] on the in-tree MFMA GEMMs.  Channels-last
    (``nhwc``): image, offsets, mask and all their gradients in [N, H, W, C] memory, the sampling and the
    fused backward (data + offset + mask gradients in one pass) one wave per output pixel."""

    @staticmethod
    def forward(ctx, x, offset, mask, weight, bias, geom, num_group):
        from . import kernels as _K
        from . import gemm as G
        from .kernel_fns import _DT, _stream
        lib = _K.lib()
        N, C, H, W = x.shape
        O = weight.shape[0]
        Ho, Wo = geom[4], geom[5]
        K = geom[6] * geom[7]
        L = Ho * Wo
        nhwc = _nhwc_ok(x, weight, geom[14], (geom[6], geom[7]))
        cols = torch.empty((N * L, C * K), dtype=x.dtype, device=x.device)
        if nhwc:
            x = x.permute(0, 2, 3, 1).contiguous()                  # free for channels-last activations
            offset, ld_off = _pixel_rows(offset)
            mask, ld_msk = _pixel_rows(mask) if mask is not None else (None, 0)
            lib.deform_im2col_nhwc(_DT[x.dtype], x.data_ptr(), offset.data_ptr(),
                                   0 if mask is None else mask.data_ptr(), cols.data_ptr(), list(geom), ld_off,
                                   ld_msk, _stream())
            ctx.ld = (ld_off, ld_msk)
        else:
            x, offset = x.contiguous(), offset.contiguous()
            mask = mask.contiguous() if mask is not None else None
            lib.deform_im2col(_DT[x.dtype], x.data_ptr(), offset.data_ptr(), 0 if mask is None else mask.data_ptr(),
                              cols.data_ptr(), list(geom) + [1], _stream())
        ctx.nhwc = nhwc
        g = num_group
        cg, og = (C // g) * K, O // g
        wmat = weight.reshape(O, cg).contiguous()
        b32 = None if bias is None else bias.float().contiguous()
        out = torch.empty((N * L, O), dtype=x.dtype, device=x.device)
        for gi in range(g):
            a = cols[:, gi * cg:(gi + 1) * cg]
            b = wmat[gi * og:(gi + 1) * og]
            bb = None if b32 is None else b32[gi * og:(gi + 1) * og]
            o = out[:, gi * og:(gi + 1) * og]
            cands = [(n, (lambda c=c: G.gemm_nt(a, b, bias=bb, out=o, cfg=c)))
                     for n, c in ((n, G.parse_name(n)) for n, _ in G.candidates(a, b))
                     if g == 1 or c[1] == 1]
            _pick(('deform_fwd', tuple(a.shape), tuple(b.shape), x.dtype, bb is not None), cands,
                  lambda: o.copy_(torch.addmm(bb.to(x.dtype), a, b.t()) if bb is not None else a @ b.t()))
        DISPATCH['gemm'] += 1
        ctx.save_for_backward(x, offset, mask, wmat, cols)
        ctx.geom, ctx.g, ctx.has_bias = geom, g, bias is not None
        ctx.bdtype = None if bias is None else bias.dtype
        ctx.b_ref = bias
        ctx.wdtype = weight.dtype
        return out.view(N, Ho, Wo, O).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, gout):
        from . import kernels as _K
        from . import gemm as G
        from . import kernel_fns as KF
        from .kernel_fns import _DT, _stream
        lib = _K.lib()
        x, offset, mask, wmat, cols = ctx.saved_tensors
        geom, g = ctx.geom, ctx.g
        N, C = geom[0], geom[1]
        O = wmat.shape[0]
        L = geom[4] * geom[5]
        K = geom[6] * geom[7]
        M = N * L
        cg, og = (C // g) * K, O // g
        go = gout.permute(0, 2, 3, 1).reshape(M, O).contiguous()
        gw = torch.empty((O, cg), dtype=ctx.wdtype, device=x.device)
        gcols = torch.empty((M, C * K), dtype=torch.float32, device=x.device)
        for gi in range(g):
            dy = go[:, gi * og:(gi + 1) * og]
            xc = cols[:, gi * cg:(gi + 1) * cg]
            # weight gradient: a 1x1-conv weight gradient over the M output pixels (TN, fp32 slabs);
            # a group's column / gradient slices are made contiguous for it
            xcc, dyc = (xc, dy) if g == 1 else (xc.contiguous(), dy.contiguous())
            if KF.conv_wgrad_ok(xcc.view(1, 1, M, cg), torch.empty((og, 1, 1, cg), device='meta')):
                KF.conv_wgrad(xcc.view(1, 1, M, cg), dyc.view(1, 1, M, og), (og, 1, 1, cg), (1, 1), (0, 0),
                              out=gw[gi * og:(gi + 1) * og].view(og, 1, 1, cg))
            else:
                _pick(('deform_dw', tuple(dy.shape), tuple(xc.shape), x.dtype), [],
                      lambda: gw[gi * og:(gi + 1) * og].copy_(dy.t() @ xc))
            # column gradient in fp32 (the offset gradient is a difference of products)
            wt = KF.transpose2d(wmat[gi * og:(gi + 1) * og])
            o = gcols[:, gi * cg:(gi + 1) * cg]
            cands = [(n, (lambda c=c: G.gemm_nt(dy, wt, out=o, out_f32=True, cfg=c)))
                     for n, c in ((n, G.parse_name(n)) for n, _ in G.candidates(dy, wt, out_f32=True))
                     if g == 1 or c[1] == 1]
            _pick(('deform_dcols', tuple(dy.shape), tuple(wt.shape), x.dtype), cands,
                  lambda: o.copy_(dy.float() @ wt.float().t()))
        mptr = 0 if mask is None else mask.data_ptr()
        if ctx.nhwc:
            # x [N, H, W, C], offsets / mask pixel rows: one fused pass, gradients channels-last
            gx32 = torch.zeros(x.shape, dtype=torch.float32, device=x.device)
            dg = geom[14]
            goff = torch.empty((N, geom[4], geom[5], 2 * K * dg), dtype=offset.dtype, device=x.device)
            gmask = (torch.empty((N, geom[4], geom[5], K * dg), dtype=mask.dtype, device=x.device)
                     if mask is not None else None)
            lib.deform_bwd_nhwc(_DT[x.dtype], x.data_ptr(), offset.data_ptr(), mptr, gcols.data_ptr(),
                                gx32.data_ptr(), goff.data_ptr(), 0 if gmask is None else gmask.data_ptr(),
                                list(geom), ctx.ld[0], ctx.ld[1], _stream())
            gx = gx32.to(x.dtype).permute(0, 3, 1, 2)
            goff = goff.permute(0, 3, 1, 2)
            gmask = gmask.permute(0, 3, 1, 2) if gmask is not None else None
        else:
            gx32 = torch.zeros(x.shape, dtype=torch.float32, device=x.device)
            g16 = list(geom) + [1]
            lib.deform_col2im(_DT[x.dtype], offset.data_ptr(), mptr, gcols.data_ptr(), gx32.data_ptr(), g16,
                              _stream())
            goff = torch.empty_like(offset)
            gmask = torch.empty_like(mask) if mask is not None else None
            lib.deform_col2im_coord(_DT[x.dtype], x.data_ptr(), offset.data_ptr(), mptr, gcols.data_ptr(),
                                    goff.data_ptr(), 0 if gmask is None else gmask.data_ptr(), g16, _stream())
            gx = gx32.to(x.dtype)
        gb = None
        if ctx.has_bias:
            from .nlp_fns import bias_grad
            gb = bias_grad(go, ctx.b_ref, ctx.bdtype)
        return (gx, goff, gmask, gw.view(O, C // g, geom[6], geom[7]), gb, None, None)


def _rows_ok(x, weight, num_group, kernel):
    from . import gemm as G
    C, O = x.shape[1], weight.shape[0]
    K = kernel[0] * kernel[1]
    cg, og = (C // num_group) * K, O // num_group
    return (x.dtype in G._DT and cg % 64 == 0 and og % 64 == 0 and 64 * min(16, max(1, 512 // K)) * K * 2 <= 65536)


def _deform_hip_ok(x, offset, mask, weight):
    from . import kernels as _K
    from .kernel_fns import _DT
    ts = [t for t in (x, offset, mask, weight) if t is not None]
    if not (x.is_cuda and all(t.is_cuda and t.dtype == x.dtype for t in ts) and x.dtype in _DT):
        return False
    if not _K.available():
        # fail loudly on a GPU box without the extension instead of silently using the torch path
        raise RuntimeError('deformable convolution: HIP kernel extension not available: %s' % _K.load_error())
    return _K.enabled()


def _deform_conv(x, offset, mask, weight, bias, kernel, stride, pad, dilate, num_group, dg):
    if _deform_hip_ok(x, offset, mask, weight):
        N, C, H, W = x.shape
        Ho, Wo = offset.shape[2], offset.shape[3]
        geom = (N, C, H, W, Ho, Wo, kernel[0], kernel[1], stride[0], stride[1], pad[0], pad[1], dilate[0],
                dilate[1], dg)
        if _rows_ok(x, weight, num_group, kernel):
            return _DeformConvRows.apply(x, offset, mask, weight, bias, geom, num_group)
        DISPATCH['plane'] += 1
        out = _DeformConvHip.apply(x, offset, mask, weight, geom, num_group)
        return out if bias is None else out + bias.view(1, -1, 1, 1).to(out.dtype)
    cols = _deform_columns(x, offset, mask, kernel, stride, pad, dilate, dg)
    N, C, K, Ho, Wo = cols.shape
    O = weight.shape[0]
    g = num_group
    cols = cols.reshape(N, g, C // g, K, Ho, Wo)
    w = weight.reshape(g, O // g, C // g, K)
    out = torch.einsum('ngckhw,gock->ngohw', cols, w).reshape(N, O, Ho, Wo)
    if bias is not None:
        out = out + bias.view(1, -1, 1, 1)
    return out


def _dc_out_shape(x, kernel, stride, pad, dilate):
    H, W = x.shape[2], x.shape[3]
    Ho = (H + 2 * pad[0] - dilate[0] * (kernel[0] - 1) - 1) // stride[0] + 1
    Wo = (W + 2 * pad[1] - dilate[1] * (kernel[1] - 1) - 1) // stride[1] + 1
    return Ho, Wo


def _dc_args(a):
    nb = str(a.get('no_bias', False)) in ('True', 'true', '1')
    return ['data', 'offset', 'weight'] + ([] if nb else ['bias'])


def _dc_infer(in_shapes, a):
    from .registry import parse_value
    d = in_shapes[0]
    if d is None:
        return {}
    k = parse_value('shape', a.get('kernel', '(1,1)'))
    s = parse_value('shape', a.get('stride', '(1,1)')) or (1, 1)
    p = parse_value('shape', a.get('pad', '(0,0)')) or (0, 0)
    dl = parse_value('shape', a.get('dilate', '(1,1)')) or (1, 1)
    nf = int(a['num_filter'])
    g = int(a.get('num_group', 1))
    dg = int(a.get('num_deformable_group', 1))
    Ho = (d[2] + 2 * p[0] - dl[0] * (k[0] - 1) - 1) // s[0] + 1
    Wo = (d[3] + 2 * p[1] - dl[1] * (k[1] - 1) - 1) // s[1] + 1
    res = {1: (d[0], 2 * dg * k[0] * k[1], Ho, Wo), 2: (nf, d[1] // g) + tuple(k)}
    if not (str(a.get('no_bias', False)) in ('True', 'true', '1')):
        res[3] = (nf,)
    return res


_DC_PARAMS = {'kernel': ('shape', ()), 'stride': ('shape', ()), 'dilate': ('shape', ()), 'pad': ('shape', ()),
              'num_filter': ('int', 1), 'num_group': ('int', 1), 'num_deformable_group': ('int', 1),
              'workspace': ('int', 1024), 'no_bias': ('bool', False), 'layout': ('str?', None)}


@register('_contrib_DeformableConvolution', aliases=('DeformableConvolution',), arg_names=_dc_args,
          infer_params=_dc_infer, params=_DC_PARAMS)
def deformable_convolution(data, offset, weight, bias=None, kernel=(), stride=(), dilate=(), pad=(), num_filter=1,
                           num_group=1, num_deformable_group=1, workspace=1024, no_bias=False, layout=None):
    stride = tuple(stride) or (1, 1)
    dilate = tuple(dilate) or (1, 1)
    pad = tuple(pad) or (0, 0)
    return _deform_conv(data, offset, None, weight, None if no_bias else bias, tuple(kernel), stride, pad, dilate,
                        num_group, num_deformable_group)


def _mdc_args(a):
    nb = str(a.get('no_bias', False)) in ('True', 'true', '1')
    return ['data', 'offset', 'mask', 'weight'] + ([] if nb else ['bias'])


def _mdc_infer(in_shapes, a):
    r = _dc_infer(in_shapes, a)
    if not r:
        return r
    from .registry import parse_value
    k = parse_value('shape', a.get('kernel', '(1,1)'))
    dg = int(a.get('num_deformable_group', 1))
    off = r[1]
    out = {1: off, 2: (off[0], dg * k[0] * k[1], off[2], off[3]), 3: r[2]}
    if 3 in r:
        out[4] = r[3]
    return out


@register('_contrib_ModulatedDeformableConvolution', aliases=('ModulatedDeformableConvolution',),
          arg_names=_mdc_args, infer_params=_mdc_infer, params=dict(_DC_PARAMS, im2col_step=('int', 64)))
def modulated_deformable_convolution(data, offset, mask, weight, bias=None, kernel=(), stride=(), dilate=(), pad=(),
                                     num_filter=1, num_group=1, num_deformable_group=1, workspace=1024,
                                     no_bias=False, layout=None, im2col_step=64):
    stride = tuple(stride) or (1, 1)
    dilate = tuple(dilate) or (1, 1)
    pad = tuple(pad) or (0, 0)
    return _deform_conv(data, offset, mask, weight, None if no_bias else bias, tuple(kernel), stride, pad, dilate,
                        num_group, num_deformable_group)


# ---------------------------------------------------------------------------
# SyncBatchNorm: batch statistics all-reduced over the data-parallel group
# ---------------------------------------------------------------------------

def _allreduce_(t):
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        if t.is_cuda or dist.get_backend() != 'nccl':
            dist.all_reduce(t)
        else:
            tc = t.cuda()
            dist.all_reduce(tc)
            t.copy_(tc.cpu())
    return t


class _SyncBN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, eps, axis):
        dims = [d for d in range(x.dim()) if d != axis]
        xf = x.float()
        n_local = torch.tensor([float(x.numel() // x.shape[axis])], device=x.device)
        stats = torch.cat([xf.sum(dims), (xf * xf).sum(dims), n_local])
        _allreduce_(stats)
        C = x.shape[axis]
        n = stats[-1]
        mean = stats[:C] / n
        var = torch.clamp(stats[C:2 * C] / n - mean * mean, min=0.0)
        invstd = torch.rsqrt(var + eps)
        shape = [1] * x.dim()
        shape[axis] = C
        xhat = (xf - mean.view(shape)) * invstd.view(shape)
        y = xhat * gamma.float().view(shape) + beta.float().view(shape)
        ctx.save_for_backward(xhat, gamma, invstd, n)
        ctx.axis = axis
        return y.to(x.dtype), mean, var

    @staticmethod
    def backward(ctx, dy, _dm, _dv):
        xhat, gamma, invstd, n = ctx.saved_tensors
        axis = ctx.axis
        dims = [d for d in range(xhat.dim()) if d != axis]
        C = xhat.shape[axis]
        shape = [1] * xhat.dim()
        shape[axis] = C
        dyf = dy.float()
        sums = torch.cat([dyf.sum(dims), (dyf * xhat).sum(dims)])
        dbeta_local, dgamma_local = sums[:C].clone(), sums[C:].clone()
        _allreduce_(sums)
        dbeta, dgamma = sums[:C], sums[C:]
        dx = (dyf - dbeta.view(shape) / n - xhat * dgamma.view(shape) / n) * (gamma.float() * invstd).view(shape)
        # parameter gradients are the LOCAL sums: the trainer's kvstore reduces them like any other grad
        return dx.to(dy.dtype), dgamma_local.to(gamma.dtype), dbeta_local.to(gamma.dtype), None, None


@register('_contrib_SyncBatchNorm', aliases=('SyncBatchNorm',), arg_names=('data', 'gamma', 'beta'),
          aux_names=('moving_mean', 'moving_var'), num_outputs=3,
          num_visible_outputs=lambda a: 3 if str(a.get('output_mean_var', False)) in ('True', 'true', '1') else 1,
          infer_params=lambda s, a: {} if s[0] is None else {i: (s[0][1],) for i in (1, 2, 3, 4)},
          params={'eps': ('float', 1e-3), 'momentum': ('float', 0.9), 'fix_gamma': ('bool', True),
                  'use_global_stats': ('bool', False), 'output_mean_var': ('bool', False), 'ndev': ('int', 1),
                  'key': ('str', ''), 'axis': ('int', 1)})
def sync_batch_norm(data, gamma, beta, moving_mean, moving_var, eps=1e-3, momentum=0.9, fix_gamma=True,
                    use_global_stats=False, output_mean_var=False, ndev=1, key='', axis=1):
    axis = axis % data.dim()
    g = torch.ones_like(gamma) if fix_gamma else gamma
    if _state.STATE.training and not use_global_stats:
        y, mean, var = _SyncBN.apply(data, g, beta, eps, axis)
        with torch.no_grad():
            moving_mean.mul_(momentum).add_(mean.to(moving_mean.dtype), alpha=1 - momentum)
            moving_var.mul_(momentum).add_(var.to(moving_var.dtype), alpha=1 - momentum)
        return y, mean, var
    shape = [1] * data.dim()
    shape[axis] = data.shape[axis]
    inv = torch.rsqrt(moving_var.float() + eps)
    y = (data.float() - moving_mean.float().view(shape)) * (inv * g.float()).view(shape) + beta.float().view(shape)
    return y.to(data.dtype), moving_mean, moving_var
