"""Long-tail operators and legacy operator names.

Parity (reference files):
* src/operator/nn/im2col.cc                          -- im2col / col2im
* src/operator/contrib/preloaded_multi_sgd.cc        -- preloaded_multi_(mp_)sgd(_mom)_update
* src/operator/contrib/adamw.cc                      -- _multi_adamw_update / _multi_mp_adamw_update
* src/operator/contrib/multi_lamb.cc                 -- _multi_lamb_update / _multi_mp_lamb_update
* src/operator/contrib/optimizer_op.cc               -- _contrib_group_adagrad_update
* src/operator/contrib/psroi_pooling.cc              -- _contrib_PSROIPooling (R-FCN)
* src/operator/contrib/deformable_psroi_pooling.cc   -- _contrib_DeformablePSROIPooling
* src/operator/contrib/rroi_align.cc                 -- _contrib_RROIAlign (rotated ROIAlign)
* src/operator/contrib/mrcnn_mask_target.cu          -- _contrib_mrcnn_mask_target
* src/operator/random/sample_op.cc, multisample_op.cc -- _sample_* (per-row parameters), _random_*_like
* src/operator/tensor/elemwise_*                      -- legacy CamelCase comparison / scalar op names
* src/operator/tensor/square_sum.cc, sparse_retain.cc, cast_storage.cc, elemwise_scatter_op.cc

These are torch-tensor implementations (gather/bilinear sampling vectorised over
rois x bins x samples); none of them is on a training hot path of the
benchmarked models.
"""
import math

import torch
import torch.nn.functional as F

from .registry import register, alias, has, get
from .optimizer_ops import (_sgd, _sgd_mom, _adamw, _lamb1, _lamb2, _floats, _MULTI)


# ---------------------------------------------------------------------------
# im2col / col2im
# ---------------------------------------------------------------------------

_IM2COL = {'kernel': ('shape', ()), 'stride': ('shape', ()), 'dilate': ('shape', ()), 'pad': ('shape', ())}


def _k_args(kernel, stride, dilate, pad):
    n = len(kernel)
    return (tuple(kernel), tuple(stride) or (1,) * n, tuple(dilate) or (1,) * n, tuple(pad) or (0,) * n)


@register('im2col', params=_IM2COL)
def im2col(data, kernel=(), stride=(), dilate=(), pad=()):
    """[N, C, H, W] -> [N, C*kh*kw, L] sliding blocks (channel-major, then kernel row/col)."""
    k, s, d, p = _k_args(kernel, stride, dilate, pad)
    if len(k) != 2:
        raise ValueError('im2col: only 2-D kernels are supported')
    return F.unfold(data, k, dilation=d, padding=p, stride=s)


@register('col2im', params=dict(_IM2COL, output_size=('shape', ())))
def col2im(data, output_size=(), kernel=(), stride=(), dilate=(), pad=()):
    """Inverse (sum of overlapping blocks) of im2col."""
    k, s, d, p = _k_args(kernel, stride, dilate, pad)
    return F.fold(data, tuple(output_size), k, dilation=d, padding=p, stride=s)


# ---------------------------------------------------------------------------
# optimizer multi-tensor forms
# ---------------------------------------------------------------------------

def _preloaded(per, stride):
    def names(a):
        n = int(a.get('num_weights', 1))
        base = ['weight', 'grad', 'mom', 'weight32'][:stride]
        return ['%s_%d' % (b, i) for i in range(n) for b in base] + ['lrs', 'wds']

    @torch.no_grad()
    def f(*tensors, momentum=0.0, rescale_grad=1.0, clip_gradient=-1.0, num_weights=1):
        lrs = tensors[-2].reshape(-1).float().tolist()
        wds = tensors[-1].reshape(-1).float().tolist()
        out = []
        for i in range(num_weights):
            g = tensors[i * stride:(i + 1) * stride]
            per(g, lrs[i], wds[i], momentum, rescale_grad, clip_gradient)
            out.append(g[0])
        return tuple(out)
    return names, f


_PRELOADED = {'momentum': ('float', 0.0), 'rescale_grad': ('float', 1.0), 'clip_gradient': ('float', -1.0),
              'num_weights': ('int', 1)}


def _nw(a):
    return int(a.get('num_weights', 1))


for _name, _per, _stride in [
        ('preloaded_multi_sgd_update', lambda g, lr, wd, m, rs, cl: _sgd(g[0], g[1], lr, wd, rs, cl), 2),
        ('preloaded_multi_sgd_mom_update',
         lambda g, lr, wd, m, rs, cl: _sgd_mom(g[0], g[1], g[2], lr, m, wd, rs, cl), 3),
        ('preloaded_multi_mp_sgd_update', lambda g, lr, wd, m, rs, cl: _sgd(g[0], g[1], lr, wd, rs, cl, w32=g[2]), 3),
        ('preloaded_multi_mp_sgd_mom_update',
         lambda g, lr, wd, m, rs, cl: _sgd_mom(g[0], g[1], g[2], lr, m, wd, rs, cl, w32=g[3]), 4)]:
    _names, _f = _preloaded(_per, _stride)
    register(_name, _f, arg_names=_names, params=_PRELOADED, num_outputs=_nw)


_MADAMW = {'lrs': ('any', ()), 'wds': ('any', ()), 'etas': ('any', ()), 'beta1': ('float', 0.9),
           'beta2': ('float', 0.999), 'epsilon': ('float', 1e-8), 'clip_gradient': ('float', -1.0),
           'num_weights': ('int', 1)}


def _multi_adamw(mp):
    stride = 5 if mp else 4

    def names(a):
        base = ['weight', 'grad', 'mean', 'var', 'weight32'][:stride]
        return ['%s_%d' % (b, i) for i in range(_nw(a)) for b in base] + ['rescale_grad']

    def f(*tensors, lrs=(), wds=(), etas=(), beta1=0.9, beta2=0.999, epsilon=1e-8, clip_gradient=-1.0,
          num_weights=1):
        lrs, wds, etas = _floats(lrs, num_weights), _floats(wds, num_weights), _floats(etas, num_weights)
        rs = tensors[-1]
        out = []
        for i in range(num_weights):
            g = tensors[i * stride:(i + 1) * stride]
            _adamw(g[0], g[1], g[2], g[3], rs, lrs[i], beta1, beta2, epsilon, wds[i], etas[i], clip_gradient,
                   w32=g[4] if mp else None)
            out.append(g[0])
        return tuple(out)
    return names, f


for _name, _mp in [('_multi_adamw_update', False), ('_multi_mp_adamw_update', True)]:
    _names, _f = _multi_adamw(_mp)
    register(_name, _f, arg_names=_names, params=_MADAMW, num_outputs=_nw,
             aliases=(_name.replace('_multi', '_contrib_multi', 1),))


_MLAMB = {'learning_rates': ('any', ()), 'wds': ('any', ()), 'beta1': ('float', 0.9), 'beta2': ('float', 0.999),
          'epsilon': ('float', 1e-6), 'rescale_grad': ('float', 1.0), 'lower_bound': ('float', -1.0),
          'upper_bound': ('float', -1.0), 'clip_gradient': ('float', -1.0), 'bias_correction': ('bool', True),
          'step_count': ('any', ()), 'num_tensors': ('int', 1)}


def _multi_lamb(mp):
    stride = 5 if mp else 4

    def names(a):
        base = ['weight', 'grad', 'mean', 'var', 'weight32'][:stride]
        return ['%s_%d' % (b, i) for i in range(int(a.get('num_tensors', 1))) for b in base]

    @torch.no_grad()
    def f(*tensors, learning_rates=(), wds=(), beta1=0.9, beta2=0.999, epsilon=1e-6, rescale_grad=1.0,
          lower_bound=-1.0, upper_bound=-1.0, clip_gradient=-1.0, bias_correction=True, step_count=(),
          num_tensors=1):
        lrs, wds_ = _floats(learning_rates, num_tensors), _floats(wds, num_tensors)
        steps = [int(s) for s in _floats(step_count, num_tensors)]
        out = []
        for i in range(num_tensors):
            g = tensors[i * stride:(i + 1) * stride]
            w = g[4] if mp else g[0]
            upd = _lamb1(w, g[1], g[2], g[3], beta1, beta2, epsilon, steps[i], bias_correction, wds_[i],
                         rescale_grad, clip_gradient)
            r1 = w.float().norm().reshape(1)
            r2 = upd.norm().reshape(1)
            _lamb2(g[0], upd, r1, r2, lrs[i], lower_bound, upper_bound, w32=g[4] if mp else None)
            out.append(g[0])
        return tuple(out)
    return names, f


for _name, _mp in [('_multi_lamb_update', False), ('_multi_mp_lamb_update', True)]:
    _names, _f = _multi_lamb(_mp)
    register(_name, _f, arg_names=_names, params=_MLAMB, num_outputs=lambda a: int(a.get('num_tensors', 1)),
             aliases=(_name.replace('_multi', '_contrib_multi', 1),))


@register('_contrib_group_adagrad_update', aliases=('group_adagrad_update',),
          arg_names=('weight', 'grad', 'history'),
          params={'lr': ('float', 0.01), 'rescale_grad': ('float', 1.0), 'clip_gradient': ('float', -1.0),
                  'epsilon': ('float', 1e-5)})
@torch.no_grad()
def group_adagrad_update(weight, grad, history, lr=0.01, rescale_grad=1.0, clip_gradient=-1.0, epsilon=1e-5):
    """Row-wise AdaGrad: one accumulator per row = running sum of the row's mean squared gradient."""
    g = grad.float() * rescale_grad
    if clip_gradient >= 0:
        g = torch.clamp(g, -clip_gradient, clip_gradient)
    g2 = g.reshape(g.shape[0], -1)
    history.add_(g2.pow(2).mean(1).reshape(history.shape).to(history.dtype))
    div = torch.sqrt(history.float().reshape(-1)) + epsilon
    weight.sub_((lr * g2 / div[:, None]).reshape(weight.shape).to(weight.dtype))
    return weight


@register('_sparse_adagrad_update', arg_names=('weight', 'grad', 'history'),
          params={'lr': ('float', 0.01), 'epsilon': ('float', 1e-7), 'wd': ('float', 0.0),
                  'rescale_grad': ('float', 1.0), 'clip_gradient': ('float', -1.0)})
@torch.no_grad()
def sparse_adagrad_update(weight, grad, history, lr=0.01, epsilon=1e-7, wd=0.0, rescale_grad=1.0, clip_gradient=-1.0):
    """AdaGrad touching only rows with a non-zero gradient (row_sparse semantics on dense storage)."""
    g = grad.float() * rescale_grad
    if clip_gradient >= 0:
        g = torch.clamp(g, -clip_gradient, clip_gradient)
    rows = g.reshape(g.shape[0], -1).abs().sum(1) != 0
    gr = g[rows] + wd * weight[rows].float()
    history[rows] += gr * gr
    weight[rows] -= (lr * gr / (torch.sqrt(history[rows].float()) + epsilon)).to(weight.dtype)
    return weight


# ---------------------------------------------------------------------------
# position-sensitive / rotated ROI ops
# ---------------------------------------------------------------------------

def _bilinear(img, y, x):
    """Caffe2/Detectron bilinear sample of img[C, H, W] at float coords y, x (same shape S) -> [C, *S]."""
    H, W = img.shape[-2:]
    out_of = (y < -1.0) | (y > H) | (x < -1.0) | (x > W)
    y = y.clamp(min=0)
    x = x.clamp(min=0)
    y0 = y.floor().long()
    x0 = x.floor().long()
    ylast = y0 >= H - 1
    xlast = x0 >= W - 1
    y0 = torch.where(ylast, torch.full_like(y0, H - 1), y0)
    x0 = torch.where(xlast, torch.full_like(x0, W - 1), x0)
    y = torch.where(ylast, y0.to(y.dtype), y)
    x = torch.where(xlast, x0.to(x.dtype), x)
    y1 = torch.where(ylast, y0, y0 + 1)
    x1 = torch.where(xlast, x0, x0 + 1)
    ly, lx = y - y0, x - x0
    hy, hx = 1 - ly, 1 - lx
    flat = img.reshape(img.shape[0], -1)

    def g(yy, xx):
        return flat[:, (yy * W + xx).reshape(-1)].reshape((img.shape[0],) + tuple(yy.shape))
    v = hy * hx * g(y0, x0) + hy * lx * g(y0, x1) + ly * hx * g(y1, x0) + ly * lx * g(y1, x1)
    return torch.where(out_of, torch.zeros_like(v), v)


@register('_contrib_PSROIPooling', aliases=('PSROIPooling',), arg_names=('data', 'rois'),
          params={'spatial_scale': ('float', 1.0), 'output_dim': ('int', 0), 'pooled_size': ('int', 0),
                  'group_size': ('int', 0)})
def psroi_pooling(data, rois, spatial_scale=1.0, output_dim=0, pooled_size=0, group_size=0):
    """R-FCN position-sensitive average pooling: output channel c, bin (i, j) averages input
    channel (c*G + gi)*G + gj over the bin."""
    P = pooled_size
    G = group_size or P
    N, C, H, W = data.shape
    out = data.new_zeros(rois.shape[0], output_dim, P, P)
    ph = torch.arange(P, device=data.device, dtype=torch.float32)
    gidx = torch.clamp((ph * G / P).floor().long(), 0, G - 1)
    for r in range(rois.shape[0]):
        roi = rois[r].float()
        b = int(roi[0])
        sw, sh = torch.round(roi[1]) * spatial_scale, torch.round(roi[2]) * spatial_scale
        ew, eh = (torch.round(roi[3]) + 1.) * spatial_scale, (torch.round(roi[4]) + 1.) * spatial_scale
        rw, rh = torch.clamp(ew - sw, min=0.1), torch.clamp(eh - sh, min=0.1)
        bh, bw = rh / P, rw / P
        hs = torch.clamp((ph * bh + sh).floor(), 0, H).long()
        he = torch.clamp(((ph + 1) * bh + sh).ceil(), 0, H).long()
        ws = torch.clamp((ph * bw + sw).floor(), 0, W).long()
        we = torch.clamp(((ph + 1) * bw + sw).ceil(), 0, W).long()
        for i in range(P):
            for j in range(P):
                if he[i] <= hs[i] or we[j] <= ws[j]:
                    continue
                ch = (torch.arange(output_dim, device=data.device) * G + gidx[i]) * G + gidx[j]
                blk = data[b, ch, hs[i]:he[i], ws[j]:we[j]]
                out[r, :, i, j] = blk.float().mean((1, 2)).to(out.dtype)
    return out


@register('_contrib_DeformablePSROIPooling', aliases=('DeformablePSROIPooling',),
          arg_names=lambda a: ['data', 'rois'] if str(a.get('no_trans', 'False')) in ('True', 'true', '1')
          else ['data', 'rois', 'trans'], num_outputs=2, num_visible_outputs=1,
          params={'spatial_scale': ('float', 1.0), 'output_dim': ('int', 0), 'group_size': ('int', 0),
                  'pooled_size': ('int', 0), 'part_size': ('int', 0), 'sample_per_part': ('int', 1),
                  'trans_std': ('float', 0.0), 'no_trans': ('bool', False)})
def deformable_psroi_pooling(data, rois, trans=None, spatial_scale=1.0, output_dim=0, group_size=0, pooled_size=0,
                             part_size=0, sample_per_part=1, trans_std=0.0, no_trans=False):
    """Deformable R-FCN pooling: per-part learned offsets shift each bin, which is averaged from
    sample_per_part^2 bilinear samples.  Returns (output, top_count)."""
    P, G = pooled_size, group_size
    part = part_size or P
    S = sample_per_part
    dev = data.device
    R = rois.shape[0]
    N, C, H, W = data.shape
    no_trans = no_trans or trans is None
    ncls = 1 if no_trans else trans.shape[1] // 2
    ch_each = output_dim if no_trans else output_dim // ncls
    out = torch.zeros(R, output_dim, P, P, device=dev, dtype=torch.float32)
    cnt = torch.zeros_like(out)
    pi = torch.arange(P, device=dev, dtype=torch.float32)
    ctop = torch.arange(output_dim, device=dev)
    gh = torch.clamp((pi * G / P).floor().long(), 0, G - 1)
    parts = (pi / P * part).floor().long()
    s = torch.arange(S, device=dev, dtype=torch.float32)
    for r in range(R):
        roi = rois[r].float()
        b = int(roi[0])
        sw, sh = torch.round(roi[1]) * spatial_scale - 0.5, torch.round(roi[2]) * spatial_scale - 0.5
        ew, eh = (torch.round(roi[3]) + 1.) * spatial_scale - 0.5, (torch.round(roi[4]) + 1.) * spatial_scale - 0.5
        rw, rh = torch.clamp(ew - sw, min=0.1), torch.clamp(eh - sh, min=0.1)
        bh, bw = rh / P, rw / P
        cls_id = ctop // ch_each                                                     # [D]
        if no_trans:
            tx = torch.zeros(output_dim, P, P, device=dev)
            ty = torch.zeros(output_dim, P, P, device=dev)
        else:
            t = trans[r].float()                                                     # [2*ncls, part, part]
            tx = t[(cls_id * 2)[:, None, None], parts[None, :, None], parts[None, None, :]] * trans_std
            ty = t[(cls_id * 2 + 1)[:, None, None], parts[None, :, None], parts[None, None, :]] * trans_std
        wstart = pi[None, None, :] * bw + sw + tx * rw                              # [D, P(h), P(w)]
        hstart = pi[None, :, None] * bh + sh + ty * rh
        hh = hstart[..., None, None] + s[:, None] * (bh / S)                        # [D, P, P, S, 1]
        ww = wstart[..., None, None] + s[None, :] * (bw / S)                        # [D, P, P, 1, S]
        hh, ww = torch.broadcast_tensors(hh, ww)
        valid = (ww >= -0.5) & (ww <= W - 0.5) & (hh >= -0.5) & (hh <= H - 0.5)
        wc = ww.clamp(0, W - 1)
        hc = hh.clamp(0, H - 1)
        ch = (ctop[:, None, None] * G + gh[None, :, None]) * G + gh[None, None, :]   # [D, P, P]
        img = data[b].float()
        y0, x0 = hc.floor().long(), wc.floor().long()
        y1, x1 = (y0 + 1).clamp(max=H - 1), (x0 + 1).clamp(max=W - 1)
        ly, lx = hc - y0, wc - x0
        chx = ch[..., None, None].expand_as(y0)

        def g(yy, xx):
            return img[chx, yy, xx]
        v = (1 - ly) * (1 - lx) * g(y0, x0) + (1 - ly) * lx * g(y0, x1) + ly * (1 - lx) * g(y1, x0) + \
            ly * lx * g(y1, x1)
        v = torch.where(valid, v, torch.zeros_like(v))
        n = valid.float().sum((-1, -2))
        out[r] = torch.where(n > 0, v.sum((-1, -2)) / n.clamp(min=1), torch.zeros_like(n))
        cnt[r] = n
    return out.to(data.dtype), cnt.to(data.dtype)


@register('_contrib_RROIAlign', aliases=('RROIAlign',), arg_names=('data', 'rois'),
          params={'pooled_size': ('shape', ()), 'spatial_scale': ('float', 1.0), 'sampling_ratio': ('int', -1)})
def rroi_align(data, rois, pooled_size=(), spatial_scale=1.0, sampling_ratio=-1):
    """Rotated ROIAlign: rois are (batch, cx, cy, w, h, theta_degrees)."""
    PH, PW = pooled_size
    R = rois.shape[0]
    N, C, H, W = data.shape
    out = data.new_zeros(R, C, PH, PW)
    for r in range(R):
        roi = rois[r].float()
        b = int(roi[0])
        cw, chh = roi[1] * spatial_scale, roi[2] * spatial_scale
        rw = torch.clamp(roi[3] * spatial_scale, min=1.0)
        rh = torch.clamp(roi[4] * spatial_scale, min=1.0)
        th = roi[5] * math.pi / 180.0
        bh, bw = rh / PH, rw / PW
        gh = sampling_ratio if sampling_ratio > 0 else int(math.ceil(float(rh) / PH))
        gw = sampling_ratio if sampling_ratio > 0 else int(math.ceil(float(rw) / PW))
        ph = torch.arange(PH, device=data.device, dtype=torch.float32)
        pw = torch.arange(PW, device=data.device, dtype=torch.float32)
        iy = torch.arange(gh, device=data.device, dtype=torch.float32)
        ix = torch.arange(gw, device=data.device, dtype=torch.float32)
        yy = -rh / 2 + ph[:, None, None, None] * bh + (iy[None, None, :, None] + .5) * bh / gh   # [PH,1,gh,1]
        xx = -rw / 2 + pw[None, :, None, None] * bw + (ix[None, None, None, :] + .5) * bw / gw   # [1,PW,1,gw]
        yy, xx = torch.broadcast_tensors(yy, xx)
        c, s_ = torch.cos(th), torch.sin(th)
        x = xx * c + yy * s_ + cw
        y = yy * c - xx * s_ + chh
        v = _bilinear(data[b].float(), y, x)                                        # [C, PH, PW, gh, gw]
        out[r] = (v.sum((-1, -2)) / (gh * gw)).to(out.dtype)
    return out


@register('_contrib_mrcnn_mask_target', aliases=('mrcnn_mask_target',),
          arg_names=('rois', 'gt_masks', 'matches', 'cls_targets'), num_outputs=2,
          params={'num_rois': ('int', 0), 'num_classes': ('int', 0), 'mask_size': ('shape', ()),
                  'sample_ratio': ('int', 2), 'aligned': ('bool', False)})
def mrcnn_mask_target(rois, gt_masks, matches, cls_targets, num_rois=0, num_classes=0, mask_size=(),
                      sample_ratio=2, aligned=False):
    """Mask R-CNN targets: ROIAlign of each roi's matched gt mask at mask_size (broadcast over
    classes) and the per-class one-hot mask weights.  Returns ([B,N,C,h,w], [B,N,C,h,w])."""
    B, N = rois.shape[:2]
    Hm, Wm = gt_masks.shape[-2:]
    mh, mw = mask_size
    off = 0.5 if aligned else 0.0
    dev = rois.device
    ph = torch.arange(mh, device=dev, dtype=torch.float32)
    pw = torch.arange(mw, device=dev, dtype=torch.float32)
    masks = torch.zeros(B, N, mh, mw, device=dev)
    for b in range(B):
        for n in range(N):
            r = rois[b, n].float() - off
            rw, rh = r[2] - r[0], r[3] - r[1]
            if not aligned:
                rw, rh = torch.clamp(rw, min=1.0), torch.clamp(rh, min=1.0)
            bh, bw = rh / mh, rw / mw
            gh = sample_ratio if sample_ratio > 0 else int(math.ceil(float(rh) / mh))
            gw = sample_ratio if sample_ratio > 0 else int(math.ceil(float(rw) / mw))
            iy = torch.arange(gh, device=dev, dtype=torch.float32)
            ix = torch.arange(gw, device=dev, dtype=torch.float32)
            y = r[1] + ph[:, None, None, None] * bh + (iy[None, None, :, None] + .5) * bh / gh
            x = r[0] + pw[None, :, None, None] * bw + (ix[None, None, None, :] + .5) * bw / gw
            y, x = torch.broadcast_tensors(y, x)
            img = gt_masks[b, int(matches[b, n])].float()[None]
            masks[b, n] = _bilinear(img, y, x)[0].sum((-1, -2)) / (gh * gw)
    cls = torch.arange(num_classes, device=dev, dtype=torch.float32)
    mask_cls = (cls_targets.float()[:, :, None] == cls[None, None, :]).float()
    out_masks = masks[:, :, None].expand(B, N, num_classes, mh, mw).contiguous()
    out_cls = mask_cls[..., None, None].expand(B, N, num_classes, mh, mw).contiguous()
    return out_masks.to(rois.dtype), out_cls.to(rois.dtype)


# ---------------------------------------------------------------------------
# random: per-row parameter sampling and *_like forms
# ---------------------------------------------------------------------------

def _sample(draw, nparams):
    def f(*params, shape=(), dtype='None'):
        p0 = params[0]
        s = tuple(shape) if shape else ()
        ext = (1,) * len(s)
        full = tuple(p0.shape) + s
        ps = [p.reshape(tuple(p.shape) + ext).expand(full).float() for p in params]
        out = draw(*ps)
        return out.to(p0.dtype if dtype in ('None', None) else getattr(torch, dtype))
    return f


def _gamma(alpha, beta):
    return torch._standard_gamma(alpha) * beta


def _negbin(k, p):
    return torch.poisson(torch._standard_gamma(k) * (1 - p) / p)


def _gennegbin(mu, alpha):
    """Gamma-Poisson mixture with mean mu and dispersion alpha (alpha = 0: Poisson(mu)); either
    argument may be a scalar (the *_like samplers) or a per-element tensor."""
    mu_t = mu if torch.is_tensor(mu) else torch.tensor(float(mu))
    al_t = alpha if torch.is_tensor(alpha) else torch.full_like(mu_t, float(alpha))
    safe = torch.where(al_t > 0, al_t, torch.ones_like(al_t))
    rate = torch.where(al_t > 0, torch._standard_gamma(1.0 / safe) * mu_t * safe, mu_t.expand_as(safe))
    return torch.poisson(rate)


for _name, _args, _draw in [
        ('_sample_exponential', ('lam',), lambda lam: torch.empty_like(lam).exponential_() / lam),
        ('_sample_gamma', ('alpha', 'beta'), _gamma),
        ('_sample_poisson', ('lam',), torch.poisson),
        ('_sample_negative_binomial', ('k', 'p'), _negbin),
        ('_sample_generalized_negative_binomial', ('mu', 'alpha'), _gennegbin)]:
    register(_name, _sample(_draw, len(_args)), arg_names=_args, aliases=(_name[1:],),
             params={'shape': ('shape', ()), 'dtype': ('str', 'None')})


def _like(name, draw, params):
    def f(data, **kw):
        return draw(torch.empty(data.shape, device=data.device, dtype=torch.float32), **kw).to(data.dtype)
    register(name, f, params=params)


_like('_random_exponential_like', lambda t, lam=1.0: t.exponential_(lam), {'lam': ('float', 1.0)})
_like('_random_gamma_like', lambda t, alpha=1.0, beta=1.0: torch._standard_gamma(t.fill_(alpha)) * beta,
      {'alpha': ('float', 1.0), 'beta': ('float', 1.0)})
_like('_random_poisson_like', lambda t, lam=1.0: torch.poisson(t.fill_(lam)), {'lam': ('float', 1.0)})
_like('_random_negative_binomial_like', lambda t, k=1, p=1.0: _negbin(t.fill_(float(k)), p),
      {'k': ('int', 1), 'p': ('float', 1.0)})
_like('_random_generalized_negative_binomial_like',
      lambda t, mu=1.0, alpha=1.0: _gennegbin(t.fill_(mu), alpha),
      {'mu': ('float', 1.0), 'alpha': ('float', 1.0)})


@register('_sample_unique_zipfian', arg_names=(), num_outputs=2,
          params={'range_max': ('int', 1), 'shape': ('shape', ())})
def sample_unique_zipfian(range_max=1, shape=()):
    """Log-uniform (Zipfian) candidate sampling without replacement per row; returns (samples, num_tries)."""
    rows, k = (shape[0], shape[1]) if len(shape) == 2 else (1, shape[0])
    log_range = math.log(range_max + 1)
    out = torch.empty(rows, k, dtype=torch.int64)
    tries = torch.empty(rows, dtype=torch.int64)
    for r in range(rows):
        seen, n = [], 0
        sset = set()
        while len(seen) < k:
            v = int(math.exp(torch.rand(()).item() * log_range)) - 1
            v = min(max(v, 0), range_max - 1)
            n += 1
            if v not in sset:
                sset.add(v)
                seen.append(v)
        out[r] = torch.tensor(seen)
        tries[r] = n
    return out.reshape(tuple(shape)), tries


# ---------------------------------------------------------------------------
# misc tensor ops
# ---------------------------------------------------------------------------

@register('_square_sum', aliases=('square_sum',), params={'axis': ('shape', None), 'keepdims': ('bool', False),
                                                           'exclude': ('bool', False)})
def square_sum(data, axis=None, keepdims=False, exclude=False):
    d = data.float() ** 2
    if axis is None or axis == ():
        return d.sum().reshape(1).to(data.dtype) if not keepdims else d.sum().reshape((1,) * data.dim()).to(data.dtype)
    ax = tuple(a % data.dim() for a in (axis if isinstance(axis, (tuple, list)) else (axis,)))
    if exclude:
        ax = tuple(i for i in range(data.dim()) if i not in ax)
    return d.sum(ax, keepdim=keepdims).to(data.dtype)


@register('_grad_add', arg_names=('lhs', 'rhs'))
def grad_add(lhs, rhs):
    return lhs + rhs


@register('_identity_with_attr_like_rhs', arg_names=('lhs', 'rhs'))
def identity_with_attr_like_rhs(lhs, rhs):
    return lhs


@register('_CrossDeviceCopy')
def cross_device_copy(data):
    return data.clone()


@register('_zeros_without_dtype', arg_names=(), params={'shape': ('shape', ()), 'ctx': ('str', ''),
                                                        'dtype': ('int', -1)})
def zeros_without_dtype(shape=(), ctx='', dtype=-1):
    return torch.zeros(tuple(shape) or (1,))


@register('_scatter_elemwise_div', arg_names=('lhs', 'rhs'))
def scatter_elemwise_div(lhs, rhs):
    """lhs / rhs evaluated only where lhs is non-zero (sparse-lhs semantics; zeros stay zero)."""
    return torch.where(lhs != 0, lhs / rhs, torch.zeros_like(lhs))


@register('_scatter_plus_scalar', params={'scalar': ('float', 0.0)})
def scatter_plus_scalar(data, scalar=0.0):
    return torch.where(data != 0, data + scalar, data)


@register('_scatter_minus_scalar', params={'scalar': ('float', 0.0)})
def scatter_minus_scalar(data, scalar=0.0):
    return torch.where(data != 0, data - scalar, data)


# ---------------------------------------------------------------------------
# legacy / alternative operator names (old -symbol.json files and mx.nd aliases)
# ---------------------------------------------------------------------------

_LEGACY = {
    '_equal': ['_Equal', 'equal'], '_not_equal': ['_Not_Equal', 'not_equal'], '_greater': ['_Greater', 'greater'],
    '_greater_equal': ['_Greater_Equal', 'greater_equal'], '_lesser': ['_Lesser', 'less', 'lesser'],
    '_lesser_equal': ['_Lesser_Equal', 'less_equal', 'lesser_equal'],
    '_logical_and': ['_Logical_And'], '_logical_or': ['_Logical_Or'], '_logical_xor': ['_Logical_Xor'],
    '_equal_scalar': ['_EqualScalar'], '_not_equal_scalar': ['_NotEqualScalar'],
    '_greater_scalar': ['_GreaterScalar'], '_greater_equal_scalar': ['_GreaterEqualScalar'],
    '_lesser_scalar': ['_LesserScalar'], '_lesser_equal_scalar': ['_LesserEqualScalar'],
    '_logical_and_scalar': ['_LogicalAndScalar'], '_logical_or_scalar': ['_LogicalOrScalar'],
    '_logical_xor_scalar': ['_LogicalXorScalar'], '_maximum_scalar': ['_MaximumScalar'],
    '_minimum_scalar': ['_MinimumScalar'], '_mod_scalar': ['_ModScalar'], '_rmod_scalar': ['_RModScalar'],
    '_power_scalar': ['_PowerScalar'], '_rpower_scalar': ['_RPowerScalar'], '_hypot_scalar': ['_HypotScalar'],
    '_random_exponential': ['random_exponential', 'exponential'], '_random_gamma': ['random_gamma', 'gamma_sample'],
    '_random_poisson': ['random_poisson', 'poisson'],
    '_random_negative_binomial': ['random_negative_binomial', 'negative_binomial'],
    '_random_generalized_negative_binomial': ['random_generalized_negative_binomial',
                                              'generalized_negative_binomial'],
    '_random_randint': ['random_randint'],
    'pick': ['choose_element_0index'],
    '_contrib_SparseEmbedding': [],
}
for _src, _names in _LEGACY.items():
    if has(_src):
        for _a in _names:
            if not has(_a):
                alias(_src, _a)

@register('cast_storage', aliases=('_cast_storage',), params={'stype': ('str', 'default')})
def cast_storage_op(data, stype='default'):
    """Graph form of cast_storage: storage is dense in a graph; the value is unchanged."""
    return data


@register('_sparse_retain', aliases=('_retain',), arg_names=('data', 'indices'))
def sparse_retain(data, indices):
    """Keep the rows listed in ``indices`` (row_sparse retain), zero the others."""
    keep = torch.zeros(data.shape[0], dtype=torch.bool, device=data.device)
    keep[indices.long().reshape(-1)] = True
    return torch.where(keep.reshape((-1,) + (1,) * (data.dim() - 1)), data, torch.zeros_like(data))


if not has('_contrib_SparseEmbedding') and has('Embedding'):
    alias('Embedding', '_contrib_SparseEmbedding')
for _src, _dst in [('_cast_storage', 'cast_storage'), ('cast_storage', '_cast_storage'),
                   ('_retain', '_sparse_retain'), ('retain', '_sparse_retain'), ('_sparse_retain', 'retain')]:
    if has(_src) and not has(_dst):
        alias(_src, _dst)

# numpy-extension operator names (the symbols mx.npx.* records in a hybridized np-mode graph)
_NPX = {'relu': 'relu', 'sigmoid': 'sigmoid', 'softmax': 'softmax', 'log_softmax': 'log_softmax',
        'activation': 'Activation', 'batch_norm': 'BatchNorm', 'convolution': 'Convolution',
        'deconvolution': 'Deconvolution', 'fully_connected': 'FullyConnected', 'pooling': 'Pooling',
        'dropout': 'Dropout', 'embedding': 'Embedding', 'layer_norm': 'LayerNorm', 'leaky_relu': 'LeakyReLU',
        'rnn': 'RNN', 'one_hot': 'one_hot', 'pick': 'pick', 'topk': 'topk', 'sequence_mask': 'SequenceMask',
        'batch_dot': 'batch_dot', 'batch_flatten': 'Flatten', 'reshape_like': 'reshape_like',
        'shape_array': 'shape_array', 'smooth_l1': 'smooth_l1', 'erf': 'erf', 'erfinv': 'erfinv',
        'gamma': 'gamma', 'gammaln': 'gammaln', 'gather_nd': 'gather_nd', 'cast': 'Cast', 'slice': 'slice',
        'arange_like': '_contrib_arange_like', 'nonzero': '_npx_nonzero_impl', 'roi_pooling': 'ROIPooling',
        'multibox_prior': '_contrib_MultiBoxPrior', 'multibox_target': '_contrib_MultiBoxTarget',
        'multibox_detection': '_contrib_MultiBoxDetection'}
for _n, _src in _NPX.items():
    if has(_src) and not has('_npx_' + _n):
        alias(_src, '_npx_' + _n)
_IMG = ['adjust_lighting', 'crop', 'flip_left_right', 'flip_top_bottom', 'normalize', 'random_brightness',
        'random_color_jitter', 'random_contrast', 'random_flip_left_right', 'random_flip_top_bottom', 'random_hue',
        'random_lighting', 'random_saturation', 'resize', 'to_tensor']
for _n in _IMG:
    if has('_image_' + _n) and not has('_npx__image_' + _n):
        alias('_image_' + _n, '_npx__image_' + _n)


@register('_npx_nonzero_impl', aliases=('_npi_nonzero',))
def _nonzero(data):
    return torch.nonzero(data).to(torch.int64)


if not has('_npx_nonzero'):
    alias('_npx_nonzero_impl', '_npx_nonzero')
