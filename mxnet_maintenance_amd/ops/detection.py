"""Object-detection operators (parity: src/operator/contrib/{multibox_prior,multibox_target,
multibox_detection,bounding_box,roi_align,proposal,multi_proposal}*).

SSD anchors/targets/decoding, NMS, IoU, bipartite matching, box encode/decode,
ROIAlign and the Faster-RCNN RPN proposal op.  Data-dependent control flow
(greedy matching, NMS) runs per image over sorted candidates; the dense parts
(IoU matrices, decoding, bilinear ROI sampling) are batched tensor ops.
"""
import math

import torch
import torch.nn.functional as F

from .registry import register


def _corner(b, fmt):
    if fmt == 'center':
        x, y, w, h = b.unbind(-1)
        return torch.stack([x - w / 2, y - h / 2, x + w / 2, y + h / 2], -1)
    return b


def _center(b):
    x1, y1, x2, y2 = b.unbind(-1)
    return torch.stack([(x1 + x2) / 2, (y1 + y2) / 2, x2 - x1, y2 - y1], -1)


def _iou(a, b):
    """a [..., N, 4], b [..., M, 4] corner boxes -> [..., N, M]."""
    lt = torch.maximum(a[..., :, None, :2], b[..., None, :, :2])
    rb = torch.minimum(a[..., :, None, 2:], b[..., None, :, 2:])
    wh = torch.clamp(rb - lt, min=0)
    inter = wh[..., 0] * wh[..., 1]
    area_a = torch.clamp(a[..., 2] - a[..., 0], min=0) * torch.clamp(a[..., 3] - a[..., 1], min=0)
    area_b = torch.clamp(b[..., 2] - b[..., 0], min=0) * torch.clamp(b[..., 3] - b[..., 1], min=0)
    union = area_a[..., :, None] + area_b[..., None, :] - inter
    return torch.where(union > 0, inter / union, torch.zeros_like(union))


# ---------------------------------------------------------------------------
# SSD
# ---------------------------------------------------------------------------

@register('_contrib_MultiBoxPrior', aliases=('MultiBoxPrior',),
          params={'sizes': ('floats', (1.0,)), 'ratios': ('floats', (1.0,)), 'clip': ('bool', False),
                  'steps': ('floats', (-1.0, -1.0)), 'offsets': ('floats', (0.5, 0.5))})
def multibox_prior(data, sizes=(1.0,), ratios=(1.0,), clip=False, steps=(-1.0, -1.0), offsets=(0.5, 0.5)):
    H, W = data.shape[2], data.shape[3]
    step_y = steps[0] if steps[0] > 0 else 1.0 / H
    step_x = steps[1] if steps[1] > 0 else 1.0 / W
    dev = data.device
    cy = (torch.arange(H, device=dev, dtype=torch.float32) + offsets[0]) * step_y
    cx = (torch.arange(W, device=dev, dtype=torch.float32) + offsets[1]) * step_x
    whs = []
    r0 = math.sqrt(ratios[0]) if len(ratios) else 1.0
    for s in sizes:
        whs.append((s * H / W * r0 / 2, s / r0 / 2))
    for r in ratios[1:]:
        rr = math.sqrt(r)
        whs.append((sizes[0] * H / W * rr / 2, sizes[0] / rr / 2))
    wh = torch.tensor(whs, device=dev, dtype=torch.float32)          # [A, 2]
    cyy, cxx = torch.meshgrid(cy, cx, indexing='ij')
    c = torch.stack([cxx, cyy], -1).reshape(-1, 1, 2)                  # [HW, 1, 2]
    boxes = torch.cat([c - wh, c + wh], -1).reshape(1, -1, 4)
    if clip:
        boxes = boxes.clamp(0, 1)
    return boxes.to(data.dtype if data.is_floating_point() else torch.float32)


def _decode(loc, anchors, var, clip):
    aw = anchors[..., 2] - anchors[..., 0]
    ah = anchors[..., 3] - anchors[..., 1]
    ax = (anchors[..., 0] + anchors[..., 2]) / 2
    ay = (anchors[..., 1] + anchors[..., 3]) / 2
    ox = loc[..., 0] * var[0] * aw + ax
    oy = loc[..., 1] * var[1] * ah + ay
    ow = torch.exp(loc[..., 2] * var[2]) * aw / 2
    oh = torch.exp(loc[..., 3] * var[3]) * ah / 2
    out = torch.stack([ox - ow, oy - oh, ox + ow, oy + oh], -1)
    return out.clamp(0, 1) if clip else out


def _nms_rows(rows, thresh, force, topk, id_col=0, box_col=2):
    """rows [K, 6+] sorted by score desc, id<0 invalid; suppress in place (set id=-1)."""
    n = rows.shape[0]
    if topk > 0 and topk < n:
        rows[topk:, id_col] = -1
        n = topk
    if n == 0:
        return rows
    boxes = rows[:n, box_col:box_col + 4]
    iou = _iou(boxes, boxes)
    ids = rows[:n, id_col].clone()
    keep = ids >= 0
    iou_cpu = iou.cpu()
    ids_cpu = ids.cpu()
    keep_cpu = keep.cpu().clone()
    for i in range(n):
        if not keep_cpu[i]:
            continue
        same = (ids_cpu[i + 1:n] == ids_cpu[i]) if not force else torch.ones(n - i - 1, dtype=torch.bool)
        sup = (iou_cpu[i, i + 1:n] >= thresh) & same & keep_cpu[i + 1:n]
        keep_cpu[i + 1:n] &= ~sup
    kill = (~keep_cpu) & (ids_cpu >= 0)
    rows[:n, id_col] = torch.where(kill.to(rows.device), torch.full_like(rows[:n, id_col], -1), rows[:n, id_col])
    return rows


@register('_contrib_MultiBoxDetection', aliases=('MultiBoxDetection',), arg_names=('cls_prob', 'loc_pred', 'anchor'),
          params={'clip': ('bool', True), 'threshold': ('float', 0.01), 'background_id': ('int', 0),
                  'nms_threshold': ('float', 0.5), 'force_suppress': ('bool', False),
                  'variances': ('floats', (0.1, 0.1, 0.2, 0.2)), 'nms_topk': ('int', -1)})
def multibox_detection(cls_prob, loc_pred, anchor, clip=True, threshold=0.01, background_id=0, nms_threshold=0.5,
                       force_suppress=False, variances=(0.1, 0.1, 0.2, 0.2), nms_topk=-1):
    B, C, A = cls_prob.shape
    boxes = _decode(loc_pred.reshape(B, A, 4).float(), anchor.reshape(1, A, 4).float(), variances, clip)
    probs = cls_prob.float()
    fg = torch.cat([probs[:, :background_id], probs[:, background_id + 1:]], 1) if 0 <= background_id < C else probs
    score, cid = fg.max(1)                                              # [B, A]
    cid = cid.float()
    cid = torch.where(score < threshold, torch.full_like(cid, -1), cid)
    out = torch.full((B, A, 6), -1.0, device=cls_prob.device)
    for b in range(B):
        valid = cid[b] >= 0
        rows = torch.cat([cid[b, valid, None], score[b, valid, None], boxes[b, valid]], -1)
        if rows.shape[0] == 0:
            continue
        if 0 < nms_threshold <= 1:
            order = torch.argsort(rows[:, 1], descending=True, stable=True)
            rows = _nms_rows(rows[order].clone(), nms_threshold, force_suppress, nms_topk)
        out[b, :rows.shape[0]] = rows
    return out.to(cls_prob.dtype)


@register('_contrib_MultiBoxTarget', aliases=('MultiBoxTarget',), arg_names=('anchor', 'label', 'cls_pred'),
          num_outputs=3,
          params={'overlap_threshold': ('float', 0.5), 'ignore_label': ('float', -1.0),
                  'negative_mining_ratio': ('float', -1.0), 'negative_mining_thresh': ('float', 0.5),
                  'minimum_negative_samples': ('int', 0), 'variances': ('floats', (0.1, 0.1, 0.2, 0.2))})
def multibox_target(anchor, label, cls_pred, overlap_threshold=0.5, ignore_label=-1.0, negative_mining_ratio=-1.0,
                    negative_mining_thresh=0.5, minimum_negative_samples=0, variances=(0.1, 0.1, 0.2, 0.2)):
    """SSD target assignment.  GPU tensors run the gfx950 kernel (src/kernels/detection.hip,
    one workgroup per image); CPU tensors run the vectorised reference below."""
    anchors = anchor.reshape(-1, 4).float().contiguous()
    A = anchors.shape[0]
    B = label.shape[0]
    if anchor.is_cuda:
        from . import kernels as _K
        if _K.enabled() and _K.available():
            return _multibox_target_hip(_K.lib(), anchors, label, cls_pred, overlap_threshold, ignore_label,
                                        negative_mining_ratio, negative_mining_thresh, minimum_negative_samples,
                                        variances)
        from .hip_ops import _ALLOW_FALLBACK
        if not _ALLOW_FALLBACK:
            raise RuntimeError('MultiBoxTarget on GPU needs the HIP kernel extension: %s' % _K.load_error())
    dev = anchor.device
    loc_target = torch.zeros(B, A, 4, device=dev)
    loc_mask = torch.zeros(B, A, 4, device=dev)
    cls_target = torch.full((B, A), float(ignore_label), device=dev)
    anchors_c = anchors.cpu()
    for b in range(B):
        lab = label[b].float().cpu()
        inval = (lab[:, 0] == -1).nonzero()
        ng = int(inval[0]) if inval.numel() else lab.shape[0]      # valid gts end at the first class == -1
        if ng == 0:
            continue
        gt = lab[:ng]
        iou = _iou(anchors_c, gt[:, 1:5])                                # [A, G]
        match_iou = torch.full((A,), -1.0)
        match_gt = torch.full((A,), -1, dtype=torch.long)
        aflag = torch.full((A,), -1, dtype=torch.long)
        gflag = torch.zeros(ng, dtype=torch.bool)
        npos = 0
        for _ in range(ng):                                              # greedy bipartite stage
            w = iou.clone()
            w[aflag == 1] = -1
            w[:, gflag] = -1
            v, flat = w.reshape(-1).max(0)                               # first max in (anchor, gt) order
            if float(v) <= 1e-6:
                break
            j, k = divmod(int(flat), ng)
            match_iou[j], match_gt[j] = float(v), k
            aflag[j] = 1
            gflag[k] = True
            npos += 1
        best_iou, best_gt = _first_max(iou)
        if overlap_threshold > 0:
            free = aflag != 1
            match_iou = torch.where(free, best_iou, match_iou)
            match_gt = torch.where(free, best_gt, match_gt)
            newpos = free & (best_iou > overlap_threshold)
            aflag[newpos] = 1
            npos += int(newpos.sum())
        if negative_mining_ratio > 0:
            nneg = min(int(npos * negative_mining_ratio), A - npos)
            nneg = max(nneg, min(minimum_negative_samples, A - npos))
            if nneg > 0:
                unset = match_iou < 0
                match_iou = torch.where(unset, best_iou, match_iou)
                match_gt = torch.where(unset, best_gt, match_gt)
                logits = cls_pred[b].float().cpu()                       # [C, A]
                p_bg = torch.softmax(logits, 0)[0]
                cand = (match_iou < negative_mining_thresh) & (aflag == -1)
                idx = torch.nonzero(cand).reshape(-1)
                order = torch.argsort(p_bg[idx], stable=True)            # lowest background prob = hardest
                aflag[idx[order[:nneg]]] = 0
        else:
            aflag[aflag != 1] = 0
        pos = aflag == 1
        neg = aflag == 0
        if pos.any():
            g = gt[match_gt[pos]].to(dev)
            a = anchors[pos.to(dev)]
            aw, ah = a[:, 2] - a[:, 0], a[:, 3] - a[:, 1]
            ax, ay = (a[:, 0] + a[:, 2]) / 2, (a[:, 1] + a[:, 3]) / 2
            gw, gh = g[:, 3] - g[:, 1], g[:, 4] - g[:, 2]
            gx, gy = (g[:, 1] + g[:, 3]) / 2, (g[:, 2] + g[:, 4]) / 2
            t = torch.stack([(gx - ax) / aw / variances[0], (gy - ay) / ah / variances[1],
                             torch.log(gw / aw) / variances[2], torch.log(gh / ah) / variances[3]], -1)
            loc_target[b, pos.to(dev)] = t
            loc_mask[b, pos.to(dev)] = 1
            cls_target[b, pos.to(dev)] = g[:, 0] + 1
        cls_target[b, neg.to(dev)] = 0
    return loc_target.reshape(B, -1), loc_mask.reshape(B, -1), cls_target


def _first_max(m):
    """Row-wise max and the FIRST column attaining it (the reference's strict '>' scan)."""
    v = m.max(1).values
    hit = m == v[:, None]
    idx = torch.argmax(hit.to(torch.uint8), 1)
    return v, idx


def _multibox_target_hip(lib, anchors, label, cls_pred, thr, ignore_label, ratio, neg_thresh, min_neg, var):
    from .kernel_fns import _DT, _stream
    B, L, W = label.shape
    A = anchors.shape[0]
    dev = anchors.device
    lab = label.float().contiguous()
    cp = cls_pred.contiguous()
    if cp.dtype not in _DT:
        cp = cp.float()
    if tuple(cp.shape) != (B, cp.shape[1], A):
        raise ValueError('MultiBoxTarget: cls_pred must be [batch, classes, anchors], got %s' % (tuple(cp.shape),))
    loc_target = torch.empty(B, A * 4, device=dev)
    loc_mask = torch.empty(B, A * 4, device=dev)
    cls_target = torch.empty(B, A, device=dev)
    scratch = torch.empty(3, B, A, dtype=torch.int32, device=dev)
    lib.multibox_target(_DT[cp.dtype], anchors.data_ptr(), lab.data_ptr(), cp.data_ptr(), loc_target.data_ptr(),
                        loc_mask.data_ptr(), cls_target.data_ptr(), scratch[0].data_ptr(), scratch[1].data_ptr(),
                        scratch[2].data_ptr(), B, A, L, W, cp.shape[1], float(thr), float(ignore_label), float(ratio),
                        float(neg_thresh), int(min_neg), float(var[0]), float(var[1]), float(var[2]), float(var[3]),
                        _stream())
    return loc_target, loc_mask, cls_target


# ---------------------------------------------------------------------------
# fused SSD training loss
# ---------------------------------------------------------------------------

def _ssd_loss_reference(cls_preds, loc_preds, cls_t, loc_t, loc_m, lambd):
    """fp32 composition (CPU / fallback): softmax-CE over anchors with ignore label -1 normalised by the
    valid anchors + smooth-L1 (sigma 1) of the masked location offsets normalised by the positives."""
    logp = torch.log_softmax(cls_preds.float(), dim=-1)
    valid = cls_t >= 0
    pick = logp.gather(-1, cls_t.clamp(min=0).long().unsqueeze(-1)).squeeze(-1)
    ce = (-pick * valid).sum()
    nvalid = valid.sum().clamp(min=1)
    npos = (cls_t > 0).sum().clamp(min=1)
    d = (loc_preds.float() - loc_t) * loc_m
    ad = d.abs()
    sl1 = torch.where(ad < 1, 0.5 * d * d, ad - 0.5).sum()
    return ce / nvalid + lambd * sl1 / npos


class _SSDLossHip(torch.autograd.Function):
    """One pass over the anchor rows for the loss, one for both gradients (detection.hip ssd_loss_*)."""

    @staticmethod
    def forward(ctx, cls_preds, loc_preds, cls_t, loc_t, loc_m, lambd):
        from . import kernels as _K
        from .kernel_fns import _DT, _stream
        lib = _K.lib()
        C1 = cls_preds.shape[-1]
        rows = cls_t.numel()
        cls_preds, loc_preds = cls_preds.contiguous(), loc_preds.contiguous()
        cls_t, loc_t, loc_m = cls_t.float().contiguous(), loc_t.float().contiguous(), loc_m.float().contiguous()
        part = torch.empty(4 * lib.ssd_loss_blocks(rows), dtype=torch.float32, device=cls_preds.device)
        out = torch.empty(3, dtype=torch.float32, device=cls_preds.device)
        lib.ssd_loss_fwd(_DT[cls_preds.dtype], cls_preds.data_ptr(), loc_preds.data_ptr(), cls_t.data_ptr(),
                         loc_t.data_ptr(), loc_m.data_ptr(), rows, C1, float(lambd), part.data_ptr(), out.data_ptr(),
                         _stream())
        ctx.save_for_backward(cls_preds, loc_preds, cls_t, loc_t, loc_m, out)
        ctx.lambd = float(lambd)
        return out[0].clone()

    @staticmethod
    def backward(ctx, g):
        from . import kernels as _K
        from .kernel_fns import _DT, _stream
        cls_preds, loc_preds, cls_t, loc_t, loc_m, stats = ctx.saved_tensors
        g = g.float().reshape(1).contiguous()
        dcls = torch.empty_like(cls_preds)
        dloc = torch.empty_like(loc_preds)
        _K.lib().ssd_loss_bwd(_DT[cls_preds.dtype], cls_preds.data_ptr(), loc_preds.data_ptr(), cls_t.data_ptr(),
                              loc_t.data_ptr(), loc_m.data_ptr(), stats.data_ptr(), g.data_ptr(), cls_t.numel(),
                              cls_preds.shape[-1], ctx.lambd, dcls.data_ptr(), dloc.data_ptr(), _stream())
        return dcls, dloc, None, None, None, None


@register('_contrib_ssd_multibox_loss', aliases=('ssd_multibox_loss',),
          arg_names=('cls_preds', 'loc_preds', 'cls_target', 'loc_target', 'loc_mask'),
          params={'lambd': ('float', 1.0)})
def ssd_multibox_loss(cls_preds, loc_preds, cls_target, loc_target, loc_mask, lambd=1.0):
    """SSD training loss (reference example/ssd/symbol/symbol_builder.py:90-102): cls_preds
    [B, A, classes+1], loc_preds [B, A*4], MultiBoxTarget's cls_target [B, A], loc_target / loc_mask
    [B, A*4] -> scalar.  Fused gfx950 kernels on the GPU, an fp32 composition elsewhere."""
    from . import kernels as _K
    from .kernel_fns import _DT
    if (cls_preds.is_cuda and cls_preds.dtype in _DT and loc_preds.dtype == cls_preds.dtype and _K.available()
            and cls_preds.shape[-1] <= 1024 and cls_target.numel() == cls_preds.numel() // cls_preds.shape[-1]
            and loc_preds.numel() == 4 * cls_target.numel()):
        return _SSDLossHip.apply(cls_preds, loc_preds, cls_target, loc_target, loc_mask, lambd)
    return _ssd_loss_reference(cls_preds, loc_preds, cls_target, loc_target, loc_mask, lambd)


# ---------------------------------------------------------------------------
# generic bounding-box ops
# ---------------------------------------------------------------------------

@register('_contrib_box_nms', aliases=('_contrib_box_non_maximum_suppression', 'box_nms'), num_outputs=2,
          num_visible_outputs=1,
          params={'overlap_thresh': ('float', 0.5), 'valid_thresh': ('float', 0.0), 'topk': ('int', -1),
                  'coord_start': ('int', 2), 'score_index': ('int', 1), 'id_index': ('int', -1),
                  'background_id': ('int', -1), 'force_suppress': ('bool', False), 'in_format': ('str', 'corner'),
                  'out_format': ('str', 'corner')})
def box_nms(data, overlap_thresh=0.5, valid_thresh=0.0, topk=-1, coord_start=2, score_index=1, id_index=-1,
            background_id=-1, force_suppress=False, in_format='corner', out_format='corner'):
    shape = data.shape
    x = data.reshape(-1, shape[-2], shape[-1]).float()
    out = torch.full_like(x, -1.0)
    idx_out = torch.full(x.shape[:2], -1.0, device=x.device)
    for b in range(x.shape[0]):
        rows = x[b]
        valid = rows[:, score_index] > valid_thresh
        if id_index >= 0:       # entries of the background class (default id -1) are never kept
            valid &= rows[:, id_index] != background_id
        vidx = torch.nonzero(valid).reshape(-1)
        if vidx.numel() == 0:
            continue
        order = vidx[torch.argsort(rows[vidx, score_index], descending=True, stable=True)]
        cand = rows[order].clone()
        boxes = _corner(cand[:, coord_start:coord_start + 4], in_format)
        # column 0 = class id shifted to >= 1 (a kept box of class -1 must not read as suppressed)
        cls = cand[:, id_index:id_index + 1] + 2.0 if id_index >= 0 else torch.zeros_like(cand[:, :1])
        work = torch.cat([cls, cand[:, score_index:score_index + 1], boxes], -1)
        work = _nms_rows(work, overlap_thresh, force_suppress or id_index < 0, topk)
        keep = work[:, 0] >= 0
        kept = cand[keep]
        if in_format != out_format:
            b4 = kept[:, coord_start:coord_start + 4]
            kept[:, coord_start:coord_start + 4] = _center(b4) if out_format == 'center' else _corner(b4, 'center')
        out[b, :kept.shape[0]] = kept
        idx_out[b, :kept.shape[0]] = order[keep].float()
    return out.reshape(shape).to(data.dtype), idx_out.reshape(shape[:-1])


@register('_contrib_box_iou', aliases=('box_iou',), arg_names=('lhs', 'rhs'), params={'format': ('str', 'corner')})
def box_iou(lhs, rhs, format='corner'):  # noqa: A002
    a = _corner(lhs.float(), format)
    b = _corner(rhs.float(), format)
    la = a.reshape(-1, 4)
    lb = b.reshape(-1, 4)
    return _iou(la, lb).reshape(tuple(lhs.shape[:-1]) + tuple(rhs.shape[:-1])).to(lhs.dtype)


@register('_contrib_bipartite_matching', aliases=('bipartite_matching',), num_outputs=2,
          params={'is_ascend': ('bool', False), 'threshold': ('float', 0.0), 'topk': ('int', -1)})
def bipartite_matching(data, is_ascend=False, threshold=0.0, topk=-1):
    shape = data.shape
    x = data.reshape(-1, shape[-2], shape[-1]).float().cpu()
    rows = torch.full((x.shape[0], shape[-2]), -1.0)
    cols = torch.full((x.shape[0], shape[-1]), -1.0)
    for b in range(x.shape[0]):
        flat = x[b].reshape(-1)
        order = torch.argsort(flat, descending=not is_ascend, stable=True)
        count = 0
        for o in order.tolist():
            v = float(flat[o])
            if (not is_ascend and v <= threshold) or (is_ascend and v >= threshold):
                break
            i, j = divmod(o, shape[-1])
            if rows[b, i] < 0 and cols[b, j] < 0:
                rows[b, i] = j
                cols[b, j] = i
                count += 1
                if 0 < topk <= count:
                    break
    return (rows.reshape(shape[:-1]).to(data.device), cols.reshape(tuple(shape[:-2]) + (shape[-1],)).to(data.device))


@register('_contrib_box_encode', aliases=('box_encode',), arg_names=('samples', 'matches', 'anchors', 'refs',
                                                                     'means', 'stds'), num_outputs=2)
def box_encode(samples, matches, anchors, refs, means, stds):
    m = matches.long().clamp(min=0)
    ref = torch.gather(refs.float(), 1, m.unsqueeze(-1).expand(-1, -1, 4))
    a = anchors.float()
    aw, ah = a[..., 2] - a[..., 0], a[..., 3] - a[..., 1]
    ax, ay = a[..., 0] + aw / 2, a[..., 1] + ah / 2
    gw, gh = ref[..., 2] - ref[..., 0], ref[..., 3] - ref[..., 1]
    gx, gy = ref[..., 0] + gw / 2, ref[..., 1] + gh / 2
    t = torch.stack([(gx - ax) / aw, (gy - ay) / ah, torch.log(gw / aw), torch.log(gh / ah)], -1)
    t = (t - means.float().reshape(1, 1, 4)) / stds.float().reshape(1, 1, 4)
    mask = (samples > 0.5).float().unsqueeze(-1).expand_as(t)
    return t * mask, mask


@register('_contrib_box_decode', aliases=('box_decode',), arg_names=('data', 'anchors'),
          params={'std0': ('float', 1.0), 'std1': ('float', 1.0), 'std2': ('float', 1.0), 'std3': ('float', 1.0),
                  'clip': ('float', -1.0), 'format': ('str', 'center')})
def box_decode(data, anchors, std0=1.0, std1=1.0, std2=1.0, std3=1.0, clip=-1.0, format='center'):  # noqa: A002
    a = anchors.float()
    if format == 'corner':
        a = _center(a)
    ax, ay, aw, ah = a.unbind(-1)
    d = data.float()
    ox = d[..., 0] * std0 * aw + ax
    oy = d[..., 1] * std1 * ah + ay
    dw, dh = d[..., 2] * std2, d[..., 3] * std3
    if clip > 0:
        dw, dh = dw.clamp(max=clip), dh.clamp(max=clip)
    ow, oh = torch.exp(dw) * aw / 2, torch.exp(dh) * ah / 2
    return torch.stack([ox - ow, oy - oh, ox + ow, oy + oh], -1).to(data.dtype)


# ---------------------------------------------------------------------------
# ROIAlign and RPN proposals
# ---------------------------------------------------------------------------

@register('_contrib_ROIAlign', aliases=('ROIAlign',), arg_names=('data', 'rois'),
          params={'pooled_size': ('shape', ()), 'spatial_scale': ('float', 1.0), 'sample_ratio': ('int', -1),
                  'position_sensitive': ('bool', False), 'aligned': ('bool', False)})
def roi_align(data, rois, pooled_size=(), spatial_scale=1.0, sample_ratio=-1, position_sensitive=False,
              aligned=False):
    """ROIAlign (reference src/operator/contrib/roi_align.cc): per-ROI sampling grids
    (ceil(roi / pooled) points per bin unless sample_ratio > 0), bilinear samples that vanish beyond
    one pixel outside the map and clamp to the border inside it, averaged per bin.  Gradients reach
    ``data`` only (the ROI coordinates get none, as in the reference)."""
    N, C, H, W = data.shape
    ph, pw = pooled_size
    R = rois.shape[0]
    dev, dt = data.device, data.dtype
    r = rois.detach().to(dt)
    off = 0.5 if aligned else 0.0
    bidx = r[:, 0].long()
    x1 = r[:, 1] * spatial_scale - off
    y1 = r[:, 2] * spatial_scale - off
    rw = r[:, 3] * spatial_scale - off - x1
    rh = r[:, 4] * spatial_scale - off - y1
    if not aligned:
        rw, rh = rw.clamp(min=1.0), rh.clamp(min=1.0)
    bw, bh = rw / pw, rh / ph
    if sample_ratio > 0:
        gh = torch.full((R,), sample_ratio, device=dev, dtype=torch.long)
        gw = gh.clone()
    else:
        gh = torch.ceil(rh / ph).long().clamp(min=1)
        gw = torch.ceil(rw / pw).long().clamp(min=1)
    GH = int(gh.max()) if R else 1
    GW = int(gw.max()) if R else 1
    iy = torch.arange(GH, device=dev, dtype=dt)
    ix = torch.arange(GW, device=dev, dtype=dt)
    # sample coordinates [R, ph, GH] / [R, pw, GW]
    ys = (y1[:, None, None] + torch.arange(ph, device=dev, dtype=dt)[None, :, None] * bh[:, None, None]
          + (iy[None, None, :] + 0.5) * bh[:, None, None] / gh[:, None, None].to(dt))
    xs = (x1[:, None, None] + torch.arange(pw, device=dev, dtype=dt)[None, :, None] * bw[:, None, None]
          + (ix[None, None, :] + 0.5) * bw[:, None, None] / gw[:, None, None].to(dt))
    my = (iy[None, :] < gh[:, None].to(dt)).to(dt)                  # [R, GH] points in use
    mx_ = (ix[None, :] < gw[:, None].to(dt)).to(dt)

    def axis(v, size):
        inside = ((v >= -1.0) & (v <= size)).to(dt)
        v = v.clamp(min=0.0)
        lo = v.floor().long()
        top = lo >= size - 1
        lo = torch.where(top, torch.full_like(lo, size - 1), lo)
        hi = torch.where(top, lo, lo + 1)
        v = torch.where(top, lo.to(dt), v)
        frac = v - lo.to(dt)
        return lo, hi, frac, inside

    ylo, yhi, ly, yin = axis(ys, H)
    xlo, xhi, lx, xin = axis(xs, W)
    P = ph * GH * pw * GW
    shp = (R, ph, GH, pw, GW)

    def idx(yi, xi):
        return (yi[:, :, :, None, None] * W + xi[:, None, None, :, :]).expand(shp).reshape(R, 1, P)

    wy = {0: (1.0 - ly), 1: ly}
    wx = {0: (1.0 - lx), 1: lx}
    valid = (yin[:, :, :, None, None] * xin[:, None, None, :, :] * my[:, None, :, None, None]
             * mx_[:, None, None, None, :])
    feats = data[bidx].reshape(R, C, H * W)
    acc = None
    for a, yi in ((0, ylo), (1, yhi)):
        for b_, xi in ((0, xlo), (1, xhi)):
            wgt = (wy[a][:, :, :, None, None] * wx[b_][:, None, None, :, :] * valid).reshape(R, 1, P)
            v = feats.gather(2, idx(yi, xi).expand(R, C, P)) * wgt
            acc = v if acc is None else acc + v
    cnt = (gh * gw).to(dt)
    s = acc.reshape(R, C, ph, GH, pw, GW).sum(dim=(3, 5)) / cnt[:, None, None, None]
    if position_sensitive:
        co = C // (ph * pw)
        s = s.reshape(R, co, ph, pw, ph, pw)
        i = torch.arange(ph, device=dev)
        j = torch.arange(pw, device=dev)
        s = s[:, :, i[:, None], j[None, :], i[:, None], j[None, :]]
    return s


def _generate_anchors(base, scales, ratios):
    ctr = (base - 1) / 2.0
    out = []
    for r in ratios:
        size = base * base / r
        ws = round(math.sqrt(size))
        hs = round(ws * r)
        for s in scales:
            w, h = ws * s, hs * s
            out.append([ctr - (w - 1) / 2, ctr - (h - 1) / 2, ctr + (w - 1) / 2, ctr + (h - 1) / 2])
    return torch.tensor(out, dtype=torch.float32)


def _proposal_single(score, bbox, info, anchors_base, feature_stride, pre_n, post_n, thresh, min_size, iou_loss):
    A = anchors_base.shape[0]
    H, W = score.shape[-2:]
    dev = score.device
    sx = torch.arange(W, device=dev, dtype=torch.float32) * feature_stride
    sy = torch.arange(H, device=dev, dtype=torch.float32) * feature_stride
    yy, xx = torch.meshgrid(sy, sx, indexing='ij')
    shifts = torch.stack([xx, yy, xx, yy], -1).reshape(-1, 1, 4)
    anchors = (anchors_base.to(dev).reshape(1, A, 4) + shifts).reshape(-1, 4)   # (H*W*A, 4)
    fg = score[A:].permute(1, 2, 0).reshape(-1)
    d = bbox.reshape(A, 4, H, W).permute(2, 3, 0, 1).reshape(-1, 4)
    w = anchors[:, 2] - anchors[:, 0] + 1
    h = anchors[:, 3] - anchors[:, 1] + 1
    cx = anchors[:, 0] + 0.5 * (w - 1)
    cy = anchors[:, 1] + 0.5 * (h - 1)
    if iou_loss:
        boxes = anchors + d
    else:
        pcx = d[:, 0] * w + cx
        pcy = d[:, 1] * h + cy
        pw_ = torch.exp(d[:, 2]) * w
        ph_ = torch.exp(d[:, 3]) * h
        boxes = torch.stack([pcx - 0.5 * (pw_ - 1), pcy - 0.5 * (ph_ - 1), pcx + 0.5 * (pw_ - 1),
                             pcy + 0.5 * (ph_ - 1)], -1)
    im_h, im_w, scale = float(info[0]), float(info[1]), float(info[2])
    boxes[:, 0::2] = boxes[:, 0::2].clamp(0, im_w - 1)
    boxes[:, 1::2] = boxes[:, 1::2].clamp(0, im_h - 1)
    ms = min_size * scale
    keep = ((boxes[:, 2] - boxes[:, 0] + 1) >= ms) & ((boxes[:, 3] - boxes[:, 1] + 1) >= ms)
    fg = torch.where(keep, fg, torch.full_like(fg, -1.0))
    order = torch.argsort(fg, descending=True, stable=True)[:pre_n]
    cand = torch.cat([torch.zeros_like(fg[order, None]), fg[order, None], boxes[order]], -1)
    cand = _nms_rows(cand, thresh, True, -1)
    kept = cand[cand[:, 0] >= 0][:post_n]
    if kept.shape[0] < post_n:                                   # pad by repeating (reference behaviour)
        reps = kept if kept.shape[0] else cand[:1]
        idx = torch.arange(post_n - kept.shape[0], device=dev) % max(reps.shape[0], 1)
        kept = torch.cat([kept, reps[idx]], 0)
    return kept[:, 2:6], kept[:, 1:2]


_PROP_PARAMS = {'rpn_pre_nms_top_n': ('int', 6000), 'rpn_post_nms_top_n': ('int', 300), 'threshold': ('float', 0.7),
                'rpn_min_size': ('int', 16), 'scales': ('floats', (4.0, 8.0, 16.0, 32.0)),
                'ratios': ('floats', (0.5, 1.0, 2.0)), 'feature_stride': ('int', 16), 'output_score': ('bool', False),
                'iou_loss': ('bool', False)}


def _prop_nout(a):
    return 2 if str(a.get('output_score', False)) in ('True', 'true', '1') else 1


@register('_contrib_MultiProposal', aliases=('MultiProposal', '_contrib_Proposal', 'Proposal'),
          arg_names=('cls_prob', 'bbox_pred', 'im_info'), num_outputs=_prop_nout, params=_PROP_PARAMS)
def multi_proposal(cls_prob, bbox_pred, im_info, rpn_pre_nms_top_n=6000, rpn_post_nms_top_n=300, threshold=0.7,
                   rpn_min_size=16, scales=(4.0, 8.0, 16.0, 32.0), ratios=(0.5, 1.0, 2.0), feature_stride=16,
                   output_score=False, iou_loss=False):
    base = _generate_anchors(feature_stride, scales, ratios)
    rois, scores = [], []
    for b in range(cls_prob.shape[0]):
        bx, sc = _proposal_single(cls_prob[b].float(), bbox_pred[b].float(), im_info[b], base, feature_stride,
                                  rpn_pre_nms_top_n, rpn_post_nms_top_n, threshold, rpn_min_size, iou_loss)
        rois.append(torch.cat([torch.full_like(bx[:, :1], float(b)), bx], -1))
        scores.append(sc)
    r = torch.cat(rois, 0)
    if output_score:
        return r, torch.cat(scores, 0)
    return r
