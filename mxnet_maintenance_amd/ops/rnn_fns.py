"""Fused RNN / LSTM / GRU layers on the in-tree gfx950 recurrent kernels (src/kernels/rnn.hip).

Reference: the cuDNN path of src/operator/rnn-inl.h (:418 forward, :743 backward).  Per (layer,
direction) the work is split the MI355X way:

* the input projection of ALL time steps is one GEMM ``x . W_ih^T + b`` (in-tree MFMA GEMM for
  f16/bf16 operands that tile, hipBLASLt otherwise), kept in fp32;
* the time loop runs in C++ (``rnn_fwd_seq``): one launch per step computes the recurrent GEMM of
  every gate of a 16x16 (batch x hidden) tile on the matrix cores and the cell update in
  registers; fp32 layers use the exact-f32 MFMA;
* backward (``rnn_bwd_seq``) produces the gate gradients step by step with the same fused
  structure, then the weight / input gradients are three large GEMMs over all steps: dX on the
  in-tree GEMM (gemm.hip), dW_ih / dW_hh on the in-tree TN weight-gradient kernel (conv_wgrad.hip),
  hipBLASLt only for widths that do not tile (I, H not multiples of 64) or fp32 layers.

Each (layer, direction) is one ``torch.autograd.Function``; layers chain through autograd
(inter-layer dropout in between), directions are concatenated along the feature axis.
"""
import torch

from . import kernels as _K

_MODES = {'rnn_tanh': 0, 'rnn_relu': 1, 'lstm': 2, 'gru': 3}
_GATES = {'rnn_tanh': 1, 'rnn_relu': 1, 'lstm': 4, 'gru': 3}
_SAVE = {'rnn_tanh': 1, 'rnn_relu': 1, 'lstm': 4, 'gru': 4}
_DT = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}


def available(data):
    return data.is_cuda and data.dtype in _DT and _K.available()


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _proj(x2, w, bias):
    """fp32 ``x2 @ w.T + bias`` (x2 [M, I], w [GH, I]) on the in-tree GEMM when it tiles."""
    from . import gemm as G
    if x2.dtype in G._DT and G.gemm_ok(x2, w):
        cfgs = [c for c in G.configs(x2.shape[0], w.shape[0], x2.shape[1]) if c[1] == 1]
        if cfgs:
            return G.gemm_nt(x2, w, bias=bias, out_f32=True, cfg=cfgs[0])
    return torch.addmm(bias.float(), x2.float(), w.float().t()) if x2.dtype != torch.float32 else \
        torch.addmm(bias, x2, w.t())


# which path each backward GEMM took (tests assert the in-tree one): 'gemm' = gemm.hip (dX),
# 'wgrad' = conv_wgrad.hip's TN reduction (dW), 'vendor' = torch.mm (hipBLASLt) / fp32
DISPATCH = {'gemm': 0, 'wgrad': 0, 'vendor': 0}


def _require_hip():
    import os
    return os.environ.get('MXAMD_REQUIRE_HIP', '0') == '1'


def _vendor(what):
    if _require_hip():
        from ..base import MXNetError
        raise MXNetError('RNN backward: %s does not tile for the in-tree GEMM kernels (MXAMD_REQUIRE_HIP=1)' % what)
    DISPATCH['vendor'] += 1


def _input_grad(g, w):
    """dX = g . w for g [M, G*H] and the layer weight w [G*H, I]: the in-tree NT GEMM on w^T (one
    small transposed copy per call), tile chosen by the autotuner among the gemm.hip configs."""
    from . import gemm as G
    from . import kernel_fns as KF
    wt = KF.transpose2d(w)
    if g.dtype in G._DT and g.is_contiguous() and G.gemm_ok(g, wt):
        cands = G.candidates(g, wt)
        if cands:
            DISPATCH['gemm'] += 1
            key = ('rnn_dx', tuple(g.shape), tuple(wt.shape), g.dtype)
            return KF._select(key, cands, cands[0][0])
    _vendor('dX %s x %s' % (tuple(g.shape), tuple(w.shape)))
    return torch.mm(g, w)


def _weight_grad(g, x, wdtype):
    """dW = g^T . x for g [M, G*H], x [M, C]: a reduction over the M = T*N rows, i.e. the weight
    gradient of a 1x1 convolution -- the in-tree TN kernel of conv_wgrad.hip (fp32 slabs + a
    deterministic reduce)."""
    from . import kernel_fns as KF
    M, GH = g.shape
    C = x.shape[1]
    x4 = x.contiguous().view(1, 1, M, C)
    if g.dtype == x.dtype and KF.conv_wgrad_ok(x4, torch.empty((GH, 1, 1, C), device='meta')):
        DISPATCH['wgrad'] += 1
        out = torch.empty((GH, 1, 1, C), dtype=wdtype, device=g.device)
        KF.conv_wgrad(x4, g.contiguous().view(1, 1, M, GH), (GH, 1, 1, C), (1, 1), (0, 0), out=out)
        return out.view(GH, C)
    _vendor('dW %s x %s' % (tuple(g.shape), tuple(x.shape)))
    return torch.mm(g.t(), x)


class _LayerDir(torch.autograd.Function):
    """One direction of one recurrent layer over the whole sequence."""

    @staticmethod
    def forward(ctx, x, h0, c0, w_ih, w_hh, b_ih, b_hh, mode, reverse):
        T, N, I = x.shape
        H = w_hh.shape[1]
        G = _GATES[mode]
        dt = x.dtype
        x = x.contiguous()
        w_ih = w_ih.contiguous()
        w_hh = w_hh.contiguous()
        ctx.h0_dtype = h0.dtype
        h0 = h0.contiguous().to(dt)
        gru = mode == 'gru'
        bias = (b_ih.float() if gru else (b_ih.float() + b_hh.float())).contiguous()
        gx = _proj(x.reshape(T * N, I), w_ih, bias)
        out = torch.empty((T, N, H), dtype=dt, device=x.device)
        save = torch.empty((T, N, _SAVE[mode] * H), dtype=torch.float32, device=x.device)
        c0f = c0.float().contiguous() if c0 is not None else None
        cseq = torch.empty((T, N, H), dtype=torch.float32, device=x.device) if mode == 'lstm' else None
        bhh = b_hh.float().contiguous() if gru else None
        _K.lib().rnn_fwd_seq(_DT[dt], _MODES[mode], gx.data_ptr(), h0.data_ptr(),
                             0 if c0f is None else c0f.data_ptr(), w_hh.data_ptr(), 0 if bhh is None else bhh.data_ptr(),
                             out.data_ptr(), H, 0 if cseq is None else cseq.data_ptr(), save.data_ptr(), T, N, H,
                             int(bool(reverse)), _stream())
        last = 0 if reverse else T - 1
        hT = out[last].clone()
        cT = cseq[last].to(dt) if cseq is not None else None
        ctx.mode, ctx.reverse = mode, bool(reverse)
        ctx.save_for_backward(x, h0, c0f, w_ih, w_hh, out, cseq, save)
        ctx.has_c0 = c0 is not None
        ctx.c0_dtype = None if c0 is None else c0.dtype
        if cT is None:
            return out, hT
        return out, hT, cT

    @staticmethod
    def backward(ctx, dy, dhT, dcT=None):
        x, h0, c0f, w_ih, w_hh, out, cseq, save = ctx.saved_tensors
        mode, reverse = ctx.mode, ctx.reverse
        T, N, I = x.shape
        H = w_hh.shape[1]
        G = _GATES[mode]
        dt = x.dtype
        dev = x.device
        dy = dy.contiguous().to(dt) if dy is not None else None
        dhT32 = dhT.float().contiguous() if dhT is not None else torch.zeros((N, H), dtype=torch.float32, device=dev)
        from . import kernel_fns as _KF2
        whhT = _KF2.transpose2d(w_hh)
        dgh = torch.empty((T, N, G * H), dtype=dt, device=dev)
        gru = mode == 'gru'
        dgx = torch.empty_like(dgh) if gru else None
        dc = None
        if mode == 'lstm':
            dc = dcT.float().clone().contiguous() if dcT is not None else torch.zeros((N, H), dtype=torch.float32,
                                                                                        device=dev)
        dhd = torch.zeros((N, H), dtype=torch.float32, device=dev) if gru else None
        dh0 = torch.empty((N, H), dtype=torch.float32, device=dev)
        _K.lib().rnn_bwd_seq(_DT[dt], _MODES[mode], whhT.data_ptr(), 0 if dy is None else dy.data_ptr(), H,
                             dhT32.data_ptr(), save.data_ptr(), 0 if cseq is None else cseq.data_ptr(),
                             0 if c0f is None else c0f.data_ptr(), h0.data_ptr(), out.data_ptr(), H, dgh.data_ptr(),
                             0 if dgx is None else dgx.data_ptr(), 0 if dc is None else dc.data_ptr(),
                             0 if dhd is None else dhd.data_ptr(), dh0.data_ptr(), T, N, H, int(reverse), _stream())
        gX = (dgx if gru else dgh).reshape(T * N, G * H)
        gH = dgh.reshape(T * N, G * H)
        # h_{t-1} of every step in forward order
        hprev = torch.cat([out[1:], h0[None]], 0) if reverse else torch.cat([h0[None], out[:-1]], 0)
        dx = _input_grad(gX, w_ih).view(T, N, I) if ctx.needs_input_grad[0] else None
        dw_ih = _weight_grad(gX, x.reshape(T * N, I), w_ih.dtype) if ctx.needs_input_grad[3] else None
        dw_hh = _weight_grad(gH, hprev.reshape(T * N, H), w_hh.dtype) if ctx.needs_input_grad[4] else None
        db_ih = gX.sum(0, dtype=torch.float32) if ctx.needs_input_grad[5] else None
        db_hh = gH.sum(0, dtype=torch.float32) if ctx.needs_input_grad[6] else None
        dc0 = dc.to(ctx.c0_dtype) if (dc is not None and ctx.has_c0) else None
        return dx, dh0.to(ctx.h0_dtype), dc0, dw_ih, dw_hh, \
            (db_ih.to(w_ih.dtype) if db_ih is not None else None), \
            (db_hh.to(w_hh.dtype) if db_hh is not None else None), None, None


def fused_rnn(data, ws, h0, c0, mode, num_layers, bidirectional, p, train):
    """Multi-layer (bi)directional RNN over ``data`` [T, N, I] with per-(layer, direction) weights
    ``ws[k] = [w_ih, w_hh, b_ih, b_hh]``; returns (out [T, N, D*H], h [L*D, N, H], c or None)."""
    d = 2 if bidirectional else 1
    x = data
    hs, cs = [], []
    for layer in range(num_layers):
        outs = []
        for di in range(d):
            k = layer * d + di
            w_ih, w_hh, b_ih, b_hh = ws[k][:4]
            c_in = c0[k] if (mode == 'lstm' and c0 is not None) else None
            if mode == 'lstm' and c_in is None:
                c_in = torch.zeros_like(h0[k])
            res = _LayerDir.apply(x, h0[k], c_in, w_ih, w_hh, b_ih, b_hh, mode, di == 1)
            outs.append(res[0])
            hs.append(res[1])
            if mode == 'lstm':
                cs.append(res[2])
        x = torch.cat(outs, -1) if d == 2 else outs[0]
        if p > 0 and train and layer < num_layers - 1:
            x = torch.nn.functional.dropout(x, p, True)
    return x, torch.stack(hs), (torch.stack(cs) if cs else None)


def reference_rnn(data, ws, h0, c0, mode, num_layers, bidirectional):
    """fp32 PyTorch reference (tests): torch's own fused RNN on fp32 copies."""
    flat = [t.float() for group in ws for t in group[:4]]
    d32 = data.float()
    if mode == 'lstm':
        out, h, c = torch._VF.lstm(d32, (h0.float(), c0.float()), flat, True, num_layers, 0.0, True,
                                   bidirectional, False)
        return out, h, c
    fn = {'gru': torch._VF.gru, 'rnn_tanh': torch._VF.rnn_tanh, 'rnn_relu': torch._VF.rnn_relu}[mode]
    out, h = fn(d32, h0.float(), flat, True, num_layers, 0.0, True, bidirectional, False)
    return out, h, None
