"""In-tree gfx950 recurrent kernels (src/kernels/rnn.hip) vs an fp32 PyTorch reference."""
import pytest
import torch

from mxnet_maintenance_amd.ops import rnn_fns

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))


def _make(mode, L, D, I, H, dt, dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    G = {'lstm': 4, 'gru': 3, 'rnn_tanh': 1, 'rnn_relu': 1}[mode]
    ws = []
    for layer in range(L):
        ni = I if layer == 0 else H * D
        for _ in range(D):
            s = 1.0 / H ** 0.5
            ws.append([(torch.rand(G * H, ni, generator=g) * 2 - 1) * s, (torch.rand(G * H, H, generator=g) * 2 - 1) * s,
                       (torch.rand(G * H, generator=g) * 2 - 1) * s, (torch.rand(G * H, generator=g) * 2 - 1) * s])
    ws = [[t.to(dev, dt).requires_grad_(True) for t in grp] for grp in ws]
    return ws


@pytest.mark.parametrize('mode', ['lstm', 'gru', 'rnn_tanh', 'rnn_relu'])
@pytest.mark.parametrize('dt,H', [(torch.float32, 40), (torch.bfloat16, 64), (torch.float16, 48), (torch.float32, 37)])
def test_fused_rnn_matches_fp32_reference(mode, dt, H):
    from mxnet_maintenance_amd.ops import kernels
    assert kernels.available(), kernels.load_error()
    dev = torch.device('cuda', 0)
    T, N, I, L, D = 7, 19, 24, 2, 2
    ws = _make(mode, L, D, I, H, dt, dev)
    g = torch.Generator().manual_seed(1)
    x = (torch.rand(T, N, I, generator=g) * 2 - 1).to(dev, dt).requires_grad_(True)
    h0 = (torch.rand(L * D, N, H, generator=g) * 0.5).to(dev, dt).requires_grad_(True)
    c0 = (torch.rand(L * D, N, H, generator=g) * 0.5).to(dev, dt).requires_grad_(True) if mode == 'lstm' else None
    out, h, c = rnn_fns.fused_rnn(x, ws, h0, c0, mode, L, True, 0.0, True)
    # fp32 reference on copies of the same values
    wr = [[t.detach().float().requires_grad_(True) for t in grp] for grp in ws]
    xr = x.detach().float().requires_grad_(True)
    h0r = h0.detach().float().requires_grad_(True)
    c0r = c0.detach().float().requires_grad_(True) if c0 is not None else None
    ro, rh, rc = rnn_fns.reference_rnn(xr, wr, h0r, c0r, mode, L, True)
    tol = 2e-5 if dt == torch.float32 else 3e-2
    assert _rel(out, ro) < tol and _rel(h, rh) < tol
    if c is not None:
        assert _rel(c, rc) < tol
    # gradients through every output
    gy = torch.rand(out.shape, generator=g).to(dev) - 0.5
    gh = torch.rand(h.shape, generator=g).to(dev) - 0.5
    loss = (out.float() * gy).sum() + (h.float() * gh).sum()
    rloss = (ro * gy).sum() + (rh * gh).sum()
    if c is not None:
        gc = torch.rand(c.shape, generator=g).to(dev) - 0.5
        loss = loss + (c.float() * gc).sum()
        rloss = rloss + (rc * gc).sum()
    loss.backward()
    rloss.backward()
    gtol = 1e-4 if dt == torch.float32 else 6e-2
    assert _rel(x.grad, xr.grad) < gtol
    assert _rel(h0.grad, h0r.grad) < gtol
    if c0 is not None:
        assert _rel(c0.grad, c0r.grad) < gtol
    for grp, rgrp in zip(ws, wr):
        for t, r in zip(grp, rgrp):
            assert _rel(t.grad, r.grad) < gtol, (mode, dt, H)


def test_rnn_op_runs_in_tree_kernels():
    """The registered RNN operator takes the in-tree path on the GPU (a Gluon LSTM layer step): the
    recurrent kernels forward and backward, dX on gemm.hip and dW on conv_wgrad.hip -- counted per
    dispatch, with MXAMD_REQUIRE_HIP=1 turning any vendor fallback into an error."""
    import os
    import mxnet_maintenance_amd as mx
    from mxnet_maintenance_amd import gluon, autograd, nd
    from mxnet_maintenance_amd.ops import rnn_fns
    os.environ['MXAMD_REQUIRE_HIP'] = '1'
    try:
        layer = gluon.rnn.LSTM(64, num_layers=2, bidirectional=True)
        layer.initialize(ctx=mx.gpu(0))
        layer.cast('float16')
        x = nd.random.uniform(shape=(12, 8, 64), ctx=mx.gpu(0)).astype('float16')
        x.attach_grad()
        before = dict(rnn_fns.DISPATCH)
        with autograd.record():
            y = layer(x)
        y.backward()
        assert y.shape == (12, 8, 128)
        assert float(x.grad.abs().sum().asscalar()) > 0
        # 2 layers x 2 directions: one dX GEMM and two dW reductions each
        assert rnn_fns.DISPATCH['gemm'] - before['gemm'] == 4
        assert rnn_fns.DISPATCH['wgrad'] - before['wgrad'] == 8
        assert rnn_fns.DISPATCH['vendor'] == before['vendor']
    finally:
        os.environ.pop('MXAMD_REQUIRE_HIP', None)
