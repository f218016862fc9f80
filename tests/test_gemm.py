"""In-tree gfx950 GEMM (src/kernels/gemm.hip) against a plain PyTorch fp32 reference: every tile
config, split-K, bias / ReLU / GELU epilogues, residual addend, fp32 output, ragged M."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-6))


@pytest.mark.parametrize('dt', [torch.bfloat16, torch.float16])
@pytest.mark.parametrize('cfg', list(range(18)))
def test_gemm_nt_tiles(dt, cfg):
    from mxnet_maintenance_amd.ops import gemm as G
    torch.manual_seed(cfg)
    assert cfg in G.TILES
    M, N, K = 1000, 768, 320          # M not a tile multiple, K = 5 k-tiles, N a multiple of every tile
    a = torch.randn(M, K, device='cuda', dtype=dt)
    b = torch.randn(N, K, device='cuda', dtype=dt) * 0.1
    bias = torch.randn(N, device='cuda')
    y = G.gemm_nt(a, b, bias=bias, cfg=(cfg, 1))
    assert _rel(y, G.gemm_reference(a, b, bias)) < 1e-2


@pytest.mark.parametrize('splits', [2, 3, 5])
@pytest.mark.parametrize('act', [None, 'relu', 'gelu'])
def test_gemm_nt_splitk_epilogues(splits, act):
    from mxnet_maintenance_amd.ops import gemm as G
    torch.manual_seed(splits)
    M, N, K = 777, 256, 640
    dt = torch.bfloat16
    a = torch.randn(M, K, device='cuda', dtype=dt)
    b = torch.randn(N, K, device='cuda', dtype=dt) * 0.1
    bias = torch.randn(N, device='cuda')
    add = torch.randn(M, N, device='cuda', dtype=dt)
    ref = G.gemm_reference(a, b, bias, act, add)
    for s in (1, splits):
        y = G.gemm_nt(a, b, bias=bias, act=act, addend=add, cfg=(0, s))
        assert _rel(y, ref) < 1e-2, (s, act)


@pytest.mark.parametrize('cfg', [14, 15, 16, 17])
def test_gemm_nt_wide_tiles_epilogues(cfg):
    """192 / 384-column tiles (FI = 3 / 6 fragments per wave): GELU, residual addend and split-K."""
    from mxnet_maintenance_amd.ops import gemm as G
    torch.manual_seed(100 + cfg)
    M, N, K = 517, 1152, 384
    dt = torch.bfloat16
    a = torch.randn(M, K, device='cuda', dtype=dt)
    b = torch.randn(N, K, device='cuda', dtype=dt) * 0.1
    bias = torch.randn(N, device='cuda')
    add = torch.randn(M, N, device='cuda', dtype=dt)
    ref = G.gemm_reference(a, b, bias, 'gelu', add)
    for s in (1, 2):
        y = G.gemm_nt(a, b, bias=bias, act='gelu', addend=add, cfg=(cfg, s))
        assert _rel(y, ref) < 1e-2, s


@pytest.mark.parametrize('dt', [torch.bfloat16, torch.float16])
@pytest.mark.parametrize('splits', [1, 3])
def test_gemm_nt_bias_in_operand_dtype(dt, splits):
    """A bias in the operand dtype is read as such by the epilogue (and the split-K reduction)."""
    from mxnet_maintenance_amd.ops import gemm as G
    torch.manual_seed(7)
    M, N, K = 300, 384, 448
    a = torch.randn(M, K, device='cuda', dtype=dt)
    b = torch.randn(N, K, device='cuda', dtype=dt) * 0.1
    bias = torch.randn(N, device='cuda', dtype=dt)
    y = G.gemm_nt(a, b, bias=bias, act='relu', cfg=(1, splits))
    assert _rel(y, G.gemm_reference(a, b, bias.float(), 'relu')) < 1e-2


def test_gemm_nt_fp32_out_and_strided_rows():
    from mxnet_maintenance_amd.ops import gemm as G
    torch.manual_seed(0)
    big = torch.randn(300, 256 + 64, device='cuda', dtype=torch.float16)
    a = big[:, :256]                   # row stride 320 elements
    b = torch.randn(128, 256, device='cuda', dtype=torch.float16)
    out = torch.empty(300, 128, device='cuda', dtype=torch.float32)
    G.gemm_nt(a, b, out=out, out_f32=True, cfg=(6, 2))
    assert _rel(out, G.gemm_reference(a, b)) < 1e-3


def test_fc_layer_uses_gemm_candidates():
    """A Dense layer forward/backward through the autotuned FullyConnected path matches fp32."""
    import mxnet_maintenance_amd as mx
    from mxnet_maintenance_amd import autograd, gluon, nd
    net = gluon.nn.Dense(384, in_units=256, flatten=False)
    net.initialize(mx.init.Xavier(), ctx=mx.gpu(0))
    net.cast('bfloat16')
    x = nd.random.uniform(-1, 1, shape=(4, 100, 256), ctx=mx.gpu(0)).astype('bfloat16')
    x.attach_grad()
    with autograd.record():
        y = net(x)
    y.backward()
    w = net.weight.data()._data.float()
    b = net.bias.data()._data.float()
    xf = x._data.float()
    ref = xf @ w.t() + b
    assert _rel(y._data, ref) < 2e-2
    assert _rel(x.grad._data, torch.ones_like(ref) @ w) < 2e-2


@pytest.mark.parametrize('shape,dt', [((768, 3072), torch.bfloat16), ((30528, 768), torch.float16),
                                      ((64, 256), torch.float16), ((40, 24), torch.float32), ((33, 16), torch.float16)])
def test_transpose2d_matches_torch(shape, dt):
    """kernel_fns.transpose2d (the LDS-tiled tap-transpose kernel for every weight transpose of the data
    gradients) equals w.t().contiguous(), including its torch fallback for rows that are not 8-multiples."""
    from mxnet_maintenance_amd.ops import kernel_fns as KF
    w = torch.randn(*shape, device='cuda').to(dt)
    t = KF.transpose2d(w)
    assert t.is_contiguous() and torch.equal(t, w.t().contiguous())
