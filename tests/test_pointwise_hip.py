"""In-tree element-wise kernels (src/kernels/pointwise.hip): ReLU forward/backward and broadcasting
binary arithmetic against a plain PyTorch fp32 reference of the same op."""
import pytest
import torch

from mxnet_maintenance_amd.ops import kernel_fns as K

pytestmark = pytest.mark.gpu

DTYPES = [torch.float16, torch.bfloat16, torch.float32]
TOL = {torch.float16: 2e-3, torch.bfloat16: 1.6e-2, torch.float32: 1e-6}


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')
    assert K._K.available(), 'HIP kernel extension must be loaded on a GPU box'


@pytest.mark.parametrize('dtype', DTYPES)
@pytest.mark.parametrize('n', [8, 1000, 4099, 1 << 20])
def test_relu_forward_backward(dtype, n):
    x = torch.randn(n, device='cuda').to(dtype).requires_grad_(True)
    y = K.ReluHip.apply(x)
    g = torch.randn(n, device='cuda').to(dtype)
    y.backward(g)
    xf = x.detach().float()
    torch.testing.assert_close(y.float(), torch.relu(xf), rtol=0, atol=0)
    torch.testing.assert_close(x.grad.float(), torch.where(xf > 0, g.float(), torch.zeros_like(xf)), rtol=0, atol=0)


SHAPES = [
    ((4, 7, 9, 64), (4, 7, 9, 64)),        # equal shapes (vector path)
    ((4, 7, 9, 64), (64,)),                # row operand (bias over NHWC)
    ((1, 64), (32, 5, 64)),                # row operand on the left
    ((6, 1, 5), (1, 3, 1)),                # general broadcast (strided path)
    ((3, 5, 7), ()),                       # scalar tensor
    ((4, 8, 3), (4, 1, 3)),                # middle-axis broadcast
]


@pytest.mark.parametrize('dtype', DTYPES)
@pytest.mark.parametrize('op', ['add', 'sub', 'mul', 'div', 'maximum', 'minimum'])
@pytest.mark.parametrize('shapes', SHAPES)
def test_binary_broadcast_matches_fp32(dtype, op, shapes):
    sa, sb = shapes
    a = torch.randn(sa, device='cuda').to(dtype)
    b = torch.randn(sb, device='cuda').to(dtype)
    if op == 'div':
        b = b.sign().where(b != 0, torch.ones_like(b)) * (b.abs() + 0.5)
    a.requires_grad_(True)
    b.requires_grad_(True)
    y = K.BinaryHip.apply(a, b, op)
    ref_fn = {'add': torch.add, 'sub': torch.sub, 'mul': torch.mul, 'div': torch.div, 'maximum': torch.maximum,
              'minimum': torch.minimum}[op]
    af, bf = a.detach().float().requires_grad_(True), b.detach().float().requires_grad_(True)
    ref = ref_fn(af, bf)
    tol = TOL[dtype]
    torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)
    g = torch.randn(ref.shape, device='cuda')
    y.backward(g.to(dtype))
    if op in ('maximum', 'minimum'):
        take = (af >= bf) if op == 'maximum' else (af <= bf)
        ga = torch.where(take, g, torch.zeros_like(g))
        gref_a, gref_b = ga.sum_to_size(af.shape), (g - ga).sum_to_size(bf.shape)
    else:
        ref.backward(g.to(dtype).float())
        gref_a, gref_b = af.grad, bf.grad
    gtol = tol * 8
    torch.testing.assert_close(a.grad.float(), gref_a, rtol=gtol, atol=gtol * max(1.0, g.numel() / a.numel()))
    torch.testing.assert_close(b.grad.float(), gref_b, rtol=gtol, atol=gtol * max(1.0, g.numel() / b.numel()))


def test_registered_ops_run_the_kernel():
    import mxnet_maintenance_amd as mx
    x = mx.nd.array(torch.randn(4, 16).numpy(), ctx=mx.gpu(0), dtype='float16')
    bias = mx.nd.array(torch.randn(16).numpy(), ctx=mx.gpu(0), dtype='float16')
    out = mx.nd.broadcast_add(x, bias.reshape((1, 16)))
    ref = x.asnumpy().astype('float32') + bias.asnumpy().astype('float32')
    assert abs(out.asnumpy().astype('float32') - ref).max() < 1e-2
    r = mx.nd.relu(x)
    assert (r.asnumpy() >= 0).all()


@pytest.mark.parametrize('M,N,dt', [(4096, 768, torch.bfloat16), (333, 3072, torch.float16), (64, 8, torch.float32),
                                    (20000, 1024, torch.bfloat16)])
def test_bias_grad_colsum(M, N, dt):
    """Bias gradient column sums (partial rows + their sum), repeated on the shared scratch."""
    from mxnet_maintenance_amd.ops import nlp_fns
    g = torch.Generator().manual_seed(M + N)
    dy = (torch.rand(M, N, generator=g) * 2 - 1).to('cuda', dt)
    ref = dy.float().sum(0)
    for _ in range(3):
        out = nlp_fns.bias_grad(dy, None, torch.float32)
        torch.testing.assert_close(out.float(), ref, rtol=1e-3, atol=1e-2 * (M ** 0.5) / 10)


@pytest.mark.parametrize('shape,dt', [((64, 3, 3, 64), torch.float16), ((256, 3, 3, 128), torch.bfloat16),
                                      ((96, 5, 3, 40), torch.float32), ((512, 1, 1, 2048), torch.float16),
                                      ((60, 3, 3, 36), torch.float16), ((130, 3, 3, 72), torch.bfloat16)])
def test_dgrad_weight_tap_transpose(shape, dt):
    """The flipped [Cin][R][S][Cout] data-gradient weight from the tap-transpose kernel equals torch's
    flip + permute."""
    w = torch.randn(shape, device='cuda').to(dt)
    assert torch.equal(K._dgrad_weight(w), w.flip(1, 2).permute(3, 1, 2, 0).contiguous())


@pytest.mark.parametrize('wshape,stride,pad', [((128, 3, 3, 64), (2, 2), (1, 1)), ((256, 1, 1, 128), (2, 2), (0, 0)),
                                               ((64, 3, 3, 128), (2, 2), (1, 1))])
def test_phase_weight_slices(wshape, stride, pad):
    """The per-phase tap slices of a strided dgrad ([C][R_i][S_i][K], concatenated) built in one launch
    equal the slices gathered on the host."""
    w = torch.randn(wshape, device='cuda').to(torch.float16)
    phases, _empty, (slots, total) = K._phase_plan(w.shape, stride, pad, w.device)
    got = K._taps_t(w, torch.empty(total, dtype=w.dtype, device=w.device), [t[0] for t in slots],
                    [t[1] for t in slots], [t[2] for t in slots])
    Kc, R, S, C = wshape
    for ph, pw, ri, si, _a, _b, off in phases:
        rr = [r for _, r in K._phase_taps(R, pad[0], stride[0], ph)]
        ss = [c for _, c in K._phase_taps(S, pad[1], stride[1], pw)]
        ref = w[:, rr][:, :, ss].permute(3, 1, 2, 0).contiguous().reshape(-1)
        assert torch.equal(got[off:off + ref.numel()], ref)
