"""Python side of the in-tree gfx950 GEMM (src/kernels/gemm.hip).

``gemm_nt(a, b)`` computes ``act(a @ b.T + bias) (+ addend)`` for K-contiguous f16/bf16 operands --
the layout of every FullyConnected forward (x . W^T) and, with a transposed weight copy, of its
input gradient (dy . W).  ``configs(M, N, K)`` lists the (tile, split-K) candidates the autotuner
(kernel_fns._select) times against hipBLASLt per shape.

Reference: the FullyConnected GEMMs of src/operator/nn/fully_connected-inl.h (linalg_gemm, cuBLAS)
and the transformer projections of src/operator/contrib/transformer.cu:657.
"""
import torch

from . import kernels as _K

_DT = {torch.float16: 1, torch.bfloat16: 2}
ACT = {None: 0, 'none': 0, 'relu': 1, 'gelu': 2}
# tile config -> (BN output columns, BM output rows) of one workgroup (gemm.hip dispatch_gemm)
TILES = {0: (128, 128), 1: (128, 64), 2: (64, 128), 3: (256, 128), 4: (128, 256), 5: (256, 256), 6: (64, 64),
         7: (128, 128), 8: (256, 128), 9: (128, 64), 10: (64, 64), 11: (128, 256),   # 7..11: 3-4 LDS stages
         12: (128, 64), 13: (64, 128),   # 3 stages at two workgroups per CU
         # whole-wave grids on transformer shapes (M = 4096: N = 768 -> 256 tiles of 192x64, N = 3072 ->
         # 256 of 192x256 / 384x128, 512 of 192x128 at two workgroups per CU)
         14: (192, 64), 15: (192, 128), 16: (192, 256), 17: (384, 128)}
_WS = {}


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _workspace(n, dev):
    """Split-K fp32 partials, one buffer per (device, stream): split-K GEMMs issued on two streams of
    one device must not share it.  It is never grown during a HIP-graph capture (a buffer from the
    graph's private pool would be reused outside the graph): the eager warm-up sizes it first."""
    s = torch.cuda.current_stream(dev)
    key = (dev, s.cuda_stream)
    buf = _WS.get(key)
    if buf is None or buf.numel() < n:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError('gemm split-K workspace of %d floats requested during graph capture on a '
                               'stream without one; run the step eagerly first' % n)
        buf = _WS[key] = torch.empty(n, dtype=torch.float32, device=dev)
    return buf


def gemm_ok(a, b):
    return (a.is_cuda and a.dtype in _DT and b.dtype == a.dtype and a.dim() == 2 and b.dim() == 2
            and a.shape[1] == b.shape[1] and a.shape[1] % 64 == 0 and b.shape[0] % 64 == 0
            and a.stride(1) == 1 and b.stride(1) == 1 and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0
            and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0 and _K.available())


# the tile configs worth timing per shape (the 3-4 stage rings measured no faster on MI355X)
AUTOTUNE_TILES = (0, 1, 2, 3, 6, 12, 14, 15, 16, 17)


def configs(M, N, K, tiles=None):
    """Candidate (tile config, split-K) pairs for an M x N x K problem: tiles that divide N, and
    split-K factors that bring a grid of fewer than ~2 workgroups per CU up to the 256 CUs."""
    out = []
    kt = K // 64
    for cfg, (bn, bm) in sorted(TILES.items()):
        if N % bn or (tiles is not None and cfg not in tiles):
            continue
        ntile = (N // bn) * ((M + bm - 1) // bm)
        out.append((cfg, 1))
        for s in (2, 3, 4, 6, 8):
            if s <= kt // 2 and ntile * s <= 1024 and ntile < 512:
                out.append((cfg, s))
    return out


def gemm_nt(a, b, bias=None, act=None, addend=None, out=None, out_f32=False, cfg=(0, 1)):
    """``act(a @ b.T + bias) (+ addend)`` on the MFMA GEMM kernel.

    a: [M, K], b: [N, K] (K-contiguous, f16/bf16), bias: [N] (any float dtype; fp32 in the epilogue),
    addend: [M, N] of the output dtype, out: optional [M, N] output (row stride a multiple of 4),
    out_f32: fp32 output, cfg: (tile config, split-K factor)."""
    M, K = a.shape
    N = b.shape[0]
    tile, splits = cfg
    odt = torch.float32 if out_f32 else a.dtype
    if out is None:
        out = torch.empty(M, N, dtype=odt, device=a.device)
    assert out.dtype == odt and out.stride(1) == 1 and tuple(out.shape) == (M, N)
    if addend is not None:
        assert addend.dtype == odt and tuple(addend.shape) == (M, N) and addend.stride(1) == 1
        assert addend.stride(0) == out.stride(0)
    b32, lowp = None, 0
    if bias is not None:
        if bias.dtype == a.dtype and bias.is_contiguous() and bias.data_ptr() % 8 == 0:
            b32, lowp = bias, 1          # read in the operand dtype by the epilogue: no fp32 copy per call
        else:
            b32 = bias if (bias.dtype == torch.float32 and bias.is_contiguous()) else bias.float().contiguous()
    ws = _workspace(splits * M * N, a.device) if splits > 1 else None
    _K.lib().gemm_nt(_DT[a.dtype], a.data_ptr(), b.data_ptr(), 0 if b32 is None else b32.data_ptr(),
                     0 if addend is None else addend.data_ptr(), out.data_ptr(), int(bool(out_f32)), M, N, K,
                     a.stride(0), b.stride(0), out.stride(0), ACT[act], int(tile), int(splits),
                     0 if ws is None else ws.data_ptr(), _stream(), bias_lowp=lowp)
    return out


def gemm_reference(a, b, bias=None, act=None, addend=None):
    """fp32 PyTorch reference of gemm_nt (tests)."""
    y = a.float() @ b.float().t()
    if bias is not None:
        y = y + bias.float()
    if ACT[act] == 1:
        y = torch.relu(y)
    elif ACT[act] == 2:
        y = torch.nn.functional.gelu(y)
    if addend is not None:
        y = y + addend.float()
    return y


def candidates(a, b, bias=None, act=None, addend=None, out_f32=False, tiles=AUTOTUNE_TILES):
    """Autotuner candidates ('gemm<cfg>s<splits>', closure) for ``act(a @ b.T + bias) (+ addend)``;
    empty when the kernel cannot take the operands."""
    if not gemm_ok(a, b):
        return []
    M, K = a.shape
    N = b.shape[0]
    return [('gemm%ds%d' % c, lambda c=c: gemm_nt(a, b, bias=bias, act=act, addend=addend, out_f32=out_f32, cfg=c))
            for c in configs(M, N, K, tiles)]


def parse_name(name):
    """'gemm<cfg>s<splits>' -> (cfg, splits), else None."""
    if not name.startswith('gemm') or 's' not in name[4:]:
        return None
    c, s = name[4:].split('s', 1)
    return (int(c), int(s)) if c.isdigit() and s.isdigit() else None
