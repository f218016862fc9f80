"""Deformable convolution (v1 and modulated v2): the gfx950 HIP kernels (src/kernels/deform_conv.hip)
against an fp32 torch reference of the same op (grid_sample per tap + grouped GEMM) on the CPU,
forward and all four gradients (data, offset, mask, weight)."""
import numpy as np
import pytest
import torch

from mxnet_maintenance_amd.ops import contrib_ops as C

CASES = [
    # N, C, H, W, O, k, stride, pad, dilate, groups, deformable groups, modulated
    (2, 8, 9, 11, 6, (3, 3), (1, 1), (1, 1), (1, 1), 1, 1, False),
    (2, 8, 10, 10, 8, (3, 3), (2, 2), (1, 1), (1, 1), 2, 2, True),
    (1, 16, 7, 9, 4, (3, 2), (1, 1), (2, 1), (2, 1), 1, 4, True),
]


def _inputs(case, seed=0):
    N, Cin, H, W, O, k, s, p, d, g, dg, mod = case
    gen = torch.Generator().manual_seed(seed)
    Ho = (H + 2 * p[0] - d[0] * (k[0] - 1) - 1) // s[0] + 1
    Wo = (W + 2 * p[1] - d[1] * (k[1] - 1) - 1) // s[1] + 1
    x = torch.randn(N, Cin, H, W, generator=gen)
    off = 2.0 * torch.randn(N, dg * 2 * k[0] * k[1], Ho, Wo, generator=gen)
    mask = torch.rand(N, dg * k[0] * k[1], Ho, Wo, generator=gen) if mod else None
    w = torch.randn(O, Cin // g, k[0], k[1], generator=gen) * 0.2
    return x, off, mask, w


def _run(case, x, off, mask, w, grad_dtype=None):
    _, _, _, _, _, k, s, p, d, g, dg, _ = case
    leaves = [t.requires_grad_() for t in (x, off, mask, w) if t is not None]
    out = C._deform_conv(x, off, mask, w, None, k, s, p, d, g, dg)
    gout = torch.linspace(-1, 1, out.numel(), dtype=torch.float32).reshape(out.shape)
    if grad_dtype is not None:
        gout = gout.to(grad_dtype)          # the output gradient rounded like the device run's
    gout = gout.to(out.device, out.dtype)
    out.backward(gout)
    return [out.detach().float().cpu()] + [t.grad.detach().float().cpu() for t in leaves]


def test_cpu_path_matches_numerical_gradients():
    case = (1, 2, 5, 5, 2, (3, 3), (1, 1), (1, 1), (1, 1), 1, 1, True)
    x, off, mask, w = (t.double() if t is not None else None for t in _inputs(case))
    off = off * 0.3 + 0.37            # keep taps away from integer positions (bilinear kinks)

    def f(x, off, mask, w):
        return C._deform_conv(x, off, mask, w, None, (3, 3), (1, 1), (1, 1), (1, 1), 1, 1)
    assert torch.autograd.gradcheck(f, tuple(t.requires_grad_() for t in (x, off, mask, w)), eps=1e-6, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize('case', CASES)
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_hip_kernels_match_fp32_reference(case, dtype):
    from mxnet_maintenance_amd.ops import kernels
    assert kernels.available(), kernels.load_error()
    x, off, mask, w = _inputs(case)
    # keep every sampling position's fractional part in [0.25, 0.75): bf16 rounding would otherwise
    # put some taps exactly on the integer grid, where the bilinear weights' derivative jumps and any
    # two implementations may take different one-sided offset gradients
    off = off.floor() + 0.25 + 0.5 * (off - off.floor())
    ref = _run(case, *(t.clone() if t is not None else None for t in (x, off, mask, w)))
    dev = [t.to('cuda', dtype) if t is not None else None for t in (x, off, mask, w)]
    if dtype != torch.float32:
        # compare against the reference evaluated on the same rounded inputs
        ref = _run(case, *(t.float().cpu() if t is not None else None for t in dev), grad_dtype=dtype)
    got = _run(case, *dev)
    tol = 2e-4 if dtype == torch.float32 else 3e-2
    names = ['out', 'dx', 'doffset'] + (['dmask'] if mask is not None else []) + ['dweight']
    for name, a, b in zip(names, got, ref):
        err = (a - b).norm() / b.norm().clamp_min(1e-12)
        assert err < tol, (name, float(err))


ROW_CASES = [
    # shapes whose column width C/g*K and output channels O/g tile the in-tree MFMA GEMMs
    (2, 64, 9, 11, 64, (3, 3), (1, 1), (1, 1), (1, 1), 1, 1, False),
    (2, 128, 10, 10, 128, (3, 3), (2, 2), (1, 1), (1, 1), 2, 2, True),
    (4, 256, 8, 8, 256, (3, 3), (2, 2), (1, 1), (1, 1), 1, 1, False),     # an SSD-512 extra layer
]


@pytest.mark.gpu
@pytest.mark.parametrize('case', ROW_CASES)
@pytest.mark.parametrize('dtype', [torch.float16, torch.bfloat16])
def test_row_columns_on_intree_gemms_match_fp32_reference(case, dtype):
    """f16/bf16 deformable conv on the row-column layout: im2col rows -> gemm.hip (forward, fp32
    column gradient), conv_wgrad.hip (weight gradient) -- no torch GEMM (MXAMD_REQUIRE_HIP)."""
    import os
    from mxnet_maintenance_amd.ops import kernels
    assert kernels.available(), kernels.load_error()
    x, off, mask, w = _inputs(case)
    off = off.floor() + 0.25 + 0.5 * (off - off.floor())
    dev = [t.to('cuda', dtype) if t is not None else None for t in (x, off, mask, w)]
    ref = _run(case, *(t.float().cpu() if t is not None else None for t in dev), grad_dtype=dtype)
    before = C.DISPATCH['gemm']
    os.environ['MXAMD_REQUIRE_HIP'] = '1'
    try:
        got = _run(case, *dev)
    finally:
        os.environ.pop('MXAMD_REQUIRE_HIP', None)
    assert C.DISPATCH['gemm'] == before + 1
    names = ['out', 'dx', 'doffset'] + (['dmask'] if mask is not None else []) + ['dweight']
    for name, a, b in zip(names, got, ref):
        err = (a - b).norm() / b.norm().clamp_min(1e-12)
        assert err < 3e-2, (name, float(err))


@pytest.mark.gpu
@pytest.mark.parametrize('modulated', [False, True])
def test_channels_last_inputs_and_strided_offsets(modulated):
    """The channels-last path takes NHWC-memory activations and offsets that are a channel slice of a
    wider buffer (the padded offset conv's output) without copies; gradients match the fp32 reference."""
    from mxnet_maintenance_amd.ops import kernels
    assert kernels.available(), kernels.load_error()
    case = (2, 128, 10, 10, 128, (3, 3), (1, 1), (1, 1), (1, 1), 1, 1, modulated)
    x, off, mask, w = _inputs(case)
    off = off.floor() + 0.25 + 0.5 * (off - off.floor())
    dt = torch.float16
    xd = x.to('cuda', dt).permute(0, 2, 3, 1).contiguous().permute(0, 3, 1, 2)     # NHWC memory
    wide = torch.zeros(off.shape[0], off.shape[2], off.shape[3], 64, dtype=dt, device='cuda')
    wide[..., :off.shape[1]] = off.to('cuda', dt).permute(0, 2, 3, 1)
    offd = wide[..., :off.shape[1]].permute(0, 3, 1, 2)                             # strided channel slice
    maskd = mask.to('cuda', dt) if mask is not None else None
    dev = [xd, offd, maskd, w.to('cuda', dt)]
    ref = _run(case, *(t.float().cpu() if t is not None else None for t in dev), grad_dtype=dt)
    got = _run(case, *[t.detach() if t is not None else None for t in dev])
    names = ['out', 'dx', 'doffset'] + (['dmask'] if mask is not None else []) + ['dweight']
    for name, a, b in zip(names, got, ref):
        err = (a - b).norm() / b.norm().clamp_min(1e-12)
        assert err < 3e-2, (name, float(err))
