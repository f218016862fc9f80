"""Convolutions whose output channels do not tile the MFMA kernels (SSD heads: anchors x (classes+1),
deformable offsets: 2 x taps) run with zero-padded output channels on the in-tree kernels; forward and
all gradients against an fp32 torch reference."""
import pytest
import torch

from mxnet_maintenance_amd.ops import hip_ops


@pytest.mark.gpu
@pytest.mark.parametrize('K,stride', [(84, 1), (18, 1), (126, 2)])
def test_padded_output_channels_match_fp32_reference(K, stride):
    from mxnet_maintenance_amd.ops import kernel_fns as KF
    assert KF.kpad_ok(torch.empty(1, 1, 1, 256), torch.empty(K, 3, 3, 256))
    g = torch.Generator().manual_seed(0)
    x = torch.randn(4, 256, 12, 12, generator=g)
    w = torch.randn(K, 256, 3, 3, generator=g) * 0.05
    b = torch.randn(K, generator=g)
    dev = [t.to('cuda', torch.float16).requires_grad_() for t in (x, w, b)]
    xl = dev[0].permute(0, 2, 3, 1).contiguous().permute(0, 3, 1, 2)     # channels-last memory
    y = hip_ops.conv(xl, dev[1], dev[2], (stride, stride), (1, 1), (1, 1), 1, False)
    gy = torch.linspace(-1, 1, y.numel()).reshape(y.shape)
    y.backward(gy.to('cuda', torch.float16))
    ref = [t.clone().requires_grad_() for t in (x, w, b)]
    yr = torch.nn.functional.conv2d(ref[0], ref[1], ref[2], stride=stride, padding=1)
    yr.backward(gy)
    for name, a, r in [('y', y.detach(), yr.detach())] + [(n, d.grad, rr.grad) for n, d, rr in
                                                         zip(('dx', 'dw', 'db'), dev, ref)]:
        err = float((a.float().cpu() - r).norm() / r.norm())
        assert err < 1e-2, (name, err)
