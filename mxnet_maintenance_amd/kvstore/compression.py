"""2-bit gradient compression with error feedback.

Parity: src/kvstore/gradient_compression.{h,cc,cu} and
gradient_compression-inl.h (type '2bit', ``threshold``; residual
accumulation; values quantised to {-threshold, 0, +threshold}).

Transport on MI355X: instead of pushing compressed blobs to ps-lite servers,
every worker all-gathers the packed 2-bit codes (4 codes per byte, 16x smaller
than fp32) over RCCL and decodes + sums locally, which cuts xGMI traffic 4-8x
versus an fp32 ring all-reduce at 8 GPUs.
"""
import torch

from ..parallel import dist

__all__ = ['GradientCompression', 'quantize_2bit', 'dequantize_2bit']


def quantize_2bit(grad, residual, threshold):
    """Return packed uint8 codes (4 per byte); updates ``residual`` in place."""
    residual.add_(grad.float().reshape(-1))
    pos = residual >= threshold
    neg = residual <= -threshold
    residual.sub_(pos.float() * threshold).add_(neg.float() * threshold)
    codes = (pos.to(torch.uint8) * 3) | (neg.to(torch.uint8) * 2)
    n = codes.numel()
    pad = (-n) % 4
    if pad:
        codes = torch.cat([codes, torch.zeros(pad, dtype=torch.uint8, device=codes.device)])
    c = codes.view(-1, 4)
    packed = c[:, 0] | (c[:, 1] << 2) | (c[:, 2] << 4) | (c[:, 3] << 6)
    return packed


def dequantize_2bit(packed, n, threshold, dtype=torch.float32):
    c = torch.stack([(packed >> s) & 3 for s in (0, 2, 4, 6)], dim=1).reshape(-1)[:n]
    out = torch.zeros(n, dtype=dtype, device=packed.device)
    out = torch.where(c == 3, torch.full_like(out, threshold), out)
    out = torch.where(c == 2, torch.full_like(out, -threshold), out)
    return out


class GradientCompression:
    def __init__(self, type='2bit', threshold=0.5):  # pylint: disable=redefined-builtin
        if type != '2bit':
            raise ValueError('Unknown type for gradient compression: %s' % type)
        if threshold <= 0:
            raise ValueError('threshold must be greater than 0')
        self.type = type
        self.threshold = float(threshold)
        self._residuals = {}

    def get_params(self):
        return {'type': self.type, 'threshold': self.threshold}

    def residual(self, key, t):
        """The error-feedback residual of kvstore key ``key`` (one per key, like comm.h buf.residual)."""
        res = self._residuals.get(key)
        if res is None or res.numel() != t.numel() or res.device != t.device:
            res = torch.zeros(t.numel(), dtype=torch.float32, device=t.device)
            self._residuals[key] = res
        return res

    def allreduce(self, t, key=None):
        """Sum ``t`` over workers through 2-bit codes; ``key`` selects the residual."""
        if key is None:
            key = ('anon', tuple(t.shape), t.dtype)
        res = self.residual(key, t)
        lib = _hip(t)
        if lib is not None:
            # gfx950 kernels: quantise (+ residual update) and decode-and-sum of all ranks in one pass each
            from ..ops.kernel_fns import _DT, _stream
            n = t.numel()
            g = t.contiguous()
            packed = torch.empty(((n + 15) // 16) * 4, dtype=torch.uint8, device=t.device)
            lib.twobit_quantize(_DT[g.dtype], g.data_ptr(), res.data_ptr(), packed.data_ptr(), n, self.threshold,
                                _stream())
            allp = dist.all_gather(packed).contiguous()
            total = torch.empty(n, dtype=torch.float32, device=t.device)
            lib.twobit_dequantize_sum(allp.data_ptr(), packed.numel(), allp.shape[0], n, self.threshold,
                                      total.data_ptr(), _stream())
            t.copy_(total.view(t.shape).to(t.dtype))
            return
        packed = quantize_2bit(t, res, self.threshold)
        allp = dist.all_gather(packed)
        total = torch.zeros(t.numel(), dtype=torch.float32, device=t.device)
        for i in range(allp.shape[0]):
            total.add_(dequantize_2bit(allp[i], t.numel(), self.threshold))
        t.copy_(total.view(t.shape).to(t.dtype))


def _hip(t):
    if not t.is_cuda or t.dtype not in (torch.float32, torch.float16, torch.bfloat16):
        return None
    from ..ops import kernels as _K
    if _K.enabled() and _K.available():
        return _K.lib()
    return None
