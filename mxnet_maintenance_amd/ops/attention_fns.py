"""torch.autograd wrapper for the fused self-attention kernels (src/kernels/attention.hip).

``SelfAttention.apply(qkv, mask, heads, p, scale)`` takes the interleaved
(S, B, H*3*D) projection of src/operator/contrib/transformer.cc and returns the
(S, B, H*D) context; its gradient is written straight into a (S, B, H*3*D)
buffer of the projection's layout, so neither direction runs permute/copy
kernels.  Dropout on the attention probabilities uses a stateless per-element
hash of (seed, position) that the backward regenerates; under HIP-graph
capture a device counter (``_state.GRAPH_RNG``) re-keys every replay.
Numerics vs an fp32 torch reference: tests/test_attention.py.
"""
import math

import torch

from . import kernels as _K
from .. import _state
from .kernel_fns import _DT, _stream

__all__ = ['SelfAttention', 'attention_ok']

_HEAD_DIM = 64
_MAX_SEQ = 256


def attention_ok(qkv, heads, causal=False):
    """True when the fused kernels support this call (else the op takes the SDPA path)."""
    if causal or qkv.dtype not in (torch.float16, torch.bfloat16) or qkv.dim() != 3:
        return False
    S, _, C = qkv.shape
    if C % (3 * heads) or C // (3 * heads) != _HEAD_DIM:
        return False
    return (S % 32 == 0 and 32 <= S <= _MAX_SEQ and qkv.is_contiguous() and qkv.data_ptr() % 16 == 0)


def _seed():
    # torch's default CPU generator, so mx.random.seed() makes attention dropout reproducible
    return int(torch.randint(0, 2 ** 62, (1,)).item())


class SelfAttention(torch.autograd.Function):

    @staticmethod
    def forward(ctx, qkv, mask, heads, p, scale=None):
        S, B, C = qkv.shape
        D = C // (3 * heads)
        scale = 1.0 / math.sqrt(D) if scale is None else float(scale)
        out = torch.empty(S, B, heads * D, dtype=qkv.dtype, device=qkv.device)
        lse = torch.empty(B * heads, S, dtype=torch.float32, device=qkv.device)
        km = None
        if mask is not None:
            km = mask.to(torch.float32).reshape(B, S).contiguous()
        seed = _seed() if p > 0 else 0
        ctr = _state.GRAPH_RNG[0] if (p > 0 and torch.cuda.is_current_stream_capturing()) else None
        _K.lib().attention_forward(_DT[qkv.dtype], qkv.data_ptr(), 0 if km is None else km.data_ptr(),
                                   out.data_ptr(), lse.data_ptr(), S, B, heads, D, scale, float(p), seed,
                                   0 if ctr is None else ctr.data_ptr(), _stream())
        ctx.save_for_backward(qkv, out, lse, km)
        ctx.cfg = (heads, D, scale, float(p), seed, ctr)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse, km = ctx.saved_tensors
        heads, D, scale, p, seed, ctr = ctx.cfg
        S, B, _ = qkv.shape
        dout = dout.contiguous()
        dqkv = torch.empty_like(qkv)
        delta = torch.empty(B * heads, S, dtype=torch.float32, device=qkv.device)
        _K.lib().attention_backward(_DT[qkv.dtype], qkv.data_ptr(), 0 if km is None else km.data_ptr(),
                                    out.data_ptr(), dout.data_ptr(), lse.data_ptr(), delta.data_ptr(),
                                    dqkv.data_ptr(), S, B, heads, D, scale, p, seed,
                                    0 if ctr is None else ctr.data_ptr(), _stream())
        return dqkv, None, None, None, None
