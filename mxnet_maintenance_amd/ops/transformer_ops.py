"""Multi-head attention building blocks (parity: src/operator/contrib/transformer.cc,
transformer.cu: interleaved_matmul_{selfatt,encdec}_{qk,valatt}, div_sqrt_dim) plus a
fused scaled-dot-product attention op.

Layouts follow the reference: projections are (seq, batch, heads*head_dim*{3|2})
with q/k/v interleaved per head, attention scores are (batch*heads, q_len, k_len).
The batched GEMMs go to hipBLASLt through ``torch.bmm``/``baddbmm`` (scale folded
into the GEMM's alpha); ``_contrib_sdp_attention`` dispatches to the ROCm
flash-attention kernel behind ``scaled_dot_product_attention``.
"""
import math

import torch
import torch.nn.functional as F

from .registry import register


def _split_heads(x, heads, parts, which):
    """(S, B, H*parts*D) interleaved -> (B*H, S, D) for component ``which``."""
    S, B, C = x.shape
    D = C // (heads * parts)
    t = x.reshape(S, B, heads, parts, D)[:, :, :, which, :]
    return t.permute(1, 2, 0, 3).reshape(B * heads, S, D), D


def _merge_heads(o, heads):
    """(B*H, S, D) -> (S, B, H*D)."""
    BH, S, D = o.shape
    B = BH // heads
    return o.reshape(B, heads, S, D).permute(2, 0, 1, 3).reshape(S, B, heads * D)


def _scaled_qk(q, k, D):
    out = torch.empty(q.shape[0], q.shape[1], k.shape[1], dtype=q.dtype, device=q.device)
    return torch.baddbmm(out, q, k.transpose(1, 2), beta=0.0, alpha=1.0 / math.sqrt(D))


@register('_contrib_interleaved_matmul_selfatt_qk', aliases=('interleaved_matmul_selfatt_qk',),
          arg_names=('queries_keys_values',), params={'heads': ('int', 1)})
def selfatt_qk(queries_keys_values, heads=1):
    q, D = _split_heads(queries_keys_values, heads, 3, 0)
    k, _ = _split_heads(queries_keys_values, heads, 3, 1)
    return _scaled_qk(q, k, D)


@register('_contrib_interleaved_matmul_selfatt_valatt', aliases=('interleaved_matmul_selfatt_valatt',),
          arg_names=('queries_keys_values', 'attention'), params={'heads': ('int', 1)})
def selfatt_valatt(queries_keys_values, attention, heads=1):
    v, _ = _split_heads(queries_keys_values, heads, 3, 2)
    return _merge_heads(torch.bmm(attention.to(v.dtype), v), heads)


@register('_contrib_interleaved_matmul_encdec_qk', aliases=('interleaved_matmul_encdec_qk',),
          arg_names=('queries', 'keys_values'), params={'heads': ('int', 1)})
def encdec_qk(queries, keys_values, heads=1):
    q, D = _split_heads(queries, heads, 1, 0)
    k, _ = _split_heads(keys_values, heads, 2, 0)
    return _scaled_qk(q, k, D)


@register('_contrib_interleaved_matmul_encdec_valatt', aliases=('interleaved_matmul_encdec_valatt',),
          arg_names=('keys_values', 'attention'), params={'heads': ('int', 1)})
def encdec_valatt(keys_values, attention, heads=1):
    v, _ = _split_heads(keys_values, heads, 2, 1)
    return _merge_heads(torch.bmm(attention.to(v.dtype), v), heads)


@register('_contrib_sdp_attention', aliases=('sdp_attention',),
          arg_names=lambda a: ['queries_keys_values'] + (['mask'] if str(a.get('use_mask', False)) in
                                                         ('True', 'true', '1') else []),
          params={'heads': ('int', 1), 'dropout': ('float', 0.0), 'causal': ('bool', False),
                  'use_mask': ('bool', False)})
def sdp_attention(queries_keys_values, mask=None, heads=1, dropout=0.0, causal=False, use_mask=False):
    """Fused self-attention on an interleaved (S, B, H*3*D) projection -> (S, B, H*D).

    ``mask`` (B, S_k) with 1 = attend, 0 = padding (valid-length masking)."""
    from .. import _state
    from .hip_ops import _use_hip
    x = queries_keys_values
    p = dropout if _state.STATE.training else 0.0
    if _use_hip(x):
        from .attention_fns import SelfAttention, attention_ok
        if attention_ok(x, heads, causal):
            # hand-written gfx950 kernels: no (B*H, S, S) scores, gradient straight into the qkv layout
            return SelfAttention.apply(x, mask, heads, float(p))
    S, B, C = x.shape
    D = C // (heads * 3)
    t = x.reshape(S, B, heads, 3, D).permute(3, 1, 2, 0, 4)     # (3, B, H, S, D)
    q, k, v = t[0], t[1], t[2]
    am = None
    if mask is not None:
        am = mask.bool().reshape(B, 1, 1, -1)
    o = F.scaled_dot_product_attention(q, k, v, attn_mask=am, dropout_p=p, is_causal=causal and am is None)
    return o.permute(2, 0, 1, 3).reshape(S, B, heads * D)
