"""Bucketed gradient all-reduce overlapped with backward.

Parity: the reference reduces gradients key by key through kvstore
(src/kvstore/comm.h CommDevice::Reduce, kvstore_nccl.h with
MXNET_KVSTORE_BIGARRAY_BOUND splitting).  On an MI355X node we instead:

* lay all gradients of one dtype out in a few large flat buffers ("buckets");
  each Parameter's ``.grad`` is a view into its bucket, so no pack/unpack
  copies are needed around the collective;
* register a post-accumulate hook per parameter; when the last gradient of a
  bucket is written during backward, an async RCCL all-reduce of that bucket
  is launched immediately, overlapping communication with the rest of the
  backward pass;
* size buckets for xGMI's point-to-point ring (``bucket_bytes_for``): big enough that the per-call
  latency is amortised, small enough that several buckets overlap with backward
  (``MXAMD_BUCKET_MB`` overrides).
"""
import os

import torch

from . import dist
from ..utils import env as _env

__all__ = ['GradBuckets', 'bucket_bytes_for']

# Cost model of one bucketed all-reduce on an MI355X node (8 GPUs, each with 7 point-to-point xGMI
# links; RCCL runs its rings over all of them): t(S) = ALPHA + S / BETA with ALPHA ~ 30 us launch +
# synchronisation latency and BETA ~ 150 GB/s algorithm bandwidth for large messages.  A bucket of
# S bytes then uses the links at S / (S + ALPHA * BETA): 78 % at 16 MB, 93 % at 64 MB.  Backward
# overlap wants several buckets (the last one is exposed), so the size is a quarter of the gradient
# bytes, clamped to [16, 64] MB: ResNet-50 fp16 (51 MB) -> 16 MB x 3-4, BERT-base bf16 (220 MB) ->
# 55 MB x 4.  With one rank there is nothing to reduce and bucketing only shapes the arenas.
_ALPHA_S = 30e-6
_BETA_BPS = 150e9
_MIN_BUCKET = 16 << 20
_MAX_BUCKET = 64 << 20


def bucket_bytes_for(total_bytes, world=None):
    """Bucket size (bytes) for ``total_bytes`` of gradients; ``MXAMD_BUCKET_MB`` overrides."""
    env = os.environ.get('MXAMD_BUCKET_MB')
    if env:
        return int(float(env) * (1 << 20))
    return int(min(_MAX_BUCKET, max(_MIN_BUCKET, total_bytes // 4)))


def link_efficiency(bucket_bytes):
    """Fraction of the xGMI all-reduce bandwidth a bucket of this size reaches in the model above."""
    return bucket_bytes / (bucket_bytes + _ALPHA_S * _BETA_BPS)


class _Bucket:
    __slots__ = ('flat', 'params', 'count', 'ready', 'handle', 'dtype', 'device')

    def __init__(self, dtype, device):
        self.flat = None
        self.params = []
        self.count = 0
        self.ready = 0
        self.handle = None
        self.dtype = dtype
        self.device = device


class GradBuckets:
    """Flat gradient buckets for a list of NDArray leaves (one context each)."""

    def __init__(self, arrays, grad_reqs, bucket_bytes=None, overlap=True, average=False):
        if bucket_bytes is None:
            total = sum(a._data.numel() * a._data.element_size() for a, r in zip(arrays, grad_reqs)
                        if r != 'null' and a._grad is not None)
            bucket_bytes = bucket_bytes_for(total)
        self.overlap = overlap and dist.world_size() > 1
        self.average = average
        self.buckets = []
        self._hooks = []
        # backward visits parameters roughly in reverse order of creation
        order = list(range(len(arrays)))[::-1]
        cur = {}
        for i in order:
            a, req = arrays[i], grad_reqs[i]
            if req == 'null' or a._grad is None:
                continue
            t = a._data
            key = (t.dtype, t.device)
            b = cur.get(key)
            nbytes = t.numel() * t.element_size()
            if b is None or (b.count and sum(p._data.numel() for p in b.params) * t.element_size() + nbytes > bucket_bytes):
                b = _Bucket(t.dtype, t.device)
                self.buckets.append(b)
                cur[key] = b
            b.params.append(a)
            b.count += 1
        for b in self.buckets:
            total = sum(p._data.numel() for p in b.params)
            b.flat = torch.zeros(total, dtype=b.dtype, device=b.device)
            off = 0
            for p in b.params:
                n = p._data.numel()
                view = b.flat[off:off + n].view(p._data.shape)
                with torch.no_grad():
                    view.copy_(p._grad._data)
                p._set_grad_buffer(view, p._grad_req)
                off += n
        if self.overlap:
            for b in self.buckets:
                if any(p._grad_req == 'add' for p in b.params):
                    continue
                for p in b.params:
                    self._hooks.append(p._data.register_post_accumulate_grad_hook(self._make_hook(b)))

    def _make_hook(self, b):
        def hook(_t):
            b.ready += 1
            if b.ready == b.count and b.handle is None:
                from .. import engine
                engine.join_workers()     # gradients written on side streams are complete first
                b.handle = dist.all_reduce(b.flat, async_op=True)
        return hook

    def zero(self):
        with torch.no_grad():
            for b in self.buckets:
                b.flat.zero_()

    def reduce(self):
        """Finish the all-reduce of every bucket (launch those not yet launched)."""
        ws = dist.world_size()
        for b in self.buckets:
            if ws > 1:
                if b.handle is None:
                    dist.all_reduce(b.flat)
                else:
                    b.handle.wait()
                if self.average:
                    b.flat.div_(ws)
            b.handle = None
            b.ready = 0

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
