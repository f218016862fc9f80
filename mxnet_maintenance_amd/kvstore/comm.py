"""Single-process multi-device reduction and broadcast for the 'local'/'device'/'nccl' stores.

Parity: src/kvstore/comm.h (CommCPU / CommDevice: per-key merge buffer placed on a
device chosen to balance bytes across devices, reduce then broadcast),
src/kvstore/comm_tree.h:50 (tree reduce over P2P links) and src/kvstore/kvstore_nccl.h:62
(in-process NCCL reduce/broadcast across the GPUs of one process).

MI355X design: when the copies of a key live on *distinct* GPUs, the reduction is one
in-process RCCL reduce (``torch.cuda.comm.reduce_add_coalesced``: keys are flattened into
coalesced buffers of ``MXNET_KVSTORE_REDUCTION_BUCKET`` bytes, one collective per bucket over
xGMI) and the result fans out with one coalesced RCCL broadcast.  Each key's root device is
assigned greedily to the device with the fewest merge-buffer bytes so far (the reference's
CommDevice placement), so roots spread over the 8 GPUs and the xGMI links are loaded evenly.
Copies on the same device (or on the host) are summed directly without any transfer.
"""
import os

import torch

_BUCKET = int(os.environ.get('MXNET_KVSTORE_REDUCTION_BUCKET', str(64 << 20)))


def _distinct_gpus(ts):
    devs = [t.device for t in ts]
    return all(d.type == 'cuda' for d in devs) and len(set(devs)) == len(devs) and len(devs) > 1


def _rccl_ok(ts):
    try:
        from torch.cuda import nccl
        return nccl.is_available(ts)
    except Exception:     # pylint: disable=broad-except
        return False


def _reduce_coalesced(inputs, destination, buffer_size):
    """One in-process RCCL reduce per coalesced bucket (indirection point for tests)."""
    return torch.cuda.comm.reduce_add_coalesced(inputs, destination=destination, buffer_size=buffer_size)


def _broadcast_coalesced(tensors, devices, buffer_size):
    """One in-process RCCL broadcast per coalesced bucket (indirection point for tests)."""
    return torch.cuda.comm.broadcast_coalesced(tensors, devices, buffer_size=buffer_size)


def _rccl_broadcast_ok(src, dsts):
    devs = [d.device for d in dsts]
    return len(dsts) > 1 and src.device in devs and _distinct_gpus(dsts)


class DeviceComm:
    """Reduce/broadcast helper keyed by kvstore key (root placement is sticky per key)."""

    def __init__(self):
        self._root = {}          # key -> root device index into the value list's devices
        self._load = {}          # torch.device -> merge bytes assigned

    def root_for(self, key, ts):
        r = self._root.get(key)
        if r is None or r >= len(ts):
            devs = [t.device for t in ts]
            r = min(range(len(ts)), key=lambda i: (self._load.get(devs[i], 0), i))
            self._load[devs[r]] = self._load.get(devs[r], 0) + ts[r].numel() * ts[r].element_size()
            self._root[key] = r
        return r

    def reduce(self, keys, value_lists):
        """Sum every key's per-device copies.  Returns one tensor per key (a fresh buffer on the
        key's root device; a single copy is returned as is)."""
        out = [None] * len(keys)
        groups = {}
        for i, (k, vs) in enumerate(zip(keys, value_lists)):
            if len(vs) == 1:
                out[i] = vs[0]
                continue
            if _distinct_gpus(vs) and _rccl_ok(vs):
                r = self.root_for(k, vs)
                sig = (tuple(t.device for t in vs), r, vs[0].dtype)
                groups.setdefault(sig, []).append(i)
                continue
            out[i] = self._sum_local(vs, self.root_for(k, vs))
        for (devs, r, _), idx in groups.items():
            # inputs[d] = the tensors of device d for every key of the group
            inputs = [[value_lists[i][d].contiguous() for i in idx] for d in range(len(devs))]
            sums = _reduce_coalesced(inputs, devs[r].index, _BUCKET)
            for i, s in zip(idx, sums):
                out[i] = s
        return out

    @staticmethod
    def _sum_local(vs, r):
        dev = vs[r].device
        acc = vs[r].clone()
        for j, v in enumerate(vs):
            if j != r:
                # device-to-device copies are stream-ordered; anything touching the host stays blocking
                acc.add_(v.to(dev, non_blocking=v.device.type == 'cuda' and dev.type == 'cuda'))
        return acc

    @staticmethod
    def broadcast(srcs, dst_lists):
        """Copy every ``srcs[i]`` into each tensor of ``dst_lists[i]`` (coalesced RCCL broadcast
        when the destinations are on distinct GPUs)."""
        groups = {}
        for i, (s, ds) in enumerate(zip(srcs, dst_lists)):
            if _rccl_broadcast_ok(s, ds):
                devs = tuple(d.device for d in ds)
                groups.setdefault((devs, devs.index(s.device), s.dtype), []).append(i)
                continue
            for d in ds:
                if d.data_ptr() != s.data_ptr():
                    d.data.copy_(s)
        for (devs, src_pos, _), idx in groups.items():
            # positions in the destination list, the source's first (broadcast_coalesced's contract)
            order = [src_pos] + [p for p in range(len(devs)) if p != src_pos]
            outs = _broadcast_coalesced([srcs[i] for i in idx], [devs[p].index for p in order], _BUCKET)
            for p, copies in zip(order, outs):
                for i, c in zip(idx, copies):
                    dst = dst_lists[i][p]
                    if dst.data_ptr() != c.data_ptr():
                        dst.data.copy_(c)
