"""Process-group management: one process per MI355X, RCCL over xGMI.

Parity: the role of ps-lite + src/kvstore/kvstore_dist.h (worker rank,
num_workers, barrier) and kvstore_nccl.h (NCCL communicator setup), re-done
as a ``torch.distributed`` process group: backend ``nccl`` (= RCCL on ROCm) for
GPU tensors, ``gloo`` for CPU tensors/tests.  Launch with
``python -m torch.distributed.run --nproc-per-node N ...`` (or
``tools/launch.py -n N``, ``parallel/launch.py``); RANK / WORLD_SIZE /
LOCAL_RANK / MASTER_ADDR / MASTER_PORT come from the environment.  When more
local ranks than visible GPUs are started (a one-GPU rehearsal of a multi-GPU
job) the group falls back to gloo, since RCCL needs a distinct GPU per rank.
"""
import datetime
import os

import torch
import torch.distributed as dist

__all__ = ['init', 'is_initialized', 'rank', 'world_size', 'local_rank', 'barrier', 'backend',
           'all_reduce', 'broadcast', 'all_gather', 'reduce_scatter', 'all_to_all']

_cpu_group = None


def is_initialized():
    return dist.is_available() and dist.is_initialized()


def init(backend=None, timeout_s=1800):
    """Initialise the default process group from the environment (idempotent)."""
    global _cpu_group
    if is_initialized():
        return
    ws = int(os.environ.get('WORLD_SIZE', '1'))
    if ws <= 1 and 'MASTER_ADDR' not in os.environ:
        return
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29500')
    if backend is None:
        backend = os.environ.get('MXAMD_DIST_BACKEND', '') or None
    if backend is None:
        backend = 'nccl' if torch.cuda.is_available() else 'gloo'
        # RCCL needs one GPU per rank; more local ranks than visible GPUs is a single-GPU rehearsal
        local_ws = int(os.environ.get('LOCAL_WORLD_SIZE', ws))
        if backend == 'nccl' and local_ws > torch.cuda.device_count():
            backend = 'gloo'
    if backend == 'nccl':
        torch.cuda.set_device(local_device())
    kw = {}
    if backend == 'nccl':
        kw['device_id'] = torch.device('cuda', local_device())
    dist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    if backend == 'nccl':
        _cpu_group = dist.new_group(backend='gloo')


def backend():
    return dist.get_backend() if is_initialized() else None


def cpu_group():
    return _cpu_group


def rank():
    return dist.get_rank() if is_initialized() else int(os.environ.get('RANK', '0'))


def world_size():
    return dist.get_world_size() if is_initialized() else 1


def local_rank():
    return int(os.environ.get('LOCAL_RANK', os.environ.get('RANK', '0')))


def local_device():
    """GPU index of this process (local rank modulo the visible devices)."""
    n = torch.cuda.device_count() if torch.cuda.is_available() else 0
    return local_rank() % n if n else 0


def barrier():
    if is_initialized():
        if backend() == 'nccl':
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def _group_for(t):
    if backend() == 'nccl' and not t.is_cuda:
        return _cpu_group
    return None


def all_reduce(t, op='sum', async_op=False):
    """In-place all-reduce of tensor ``t`` across all workers."""
    if world_size() <= 1:
        return None
    rop = {'sum': dist.ReduceOp.SUM, 'max': dist.ReduceOp.MAX, 'min': dist.ReduceOp.MIN}[op]
    return dist.all_reduce(t, op=rop, group=_group_for(t), async_op=async_op)


def broadcast(t, src=0, async_op=False):
    if world_size() <= 1:
        return None
    return dist.broadcast(t, src=src, group=_group_for(t), async_op=async_op)


def all_gather(t):
    """Return a tensor of shape (world, *t.shape) with every worker's ``t``."""
    ws = world_size()
    if ws <= 1:
        return t.unsqueeze(0)
    # flat (world*numel,) output: gloo's all_gather_into_tensor rejects a (world, ...) shaped one
    flat = torch.empty(ws * t.numel(), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(flat, t.contiguous().view(-1), group=_group_for(t))
    return flat.view((ws,) + tuple(t.shape))


def reduce_scatter(t):
    """Sum ``t`` (first dim divisible by world) across workers, return this rank's shard."""
    ws = world_size()
    if ws <= 1:
        return t
    shard = (t.shape[0] // ws,) + tuple(t.shape[1:])
    out = torch.empty(t.numel() // ws, dtype=t.dtype, device=t.device)
    dist.reduce_scatter_tensor(out, t.contiguous().view(-1), group=_group_for(t))
    return out.view(shard)


def all_to_all(t):
    """Exchange equal chunks of dim 0 between all workers."""
    ws = world_size()
    if ws <= 1:
        return t
    out = torch.empty_like(t)
    dist.all_to_all_single(out, t.contiguous(), group=_group_for(t))
    return out
