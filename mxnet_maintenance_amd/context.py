"""Device context.

Parity: python/mxnet/context.py (Context, cpu, gpu, cpu_pinned, num_gpus,
gpu_memory_info, current_context). A ``gpu(i)`` context is HIP device ``i``
(torch ``cuda:i`` on ROCm); one process normally drives one MI355X.
"""
import threading

import torch

__all__ = ['Context', 'cpu', 'gpu', 'cpu_pinned', 'cpu_shared', 'num_gpus',
           'gpu_memory_info', 'current_context', 'Device', 'device']


class _ContextMeta(type):
    """``Context.default_ctx`` is per thread (reference context.py:70: a ``threading.local``
    behind a class property): each thread starts on cpu(0) and ``with ctx:`` / assignment only
    change the calling thread's default."""

    @property
    def default_ctx(cls):
        return current_context()

    @default_ctx.setter
    def default_ctx(cls, ctx):
        Context._default_ctx.value = ctx


class Context(metaclass=_ContextMeta):
    """A device context: ``cpu``, ``gpu``, ``cpu_pinned`` or ``cpu_shared``."""
    _default_ctx = threading.local()
    devtype2str = {1: 'cpu', 2: 'gpu', 3: 'cpu_pinned', 5: 'cpu_shared'}
    devstr2type = {'cpu': 1, 'gpu': 2, 'cpu_pinned': 3, 'cpu_shared': 5}

    def __init__(self, device_type, device_id=0):
        if isinstance(device_type, Context):
            self.device_typeid = device_type.device_typeid
            self.device_id = device_type.device_id
        else:
            if isinstance(device_type, int):
                self.device_typeid = device_type
            else:
                self.device_typeid = Context.devstr2type[device_type]
            self.device_id = int(device_id)
        self._old_ctx = None

    @property
    def device_type(self):
        return Context.devtype2str[self.device_typeid]

    @property
    def torch_device(self):
        if self.device_typeid == 2:
            return torch.device('cuda', self.device_id)
        return torch.device('cpu')

    def __hash__(self):
        return hash((self.device_typeid, self.device_id))

    def __eq__(self, other):
        return (isinstance(other, Context) and self.device_typeid == other.device_typeid
                and self.device_id == other.device_id)

    def __str__(self):
        return '%s(%d)' % (self.device_type, self.device_id)

    __repr__ = __str__

    def __enter__(self):
        if not hasattr(Context._default_ctx, 'value'):
            Context._default_ctx.value = Context('cpu', 0)
        self._old_ctx = Context._default_ctx.value
        Context._default_ctx.value = self
        return self

    def __exit__(self, ptype, value, trace):
        Context._default_ctx.value = self._old_ctx

    def empty_cache(self):
        """Release pooled device memory back to the driver."""
        if self.device_typeid == 2 and torch.cuda.is_available():
            with torch.cuda.device(self.device_id):
                torch.cuda.empty_cache()


Device = Context


def cpu(device_id=0):
    return Context('cpu', device_id)


def cpu_pinned(device_id=0):
    return Context('cpu_pinned', device_id)


def cpu_shared(device_id=0):
    return Context('cpu_shared', device_id)


def gpu(device_id=0):
    return Context('gpu', device_id)


def device(dev_str):
    if ':' in dev_str:
        t, i = dev_str.split(':')
        return Context(t, int(i))
    return Context(dev_str, 0)


def num_gpus():
    """Number of visible MI355X devices (does not initialise HIP)."""
    try:
        return torch.cuda.device_count()
    except Exception:  # pragma: no cover
        return 0


def gpu_memory_info(device_id=0):
    """Return (free, total) bytes of HBM on ``device_id``."""
    free, total = torch.cuda.mem_get_info(device_id)
    return free, total


def current_context():
    if not hasattr(Context._default_ctx, 'value'):
        Context._default_ctx.value = Context('cpu', 0)
    return Context._default_ctx.value


def context_from_torch(dev):
    if dev.type == 'cuda':
        return Context('gpu', dev.index if dev.index is not None else torch.cuda.current_device())
    return Context('cpu', 0)

