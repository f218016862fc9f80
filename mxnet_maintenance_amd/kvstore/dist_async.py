"""``dist_async``: an asynchronous parameter server.

Parity: src/kvstore/kvstore_dist.h + kvstore_dist_server.h with
``sync_mode_ = false`` (python/mxnet/kvstore/kvstore.py ``create('dist_async')``):
workers push gradients and pull weights without waiting for each other; the
server applies every push to its copy of the weight as soon as it arrives
(with the optimizer set through ``set_optimizer``, or by assignment when none
is set), so workers train on weights that may be a few updates stale.

MI355X design: the synchronous data-parallel paths use RCCL collectives over
xGMI (kvstore.KVStore); a parameter server has no collective structure, so it
runs on the host over ``torch.distributed.rpc`` (TensorPipe, TCP): rank 0's
process hosts the server state next to its worker, every worker reaches it
with ``rpc_async`` (push) / ``rpc_sync`` (pull).  Values travel as CPU fp32
tensors; the server keeps fp32 weights and optimizer states.  Push returns
immediately (the returned futures are only awaited by ``pull`` of the same key
from the same worker, which preserves that worker's own read-after-write
order), so gradient transfer overlaps with the next forward/backward.

Rendezvous: RANK / WORLD_SIZE / MASTER_ADDR from the environment (as set by
``torch.distributed.run`` or tools/launch.py); the RPC agent listens on
``MXAMD_PS_PORT`` (default MASTER_PORT + 17, so it never collides with the
process group's store).
"""
import atexit
import os
import pickle
import threading

import torch

from ..base import MXNetError
from ..ndarray.ndarray import NDArray
from .. import optimizer as opt
from .kvstore import KVStoreBase

__all__ = ['KVStoreDistAsync']


# ------------------------------------------------------------------ server state (lives in rank 0's process)
class _Server:
    def __init__(self):
        self.lock = threading.Lock()
        self.store = {}
        self.updater = None
        self.pushes = 0
        self.barrier_cv = threading.Condition()
        self.barrier_count = 0
        self.barrier_gen = 0


_SERVER = _Server()


def _srv_init(key, value):
    with _SERVER.lock:
        if key not in _SERVER.store:        # the first init wins (workers all init the same key)
            _SERVER.store[key] = value.float().clone()
    return True


def _srv_push(key, grad):
    with _SERVER.lock:
        if key not in _SERVER.store:
            raise KeyError('dist_async: key %r pushed before init' % (key,))
        w = _SERVER.store[key]
        if _SERVER.updater is None:
            # reference: kvstore_dist_server.h CHECK(updater_) 'Updater needs to be set for async mode'
            raise MXNetError('dist_async: push before set_optimizer -- the server needs an updater '
                             '(kv.set_optimizer(...)) to apply asynchronous pushes')
        wn, gn = NDArray(w), NDArray(grad.float())
        _SERVER.updater(key, gn, wn)
        _SERVER.store[key] = wn._data
        _SERVER.pushes += 1
    return True


def _srv_pull(key):
    with _SERVER.lock:
        if key not in _SERVER.store:
            raise KeyError('dist_async: key %r pulled before init' % (key,))
        return _SERVER.store[key].clone()


def _srv_set_optimizer(blob):
    optimizer = pickle.loads(blob)
    with _SERVER.lock:
        _SERVER.updater = opt.get_updater(optimizer)
    return True


def _srv_num_pushes():
    with _SERVER.lock:
        return _SERVER.pushes


def _srv_barrier(world):
    cv = _SERVER.barrier_cv
    with cv:
        gen = _SERVER.barrier_gen
        _SERVER.barrier_count += 1
        if _SERVER.barrier_count == world:
            _SERVER.barrier_count = 0
            _SERVER.barrier_gen += 1
            cv.notify_all()
        else:
            cv.wait_for(lambda: _SERVER.barrier_gen != gen, timeout=600)
    return True


# ------------------------------------------------------------------ worker-side store
_RPC_READY = [False]


def dedicated_server():
    """True when a separate server process (DMLC_ROLE=server, DMLC_NUM_SERVER >= 1) hosts the store;
    otherwise rank 0's worker process hosts it."""
    return int(os.environ.get('DMLC_NUM_SERVER', '0') or 0) > 0


def _server_name():
    return 'server' if dedicated_server() else 'worker0'


def _init_rpc(rank, world, name=None):
    """Join the RPC world: the workers (ranks 0..W-1) plus, with a dedicated server, rank W."""
    if _RPC_READY[0]:
        return
    from torch.distributed import rpc
    addr = os.environ.get('MASTER_ADDR', '127.0.0.1')
    port = int(os.environ.get('MXAMD_PS_PORT', int(os.environ.get('MASTER_PORT', '29500')) + 17))
    opts = rpc.TensorPipeRpcBackendOptions(init_method='tcp://%s:%d' % (addr, port), num_worker_threads=32,
                                           rpc_timeout=600)
    total = world + (1 if dedicated_server() else 0)
    rpc.init_rpc(name or 'worker%d' % rank, rank=rank, world_size=total, rpc_backend_options=opts)
    _RPC_READY[0] = True
    atexit.register(_shutdown_rpc)


def _shutdown_rpc():
    if _RPC_READY[0]:
        from torch.distributed import rpc
        _RPC_READY[0] = False
        try:
            rpc.shutdown(graceful=True)
        except Exception:     # pylint: disable=broad-except
            pass


def _keys(key):
    return list(key) if isinstance(key, (list, tuple)) else [key]


def _vals(v):
    return list(v) if isinstance(v, (list, tuple)) else [v]


class KVStoreDistAsync(KVStoreBase):
    """Asynchronous parameter-server KVStore (``mx.kv.create('dist_async')``)."""

    def __init__(self):
        self._rank = int(os.environ.get('RANK', '0'))
        self._world = int(os.environ.get('WORLD_SIZE', '1'))
        _init_rpc(self._rank, self._world)
        self._pending = {}          # key -> futures of this worker's in-flight pushes
        self._compression = None

    # -------------------------------------------------------------- plumbing
    @staticmethod
    def _call(fn, *args):
        from torch.distributed import rpc
        return rpc.rpc_sync(_server_name(), fn, args=args)

    def _wait_key(self, key):
        for f in self._pending.pop(key, []):
            f.wait()

    @staticmethod
    def _host(v):
        t = v._data if isinstance(v, NDArray) else torch.as_tensor(v)
        return t.detach().float().cpu()

    # -------------------------------------------------------------- KVStore API
    @property
    def type(self):
        return 'dist_async'

    @property
    def rank(self):
        return self._rank

    @property
    def num_workers(self):
        return self._world

    @staticmethod
    def is_capable(capability):
        if capability.lower() == KVStoreBase.OPTIMIZER:
            return True
        raise ValueError('Unknown capability: {}'.format(capability))

    def init(self, key, value):
        for k, v in zip(_keys(key), _vals(value) if isinstance(key, (list, tuple)) else [value]):
            v0 = _vals(v)[0]
            self._call(_srv_init, k, self._host(v0))

    def push(self, key, value, priority=0):
        from torch.distributed import rpc
        keys = _keys(key)
        values = _vals(value) if isinstance(key, (list, tuple)) else [value]
        for k, v in zip(keys, values):
            parts = _vals(v)
            g = self._host(parts[0])
            for p in parts[1:]:              # several local devices: sum before sending
                g += self._host(p)
            self._pending.setdefault(k, []).append(rpc.rpc_async(_server_name(), _srv_push, args=(k, g)))

    def pull(self, key, out=None, priority=0, ignore_sparse=True):
        assert out is not None
        keys = _keys(key)
        outs = _vals(out) if isinstance(key, (list, tuple)) else [out]
        for k, o in zip(keys, outs):
            self._wait_key(k)                # this worker's own pushes land before its pull
            w = self._call(_srv_pull, k)
            for oo in _vals(o):
                with torch.no_grad():
                    oo._data.copy_(w.to(oo._data.device, oo._data.dtype))

    def pushpull(self, key, value, out=None, priority=0):
        self.push(key, value, priority)
        if out is not None:
            self.pull(key, out, priority)

    def broadcast(self, key, value, out, priority=0):
        self.init(key, value)
        self.pull(key, out, priority)

    def row_sparse_pull(self, key, out=None, priority=0, row_ids=None):
        self.pull(key, out, priority)

    def set_optimizer(self, optimizer):
        # every worker may call this; the server keeps the last one (they are identical)
        self._call(_srv_set_optimizer, pickle.dumps(optimizer))

    def set_gradient_compression(self, compression_params):
        raise MXNetError('gradient compression is not supported by the dist_async parameter server')

    def save_optimizer_states(self, fname, dump_optimizer=False):
        raise MXNetError('optimizer states live on the dist_async server')

    def load_optimizer_states(self, fname):
        raise MXNetError('optimizer states live on the dist_async server')

    def _barrier(self):
        for k in list(self._pending):
            self._wait_key(k)
        self._call(_srv_barrier, self._world)

    def server_push_count(self):
        """Number of pushes the server has applied so far (diagnostics/tests)."""
        return self._call(_srv_num_pushes)
