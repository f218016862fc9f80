"""Key-value store for data-parallel training.

Parity: python/mxnet/kvstore/kvstore.py (KVStore: init, push, pull, pushpull,
broadcast, row_sparse_pull, set_optimizer, set_gradient_compression,
save/load_optimizer_states, rank, num_workers, type, _barrier) and
python/mxnet/kvstore/base.py (KVStoreBase registry, TestStore, create);
src/kvstore/{kvstore_local.h, comm.h, kvstore_nccl.h, kvstore_dist.h,
gradient_compression*}.

MI355X design:
* one process per GPU; the cross-device reduction is an RCCL all-reduce over
  xGMI (``torch.distributed`` backend 'nccl') instead of the reference's
  in-process tree reduce / ps-lite servers;
* values given as a list (several contexts in one process, e.g. CPU tests) are
  summed locally first;
* a list of keys is reduced as ONE flattened collective per dtype (bucket
  fusion), so per-key launch latency does not dominate on ResNet-sized models;
* ``dist_async`` is an asynchronous parameter server over torch.distributed.rpc
  (kvstore/dist_async.py): pushes are applied by the server as they arrive.
"""
import os
import pickle
import warnings

import numpy as np
import torch

from .comm import DeviceComm

from .. import engine as _engine_mod
from ..base import MXNetError, string_types
from ..ndarray.ndarray import NDArray
from .. import optimizer as opt
from ..parallel import dist
from .compression import GradientCompression

__all__ = ['KVStoreBase', 'KVStore', 'TestStore', 'create']


def _as_list(x):
    return list(x) if isinstance(x, (list, tuple)) else [x]


class KVStoreBase:
    """Abstract interface; subclasses registered with ``KVStoreBase.register``."""
    OPTIMIZER = 'optimizer'
    kv_registry = {}

    def broadcast(self, key, value, out, priority=0):
        raise NotImplementedError()

    def pushpull(self, key, value, out=None, priority=0):
        raise NotImplementedError()

    def set_optimizer(self, optimizer):
        raise NotImplementedError()

    @staticmethod
    def is_capable(capability):
        raise NotImplementedError()

    def save_optimizer_states(self, fname, dump_optimizer=False):
        raise NotImplementedError()

    def load_optimizer_states(self, fname):
        raise NotImplementedError()

    @property
    def type(self):
        raise NotImplementedError()

    @property
    def rank(self):
        raise NotImplementedError()

    @property
    def num_workers(self):
        raise NotImplementedError()

    @staticmethod
    def register(klass):
        assert isinstance(klass, type)
        name = klass.__name__.lower()
        if name in KVStoreBase.kv_registry:
            warnings.warn('WARNING: New kvstore %s.%s is overriding existing kvstore %s.%s' % (
                klass.__module__, klass.__name__, KVStoreBase.kv_registry[name].__module__,
                KVStoreBase.kv_registry[name].__name__))
        KVStoreBase.kv_registry[name] = klass
        return klass


@KVStoreBase.register
class TestStore(KVStoreBase):
    """A minimal single-process store used to test the KVStoreBase plumbing."""

    def broadcast(self, key, value, out, priority=0):
        out = _as_list(out)
        for o in out:
            o[:] = value

    def pushpull(self, key, value, out=None, priority=0):
        value = _as_list(value)
        out = value if out is None else _as_list(out)
        total = value[0].copy()
        for v in value[1:]:
            total += v.as_in_context(total.context)
        for o in out:
            o[:] = total.as_in_context(o.context)

    @staticmethod
    def is_capable(capability):
        if capability.lower() == KVStoreBase.OPTIMIZER:
            return False
        raise ValueError('Unknown capability: {}'.format(capability))

    @property
    def type(self):
        return 'teststore'

    @property
    def rank(self):
        return 0

    @property
    def num_workers(self):
        return 1

    def set_optimizer(self, optimizer):
        raise NotImplementedError()

    def save_optimizer_states(self, fname, dump_optimizer=False):
        raise NotImplementedError()

    def load_optimizer_states(self, fname):
        raise NotImplementedError()


class KVStore(KVStoreBase):
    """RCCL-backed key-value store (types local/device/nccl/dist_*/horovod)."""

    def __init__(self, kvtype='local'):
        self._type = kvtype
        if kvtype.startswith('dist') or kvtype in ('nccl', 'device', 'horovod', 'byteps'):
            dist.init()
        self._store = {}
        self._updater = None
        self._optimizer = None
        self._compression = None
        self._str_keys = {}
        self._key_kind = None          # int or str: a store takes one kind of key (reference KVStore)

    # ---------------------------------------------------------------- basics
    @property
    def type(self):
        return self._type

    @property
    def rank(self):
        return dist.rank()

    @property
    def num_workers(self):
        return dist.world_size()

    @staticmethod
    def is_capable(capability):
        if capability.lower() == KVStoreBase.OPTIMIZER:
            return True
        raise ValueError('Unknown capability: {}'.format(capability))

    def _barrier(self):
        dist.barrier()

    def _send_command_to_servers(self, head, body):
        pass

    def num_dead_node(self, node_id, timeout=60):
        return 0

    # ------------------------------------------------------------ reductions
    def _local_sums(self, keys, vals):
        """Per-key sums over the devices of this process (comm.py: in-process RCCL reduce when the
        copies sit on distinct GPUs, balanced root placement).  A single copy is returned as is."""
        if getattr(self, '_comm', None) is None:
            self._comm = DeviceComm()
        return self._comm.reduce(keys, [[v._data for v in _as_list(v)] for v in vals])

    def _fan_out(self, srcs, outs):
        if getattr(self, '_comm', None) is None:
            self._comm = DeviceComm()
        self._comm.broadcast(srcs, [[o._data for o in _as_list(o)] for o in outs])

    def _allreduce_many(self, tensors, keys=None):
        """All-reduce a list of tensors with one fused collective per (dtype, device).

        ``keys`` name the kvstore keys the tensors belong to: gradient compression
        keeps one error-feedback residual per key (reference comm.h ``buf.residual``).
        """
        if dist.world_size() <= 1 or not tensors:
            return
        if self._compression is not None:
            keys = keys if keys is not None else list(range(len(tensors)))
            for k, t in zip(keys, tensors):
                self._compression.allreduce(t, key=k)
            return
        groups = {}
        for t in tensors:
            groups.setdefault((t.dtype, t.device), []).append(t)
        for ts in groups.values():
            if len(ts) == 1:
                dist.all_reduce(ts[0])
                continue
            flat = torch.cat([t.reshape(-1) for t in ts])
            dist.all_reduce(flat)
            off = 0
            for t in ts:
                n = t.numel()
                t.copy_(flat[off:off + n].view(t.shape))
                off += n

    # ------------------------------------------------------------ engine scheduling
    def _on_engine(self, fn, reads, writes, name):
        """Run the communication ``fn`` as one dependency-engine device op on the device's comm
        stream (reference: KVStoreLocal/KVStoreNCCL push their reduce/broadcast through
        Engine::PushAsync with the arrays' variables).  The op reads the variables of ``reads``,
        writes those of ``writes`` and this store's own variable (one total order of collectives
        per process, the same on every rank); it starts after the work already queued on the
        caller's stream (which produced the gradients), and the caller's stream waits on the GPU
        for it before anything queued later can touch ``writes``.  Host arrays, and processes
        without the native engine, run ``fn`` in place."""
        from .. import engine
        flat_r = [a for v in reads for a in _as_list(v)]
        flat_w = [a for v in writes for a in _as_list(v)]
        dev = next((a._data.device for a in flat_r + flat_w if a._data.is_cuda), None)
        # one comm stream orders one device's work: arrays spread over several GPUs of this process
        # (each with its own caller streams) run in place instead
        multi = len({a._data.device for a in flat_r + flat_w if a._data.is_cuda}) > 1
        if dev is None or multi or not engine.native_available() or torch.cuda.is_current_stream_capturing() or \
                _env_flag('MXAMD_KVSTORE_ENGINE', True) is False:
            fn()
            return
        if getattr(self, '_engine_var', None) is None:
            self._engine_var = engine.new_var('kvstore')
        comm = engine.comm_stream(dev)
        producer = torch.cuda.current_stream(dev)
        ready = torch.cuda.Event()
        ready.record(producer)
        wvars = [engine.var_of(a) for a in flat_w]
        rvars = [engine.var_of(a) for a in flat_r if all(engine.var_of(a) is not w for w in wvars)]
        for a in flat_r + flat_w:
            a._data.record_stream(comm)

        def op():
            torch.cuda.current_stream().wait_event(ready)
            with torch.no_grad():
                fn()
        engine.push_device(op, rvars, [self._engine_var] + wvars, stream=comm, name=name)
        try:
            for v in wvars:
                engine.stream_wait_var(v, producer)
        except Exception:
            # the failure is reported here, once: clear it from the store's ordering variable and
            # from the other outputs, so the next collective on this store runs again
            engine.clear_exception(self._engine_var)
            for v in wvars:
                engine.clear_exception(v)
            raise

    # ------------------------------------------------------------------- API
    def _keys(self, key):
        """``key`` as a list, checked against the store's key kind (all int or all str)."""
        keys = _as_list(key)
        for k in keys:
            kind = str if isinstance(k, str) else int
            if not isinstance(k, (str, int, np.integer)):
                raise MXNetError('kvstore keys must be int or str, got %s' % type(k).__name__)
            if self._key_kind is None:
                self._key_kind = kind
            elif kind is not self._key_kind:
                raise MXNetError('this kvstore uses %s keys; got the %s key %r'
                                 % (self._key_kind.__name__, kind.__name__, k))
        return keys

    def init(self, key, value):
        keys = self._keys(key)
        vals = value if isinstance(key, (list, tuple)) else [value]
        for k, v in zip(keys, vals):
            v0 = _as_list(v)[0]
            t = v0._data.detach().clone()
            if dist.world_size() > 1:
                dist.broadcast(t, 0)
            self._store[k] = NDArray(t)

    def push(self, key, value, priority=0):
        _engine_mod.join_workers()
        keys = self._keys(key)
        vals = value if isinstance(key, (list, tuple)) else [value]
        merged = []
        with torch.no_grad():
            for v, m in zip(vals, self._local_sums(keys, vals)):
                merged.append(m.clone() if len(_as_list(v)) == 1 else m)
            self._allreduce_many(merged, keys)
            for k, m in zip(keys, merged):
                if k not in self._store:
                    raise MXNetError('key %s has not been initialized' % str(k))
                stored = self._store[k]
                if self._updater is not None:
                    # string-keyed stores hand the updater the string key, like the reference's str updater
                    self._updater(k, NDArray(m), stored)
                else:
                    stored._data.copy_(m.to(stored._data.device, stored._data.dtype))

    def _str_key(self, k):
        if k not in self._str_keys:
            self._str_keys[k] = len(self._str_keys)
        return self._str_keys[k]

    def pull(self, key, out=None, priority=0, ignore_sparse=True):
        _engine_mod.join_workers()
        assert out is not None
        keys = self._keys(key)
        outs = out if isinstance(key, (list, tuple)) else [out]
        if ignore_sparse:
            # a row_sparse destination is left untouched (reference kvstore.pull: use row_sparse_pull)
            kept = [(k, o) for k, o in zip(keys, outs)
                    if not all(getattr(x, 'stype', 'default') == 'row_sparse' for x in _as_list(o))]
            if len(kept) != len(keys):
                keys = [k for k, _ in kept]
                outs = [o for _, o in kept]
        # written through .data: a pull into a parameter is an engine-ordered write in the
        # reference, not an autograd-visible in-place op on a recorded leaf
        stored = [self._store[k] for k in keys]

        def comm():
            with torch.no_grad():
                self._fan_out([st._data for st in stored], outs)
        self._on_engine(comm, stored, outs, 'kvstore_pull')

    def pushpull(self, key, value, out=None, priority=0):
        """Sum ``value`` over devices and workers and write the result to ``out``.

        With an optimizer set (update_on_kvstore) this is push + pull; otherwise
        it is an in-place all-reduce (the Gluon Trainer fast path).
        """
        _engine_mod.join_workers()
        if self._updater is not None:
            self.push(key, value, priority)
            self.pull(key, out if out is not None else value, priority)
            return
        keys = self._keys(key)
        vals = value if isinstance(key, (list, tuple)) else [value]
        outs = vals if out is None else (out if isinstance(key, (list, tuple)) else [out])

        def comm():
            with torch.no_grad():
                sums = self._local_sums(keys, vals)
                self._allreduce_many(sums, keys)
                self._fan_out(sums, outs)
        self._on_engine(comm, vals, outs, 'kvstore_pushpull')

    def broadcast(self, key, value, out, priority=0):
        self.init(key, value)
        self.pull(key, out, priority)

    def row_sparse_pull(self, key, out=None, priority=0, row_ids=None):
        _engine_mod.join_workers()
        assert out is not None and row_ids is not None
        keys = self._keys(key)
        outs = out if isinstance(key, (list, tuple)) else [out]
        rids = row_ids if isinstance(row_ids, (list, tuple)) and isinstance(key, (list, tuple)) else [row_ids]
        from ..ndarray.sparse import RowSparseNDArray
        for o in outs:
            for oo in _as_list(o):
                if getattr(oo, 'stype', 'default') != 'row_sparse':
                    raise MXNetError('row_sparse_pull: out must be a row_sparse NDArray, got %s storage'
                                     % getattr(oo, 'stype', type(oo).__name__))
        with torch.no_grad():
            for k, o, r in zip(keys, outs, rids):
                st = self._store[k]
                src = st._data if not isinstance(st, RowSparseNDArray) else None
                for oo, rr in zip(_as_list(o), _as_list(r) * len(_as_list(o))):
                    dev = (src.device if src is not None else st._values().device)
                    idx = torch.unique(rr._data.to(torch.int64).reshape(-1).to(dev))   # sorted, no duplicates
                    # only the requested rows move: no dense zeros tensor of the full weight
                    rows = src.index_select(0, idx) if src is not None else \
                        _rsp_rows(st, idx)
                    if isinstance(oo, RowSparseNDArray):
                        odev = oo.context.torch_device
                        oo._vals, oo._aux, oo._shp = rows.to(odev), (idx.to(odev),), tuple(st.shape)
                        oo._dense, oo._stale = None, False
                    else:
                        res = torch.zeros_like(oo._data)
                        res.index_copy_(0, idx.to(res.device), rows.to(res.device, res.dtype))
                        oo._data.data.copy_(res)

    def set_gradient_compression(self, compression_params):
        if 'device' in self._type or 'dist' in self._type or self._type in ('local', 'nccl'):
            self._compression = GradientCompression(**compression_params)
        else:
            raise Exception('Gradient compression is not supported for this type of kvstore')

    def set_optimizer(self, optimizer):
        if isinstance(optimizer, string_types):
            optimizer = opt.create(optimizer)
        self._optimizer = optimizer
        self._updater = opt.get_updater(optimizer)

    def _set_updater(self, updater):
        self._updater = updater

    def save_optimizer_states(self, fname, dump_optimizer=False):
        assert self._updater is not None, 'Cannot save states for distributed training'
        with open(fname, 'wb') as fout:
            fout.write(self._updater.get_states(dump_optimizer))

    def load_optimizer_states(self, fname):
        assert self._updater is not None, 'Cannot load states for distributed training'
        with open(fname, 'rb') as f:
            self._updater.set_states(f.read())


def create(name='local'):
    """Create a KVStore: local, device, nccl, dist_sync, dist_device_sync, dist_async, horovod,
    or any registered KVStoreBase subclass (e.g. 'teststore')."""
    if not isinstance(name, string_types):
        raise TypeError('name must be a string')
    name = name.lower()
    if name in KVStoreBase.kv_registry:
        return KVStoreBase.kv_registry[name]()
    valid = ('local', 'device', 'nccl', 'dist_sync', 'dist_device_sync', 'dist_async', 'dist_sync_device',
             'dist', 'horovod', 'byteps', 'local_update_cpu', 'local_allreduce_cpu', 'local_allreduce_device',
             'dist_sync_allreduce')
    if name not in valid:
        raise MXNetError('Unknown KVStore type %s' % name)
    if name == 'dist_async':
        from .dist_async import KVStoreDistAsync
        return KVStoreDistAsync()
    return KVStore(name)


def _env_flag(name, default):
    import os
    v = os.environ.get(name)
    return default if v is None else v not in ('0', 'false', 'False', '')


def _rsp_rows(st, idx):
    """Rows ``idx`` of a row_sparse stored value (zeros for rows it does not hold)."""
    st._sync()
    have = st._aux[0]
    out = torch.zeros((idx.numel(),) + tuple(st.shape[1:]), dtype=st._vals.dtype, device=st._vals.device)
    hit = torch.isin(idx, have)
    if bool(hit.any()):
        out[hit] = st._vals.index_select(0, torch.searchsorted(have, idx[hit]))
    return out
