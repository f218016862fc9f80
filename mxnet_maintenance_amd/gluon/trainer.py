"""Gluon Trainer.

Parity: python/mxnet/gluon/trainer.py (Trainer: optimizer creation with
param_dict, kvstore selection/initialisation, update_on_kvstore, step,
allreduce_grads, update, stale-gradient checks, save_states/load_states,
learning_rate/set_learning_rate).

MI355X fast path ("flat arenas"): when every trainable parameter lives on one
GPU (one process per GPU), parameters of equal (dtype, lr_mult, wd_mult) are
re-homed into one contiguous HBM buffer, their gradients into a second one and
the optimizer state (momentum, fp32 master weights) into a third/fourth.  Then

* data-parallel gradient reduction is a handful of large RCCL all-reduces on
  slices of the gradient arena, launched from backward hooks as soon as a
  bucket is complete (parallel/buckets.py) — overlapped with backward;
* the optimizer step is ONE fused HIP kernel per arena (mp-SGD-momentum:
  fp16 grad -> fp32 master update -> fp16 weight write-back), a single pass over
  HBM instead of ~10 small kernels per parameter.

Per-parameter NDArray views keep the reference semantics (``param.grad()``,
``save_states``) unchanged.
"""
import os
import warnings

import numpy as np
import torch

from .. import engine as _engine
from .. import optimizer as opt
from ..base import MXNetError
from ..context import Context
from ..ndarray.ndarray import NDArray
from ..kvstore import kvstore as _kvs
from ..parallel import dist
from ..parallel.buckets import GradBuckets
from ..ops import kernels as _K
from .parameter import ParameterDict, Parameter
from ..utils import env as _env

__all__ = ['Trainer']


class _Arena:
    """Contiguous weight/grad/state storage for a group of same-dtype parameters."""

    def __init__(self, params, indices, lr_mult, wd_mult):
        self.params = params
        self.indices = indices
        self.lr_mult = lr_mult
        self.wd_mult = wd_mult
        d0 = params[0]._all_data()[0]._data
        self.dtype = d0.dtype
        self.device = d0.device
        align = 64   # every parameter starts on a 64-element (>=128 B) boundary
        offs = []
        off = 0
        for p in params:
            offs.append(off)
            off += (p._all_data()[0]._data.numel() + align - 1) // align * align
        self.numel = off
        self.w = torch.zeros(self.numel, dtype=self.dtype, device=self.device)
        self.g = torch.zeros(self.numel, dtype=self.dtype, device=self.device)
        self.views = []
        for p, off in zip(params, offs):
            arr = p._all_data()[0]
            t = arr._data
            n = t.numel()
            wv = self.w[off:off + n].view(t.shape)
            with torch.no_grad():
                wv.copy_(t)
            gv = self.g[off:off + n].view(t.shape)
            if arr._grad is not None:
                with torch.no_grad():
                    gv.copy_(arr._grad._data)
            arr._data = wv.detach()
            arr._set_grad_buffer(gv, p.grad_req)
            arr._arena = self
            self.views.append((off, n, t.shape))
        self.mom = None
        self.w32 = None
        self.mean = None     # Adam / AdamW / LAMB fp32 state
        self.var = None
        self.upd = None      # LAMB phase-1 direction (fp32)
        self.table = None    # LAMB chunk -> parameter segment table
        self.nrm = None
        self.all_write = all(p.grad_req == 'write' for p in params)


class Trainer:
    """Applies an Optimizer on a set of Parameters; handles gradient reduction."""

    def __init__(self, params, optimizer, optimizer_params=None, kvstore='device', compression_params=None,
                 update_on_kvstore=None):
        param_list = []
        if isinstance(params, (dict, ParameterDict)):
            for key in sorted(list(params.keys())):
                param_list.append(params[key])
            params = param_list
        if not isinstance(params, (list, tuple)):
            raise ValueError('First argument must be a list or dict of Parameters, got %s.' % (type(params)))
        self._params = []
        self._param2idx = {}
        for i, param in enumerate(params):
            if not isinstance(param, Parameter):
                raise ValueError('First argument must be a list or dict of Parameters, got list of %s.'
                                 % (type(param)))
            self._param2idx[param.name] = i
            self._params.append(param)
            param._set_trainer(self)
        self._compression_params = compression_params
        self._contexts = self._check_contexts()
        optimizer_params = optimizer_params if optimizer_params else {}
        self._init_optimizer(optimizer, optimizer_params)
        self._scale = self._optimizer.rescale_grad
        self._kvstore_params = {'kvstore': kvstore, 'update_on_kvstore': update_on_kvstore}
        self._kv_initialized = False
        self._kvstore = None
        self._update_on_kvstore = None
        self._distributed = None
        self._params_to_init = []
        self._arenas = None
        self._buckets = None
        self._hyper = None          # device hyper-parameters while a GraphStep is captured
        self._reset_kvstore()

    def _check_contexts(self):
        contexts = None
        for param in self._params:
            try:
                ctx = param.list_ctx()
            except RuntimeError:
                continue
            assert contexts is None or contexts == ctx, \
                'All Parameters must be initialized on the same set of contexts, but Parameter %s is initialized ' \
                'on %s while previous Parameters are initialized on %s.' % (param.name, str(ctx), str(contexts))
            contexts = ctx
        return contexts

    def _init_optimizer(self, optimizer, optimizer_params):
        param_dict = {i: param for i, param in enumerate(self._params)}
        if isinstance(optimizer, opt.Optimizer):
            assert not optimizer_params, 'optimizer_params must be None if optimizer is an instance of ' \
                                         'Optimizer instead of str'
            self._optimizer = optimizer
            self._optimizer.param_dict = param_dict
        else:
            self._optimizer = opt.create(optimizer, param_dict=param_dict, **optimizer_params)
        self._updaters = [opt.get_updater(self._optimizer) for _ in (self._contexts or [None])]
        for i, u in enumerate(self._updaters):
            u.device_slot = i

    def _init_params(self):
        assert self._kv_initialized, 'Cannot initialize parameters in KVStore when KVStore is not initialized.'
        params_to_init = []
        if self._kvstore:
            for param in self._params_to_init:
                if param._deferred_init:
                    params_to_init.append(param)
                else:
                    param_arrays = param._check_and_get(param._data, list)
                    idx = self._param2idx[param.name]
                    if param._stype != 'default':
                        self._kvstore.init(idx, param_arrays[0])
                    else:
                        self._kvstore.broadcast(idx, param_arrays[0], param_arrays)
        self._params_to_init = params_to_init

    def _reset_kvstore(self):
        if self._kvstore and 'dist' in self._kvstore.type:
            raise RuntimeError('Cannot reset distributed KVStore.')
        self._kv_initialized = False
        self._kvstore = None
        self._distributed = None
        self._update_on_kvstore = None
        self._params_to_init = [param for param in self._params]

    def _init_kvstore(self):
        config = self._kvstore_params
        kvstore = config['kvstore']
        update_on_kvstore = config['update_on_kvstore']
        self._contexts = self._check_contexts()
        multi_ctx = self._contexts is not None and len(self._contexts) > 1
        ranks = max(dist.world_size(), int(os.environ.get('WORLD_SIZE', '1')))
        sparse_weight = any(p._stype != 'default' for p in self._params)
        sparse_grad = any(getattr(p, '_grad_stype', 'default') != 'default' for p in self._params)
        if isinstance(kvstore, (_kvs.KVStoreBase,)):
            kv = kvstore
        elif kvstore is None or kvstore is False:
            if sparse_weight:
                # reference trainer.py _create_sparse_kvstore: sparse weights live on a kvstore
                raise TypeError('Cannot create a KVStore with row_sparse weights when kvstore=%s; '
                                'pass a kvstore type such as "local" or "device".' % (kvstore,))
            kv = None
        else:
            # reference: no kvstore for one device on one machine unless the weights are sparse
            need = multi_ctx or ('dist' in str(kvstore)) or ranks > 1 or sparse_weight
            kv = _kvs.create(kvstore) if need else None
        if kv is not None and self._compression_params:
            kv.set_gradient_compression(self._compression_params)
        self._distributed = kv is not None and ('dist' in kv.type or ranks > 1)
        if sparse_weight:
            # sparse weights live (and are updated) on the kvstore
            if update_on_kvstore is False:
                raise ValueError('Cannot set update_on_kvstore=False when sparse weights are present.')
            update_on_kvstore = True
        elif update_on_kvstore is None:
            if sparse_grad or ranks > 1:
                # dense weight + sparse grad: update locally; one process per GPU (RCCL): all-reduce the
                # gradients and run the fused local update on every rank (no parameter server round trip)
                update_on_kvstore = self._distributed and 'async' in getattr(kv, 'type', '')
            else:
                # in-process multi-device: MXNET_UPDATE_ON_KVSTORE (default 1) like the reference, when
                # the store can run the optimizer and (for 'local') no weight exceeds 16M elements
                update_on_kvstore = bool(int(os.environ.get('MXNET_UPDATE_ON_KVSTORE', '1'))) and \
                    kv is not None and kv.is_capable(_kvs.KVStoreBase.OPTIMIZER)
                if update_on_kvstore and kvstore == 'local' and \
                        max(int(np.prod(p.shape)) for p in self._params) > 1024 * 1024 * 16:
                    update_on_kvstore = False
        if kv is not None and update_on_kvstore and not kv.is_capable(_kvs.KVStoreBase.OPTIMIZER):
            raise ValueError('Please set update_on_kvstore=False when training with {}'.format(type(kv)))
        if kv is None:
            self._kvstore = None
            self._update_on_kvstore = None
        else:
            self._kvstore = kv
            self._update_on_kvstore = bool(update_on_kvstore)
            if self._update_on_kvstore:
                kv.set_optimizer(self._optimizer)
        self._kv_initialized = True

    # ------------------------------------------------------------ fast path
    def _arena_eligible(self):
        if _env.get('MXAMD_FLAT_ARENA') != 1:
            return False
        if self._update_on_kvstore or not self._contexts or len(self._contexts) != 1:
            return False
        if type(self._optimizer) not in (opt.SGD, opt.ccSGD, opt.Adam, opt.AdamW, opt.LAMB):
            return False
        if self._kvstore is not None and not isinstance(self._kvstore, _kvs.KVStore):
            return False
        if self._kvstore is not None and self._kvstore._compression is not None:
            return False
        for p in self._params:
            if p._data is None or p._stype != 'default' or getattr(p, '_grad_stype', 'default') != 'default':
                return False
        return True

    def _build_arenas(self):
        groups = {}
        order = []
        for i, p in enumerate(self._params):
            if p.grad_req == 'null':
                continue
            key = (p._all_data()[0]._data.dtype, float(p.lr_mult), float(p.wd_mult))
            if key not in groups:
                groups[key] = ([], [])
                order.append(key)
            groups[key][0].append(p)
            groups[key][1].append(i)
        self._arenas = [_Arena(groups[k][0], groups[k][1], k[1], k[2]) for k in order]
        o = self._optimizer
        mp = o.multi_precision
        upd = self._updaters[0]
        kind = 'sgd' if isinstance(o, opt.SGD) else type(o).__name__.lower()
        for a in self._arenas:
            half = a.dtype in (torch.float16, torch.bfloat16)
            if mp and half:
                a.w32 = a.w.float()
            if kind == 'sgd':
                if o.momentum != 0.0:
                    a.mom = torch.zeros(a.numel, dtype=torch.float32, device=a.device)
            else:
                a.mean = torch.zeros(a.numel, dtype=torch.float32, device=a.device)
                a.var = torch.zeros(a.numel, dtype=torch.float32, device=a.device)
                if kind == 'lamb':
                    from ..ops.nlp_fns import ChunkTable
                    a.upd = torch.empty(a.numel, dtype=torch.float32, device=a.device)
                    a.table = ChunkTable([(off, n) for (off, n, _shape) in a.views], a.device)
                    a.nrm = torch.zeros(2 * (len(a.views) + a.table.n), dtype=torch.float32, device=a.device)
            for p, (off, n, shape), idx in zip(a.params, a.views, a.indices):
                w32v = NDArray(a.w32[off:off + n].view(shape)) if a.w32 is not None else None
                if w32v is not None:
                    # fp32 master visible to kernels that want fp32 parameters (LayerNorm/BN gamma, beta):
                    # valid while the half tensor is only written by the fused update (whose raw-pointer
                    # writes keep its version counter); any torch in-place write invalidates it
                    t = p._all_data()[0]._data
                    t._mxamd_master = (w32v._data, t._version)
                if kind == 'sgd':
                    mom = NDArray(a.mom[off:off + n].view(shape)) if a.mom is not None else None
                    st = (mom, w32v) if w32v is not None else mom
                else:
                    mv = (NDArray(a.mean[off:off + n].view(shape)), NDArray(a.var[off:off + n].view(shape)))
                    if w32v is None:
                        st = mv
                    elif kind in ('adam', 'lamb'):
                        st = (w32v, mv)       # Optimizer.create_state_multi_precision layout
                    else:
                        st = (w32v,) + mv     # AdamW layout
                upd.states[idx] = st
                upd.states_synced[idx] = True
        self._arena_kind = kind
        if self._kvstore is not None and dist.world_size() > 1:
            arrays = []
            reqs = []
            for a in self._arenas:
                for p in a.params:
                    arrays.append(p._all_data()[0])
                    reqs.append(p.grad_req)
            self._buckets = _ArenaBuckets(self._arenas)

    def _on_param_grad_reset(self, param):
        if self._arenas is not None:
            warnings.warn('Parameter %s was re-initialised after the Trainer built its flat arenas; '
                          'falling back to per-parameter updates.' % param.name)
            self._arenas = None
            if self._buckets is not None:
                self._buckets.remove()
                self._buckets = None

    # ------------------------------------------------------------- public API
    @property
    def learning_rate(self):
        if not isinstance(self._optimizer, opt.Optimizer):
            raise UserWarning('Optimizer has to be defined before its learning rate can be accessed.')
        return self._optimizer.learning_rate

    @property
    def optimizer(self):
        if isinstance(self._optimizer, opt.Optimizer):
            return self._optimizer
        raise UserWarning('Optimizer has not been initialized yet')

    def set_learning_rate(self, lr):
        if not isinstance(self._optimizer, opt.Optimizer):
            raise UserWarning('Optimizer has to be defined before its learning rate is mutated.')
        self._optimizer.set_learning_rate(lr)

    def _row_sparse_pull(self, parameter, out, row_id, full_idx=False):
        if not self._kv_initialized:
            self._init_kvstore()
        if self._params_to_init:
            self._init_params()
        idx = self._param2idx[parameter.name]
        if self._kvstore is not None:
            self._kvstore.row_sparse_pull(idx, out=out, row_ids=row_id, priority=-idx)

    def _check_and_rescale_grad(self, scale):
        if self._update_on_kvstore and self._distributed and self._kv_initialized:
            if self._optimizer.rescale_grad != scale:
                raise UserWarning('Possible change in the `batch_size` from previous `step` detected. Optimizer '
                                  'gradient normalizing factor will not change w.r.t new batch_size when '
                                  'update_on_kvstore=True and when distributed kvstore is used.')
        self._optimizer.rescale_grad = scale

    def _prepare(self):
        if not self._kv_initialized:
            self._init_kvstore()
        if self._params_to_init:
            self._init_params()
        if self._arenas is None and self._arena_eligible():
            self._build_arenas()

    def step(self, batch_size, ignore_stale_grad=False):
        """One optimisation step: reduce gradients, then update with lr * (grad / batch_size)."""
        _engine.join_workers()   # worker-stream operators (engine.op_stream) done first
        rescale_grad = self._scale / batch_size
        self._check_and_rescale_grad(rescale_grad)
        self._prepare()
        self._allreduce_grads()
        if self._amp_overflow():
            return
        self._update(ignore_stale_grad)

    def _amp_overflow(self):
        """AMP dynamic loss scaling: skip the update when any gradient is non-finite."""
        scaler = getattr(self, '_amp_loss_scaler', None)
        if scaler is None:
            return False
        if scaler.has_overflow(self._params, self._arenas):
            for p in self._params:
                for d in (p._data or []):
                    d._fresh_grad = False
            return True
        return False

    def allreduce_grads(self):
        _engine.join_workers()
        self._prepare()
        assert not (self._kvstore and self._update_on_kvstore), \
            'allreduce_grads() when parameters are updated on kvstore is not supported. Try setting ' \
            '`update_on_kvstore` to False when creating trainer.'
        self._allreduce_grads()

    def _allreduce_grads(self):
        if self._kvstore is None:
            return
        if self._arenas is not None:
            if self._buckets is not None:
                self._buckets.reduce()
            return
        keys, vals = [], []
        for i, param in enumerate(self._params):
            if param.grad_req != 'null':
                keys.append(i)
                vals.append(param.list_grad())
        if not keys:
            return
        if not isinstance(self._kvstore, _kvs.KVStore):
            # a user-registered KVStoreBase: one key per call, like the reference trainer
            for k, v in zip(keys, vals):
                if self._update_on_kvstore:
                    self._kvstore.pushpull(k, v, out=self._params[k]._all_data(), priority=-k)
                else:
                    self._kvstore.pushpull(k, v, priority=-k)
            return
        if self._update_on_kvstore:
            self._kvstore.pushpull(keys, vals, [p._all_data() for p in self._params if p.grad_req != 'null'])
        else:
            self._kvstore.pushpull(keys, vals, vals)

    def update(self, batch_size, ignore_stale_grad=False):
        _engine.join_workers()
        self._prepare()
        assert not (self._kvstore and self._update_on_kvstore), \
            'update() when parameters are updated on kvstore is not supported. Try setting `update_on_kvstore` ' \
            'to False when creating trainer.'
        self._check_and_rescale_grad(self._scale / batch_size)
        if self._amp_overflow():
            return
        self._update(ignore_stale_grad)

    def _check_stale(self, ignore_stale_grad):
        for i, param in enumerate(self._params):
            if param.grad_req == 'null':
                continue
            if not ignore_stale_grad:
                for data in param._check_and_get(param._data, list):
                    if not data._fresh_grad:
                        raise UserWarning(
                            'Gradient of Parameter `%s` on context %s has not been updated by backward since last '
                            '`step`. This could mean a bug in your model that made it only use a subset of the '
                            'Parameters (Blocks) for this iteration. If you are intentionally only using a subset, '
                            'call step with ignore_stale_grad=True to suppress this warning and skip updating of '
                            'Parameters with stale gradient' % (param.name, str(data.context)))

    def _update(self, ignore_stale_grad=False):
        if self._arenas is not None:
            self._check_stale(ignore_stale_grad)
            self._fused_update(ignore_stale_grad)
            for p in self._params:
                if p._data is not None:
                    for d in p._data:
                        d._fresh_grad = False
            return
        updates = [[] for _ in self._updaters]
        for i, param in enumerate(self._params):
            if param.grad_req == 'null':
                continue
            if not ignore_stale_grad:
                for data in param._check_and_get(param._data, list):
                    if not data._fresh_grad:
                        raise UserWarning(
                            'Gradient of Parameter `%s` on context %s has not been updated by backward since last '
                            '`step`. This could mean a bug in your model that made it only use a subset of the '
                            'Parameters (Blocks) for this iteration. If you are intentionally only using a subset, '
                            'call step with ignore_stale_grad=True to suppress this warning and skip updating of '
                            'Parameters with stale gradient' % (param.name, str(data.context)))
            if self._kvstore and self._update_on_kvstore:
                continue
            for upd, arr, grad in zip(updates, param._all_data(), param.list_grad()):
                if not ignore_stale_grad or arr._fresh_grad:
                    upd.append((i, grad, arr))
                    arr._fresh_grad = False
        if not (self._kvstore and self._update_on_kvstore):
            for updater, upd in zip(self._updaters, updates):
                if upd:
                    i, g, w = zip(*upd)
                    updater(list(i), list(g), list(w))
        else:
            for param in self._params:
                for d in (param._data or []):
                    d._fresh_grad = False

    def _arena_hparams(self, a, advance=True):
        """(lr, wd, t, bc1, bc2) for arena ``a``; advances the update count unless ``advance`` is False.

        ``lr`` is the value the kernel consumes: for Adam it already carries the
        bias correction ``sqrt(1 - beta2^t) / (1 - beta1^t)``.
        """
        import math
        o = self._optimizer
        if advance:
            o._update_count(a.indices)
        lr = o._get_lrs(a.indices[:1])[0]
        wd = o._get_wds(a.indices[:1])[0]
        t = o._index_update_count.get(a.indices[0], 1) or 1
        kind = getattr(self, '_arena_kind', 'sgd')
        bc1 = bc2 = 1.0
        if kind in ('adam', 'adamw') and (kind == 'adam' or o.correct_bias):
            lr *= math.sqrt(1. - o.beta2 ** t) / (1. - o.beta1 ** t)
        elif kind == 'lamb' and o.bias_correction:
            bc1, bc2 = 1.0 - o.beta1 ** t, 1.0 - o.beta2 ** t
        return lr, wd, t, bc1, bc2

    def _fused_update(self, ignore_stale_grad=False):
        o = self._optimizer
        clip = -1.0 if o.clip_gradient is None else o.clip_gradient
        kind = getattr(self, '_arena_kind', 'sgd')
        graph = self._hyper is not None
        for i, a in enumerate(self._arenas):
            saved = self._save_stale(a) if ignore_stale_grad else None
            if not graph and not saved and kind != 'sgd':
                # an earlier stale step left the arena's parameters at different update counts
                cnt = o._index_update_count
                c0 = cnt.get(a.indices[0], 0)
                if any(cnt.get(j, 0) != c0 for j in a.indices):
                    saved = [None]
            if saved and not graph:
                # some parameters have no fresh gradient: the reference neither updates them nor
                # advances their update counts, so Adam/LAMB bias corrections (per-parameter t) stay
                # exact only if each fresh parameter is updated with its own count
                self._restore_stale([x for x in saved if x is not None])
                self._stale_arena_update(a, kind, clip)
                continue
            # graph mode: counts advance (and lr / bias corrections reach the device) in _stage_hyper,
            # before every replay; the kernels read them from self._hyper[i]
            lr, wd, t, _bc1, _bc2 = self._arena_hparams(a, advance=not graph)
            hp = self._hyper[i] if graph else None
            if kind == 'sgd':
                flat_sgd_update(a.w, a.g, a.mom, a.w32, lr, wd, o.momentum, o.rescale_grad, clip, hp=hp)
            elif kind in ('adam', 'adamw'):
                flat_adam_update(a, lr, o.beta1, o.beta2, o.epsilon, wd, o.rescale_grad, clip, kind == 'adamw',
                                 hp=hp)
            else:
                lamb_flat_update(a, lr, o, t, wd, clip, hp=hp)
            if saved:
                self._restore_stale(saved)

    def _stale_arena_update(self, a, kind, clip):
        """Update only the arena's parameters with a fresh gradient, each as its own segment with its
        own update count (torch math on the slices; the fused kernels assume one count per arena)."""
        import math
        o = self._optimizer
        for idx, p, (off, n, shape) in zip(a.indices, a.params, a.views):
            if not p._all_data()[0]._fresh_grad:
                continue
            o._update_count([idx])
            lr = o._get_lrs([idx])[0]
            wd = o._get_wds([idx])[0]
            t = o._index_update_count.get(idx, 1) or 1
            sl = _ArenaSlice(a, off, n, shape)
            if kind == 'sgd':
                flat_sgd_update(sl.w, sl.g, sl.mom, sl.w32, lr, wd, o.momentum, o.rescale_grad, clip,
                                torch_only=True)
            elif kind in ('adam', 'adamw'):
                if kind == 'adam' or o.correct_bias:
                    lr *= math.sqrt(1. - o.beta2 ** t) / (1. - o.beta1 ** t)
                flat_adam_update(sl, lr, o.beta1, o.beta2, o.epsilon, wd, o.rescale_grad, clip, kind == 'adamw',
                                 torch_only=True)
            else:
                lamb_flat_update(sl, lr, o, t, wd, clip, torch_only=True)

    # ------------------------------------------------------------------ HIP-graph capture support
    def _enter_graph_mode(self):
        """Switch the fused update to device-resident hyper-parameters (see gluon.GraphStep).

        Requirements: flat arenas on a HIP device, no AMP dynamic loss scaling
        (its overflow check reads the device), no update on kvstore.
        """
        self._prepare()
        if self._arenas is None or not self._arenas[0].w.is_cuda:
            raise RuntimeError('graph capture needs the fused flat-arena update on a HIP device')
        if getattr(self, '_amp_loss_scaler', None) is not None:
            raise RuntimeError('graph capture does not support AMP dynamic loss scaling')
        if self._update_on_kvstore and self._kvstore is not None:
            raise RuntimeError('graph capture does not support update_on_kvstore')
        dev = self._arenas[0].w.device
        self._hyper = torch.zeros((len(self._arenas), 4), dtype=torch.float32, device=dev)
        self._hyper_host = torch.zeros((len(self._arenas), 4), dtype=torch.float32)

    def _exit_graph_mode(self):
        self._hyper = None
        self._hyper_host = None

    def _stage_hyper(self, batch_size=None):
        """Advance update counts and upload this step's lr / bias corrections (before a graph replay)."""
        if batch_size is not None and self._scale / batch_size != self._optimizer.rescale_grad:
            raise RuntimeError('graph-captured step: rescale_grad is baked into the graph; batch_size changed')
        for i, a in enumerate(self._arenas):
            lr, _wd, _t, bc1, bc2 = self._arena_hparams(a, advance=True)
            self._hyper_host[i, 0] = lr
            self._hyper_host[i, 1] = bc1
            self._hyper_host[i, 2] = bc2
        self._hyper.copy_(self._hyper_host)

    @staticmethod
    @torch.no_grad()
    def _save_stale(a):
        """Copies of the weight/state slices of ``a``'s parameters without a fresh gradient.

        The fused kernels update a whole arena; with ``ignore_stale_grad`` the
        reference leaves stale parameters (and their optimizer state) untouched,
        so their slices are snapshotted here and written back after the update.
        """
        saved = []
        for p, (off, n, _shape) in zip(a.params, a.views):
            if p._all_data()[0]._fresh_grad:
                continue
            for buf in (a.w, a.w32, a.mom, a.mean, a.var):
                if buf is not None:
                    saved.append((buf, off, buf[off:off + n].clone()))
        return saved

    @staticmethod
    @torch.no_grad()
    def _restore_stale(saved):
        for buf, off, val in saved:
            buf[off:off + val.numel()].copy_(val)

    def save_states(self, fname):
        assert self._optimizer is not None
        if not self._kv_initialized:
            self._init_kvstore()
        if self._params_to_init:
            self._init_params()
        if self._update_on_kvstore:
            assert not self._params_to_init, 'Cannot save trainer states when some parameters are not yet ' \
                                             'initialized in kvstore.'
            self._kvstore.save_optimizer_states(fname, dump_optimizer=True)
        else:
            with open(fname, 'wb') as fout:
                fout.write(self._updaters[0].get_states(dump_optimizer=True))

    def load_states(self, fname):
        if not self._kv_initialized:
            self._init_kvstore()
        if self._params_to_init:
            self._init_params()
        if self._update_on_kvstore:
            self._kvstore.load_optimizer_states(fname)
            self._optimizer = self._kvstore._updater.optimizer
        else:
            with open(fname, 'rb') as f:
                states = f.read()
            for updater in self._updaters:
                updater.set_states(states)
                updater.optimizer = self._updaters[0].optimizer
            self._optimizer = self._updaters[0].optimizer
            if self._arenas is not None:
                upd = self._updaters[0]
                for a in self._arenas:
                    kind = getattr(self, '_arena_kind', 'sgd')
                    for (off, n, shape), idx in zip(a.views, a.indices):
                        st = upd.states[idx]

                        def cp(dst, src):
                            dst[off:off + n].copy_(src._data.reshape(-1).to(dst.device, dst.dtype))
                        with torch.no_grad():
                            if kind == 'sgd':
                                if a.w32 is not None:
                                    mom, w32 = st
                                    cp(a.w32, w32)
                                else:
                                    mom = st
                                if a.mom is not None and mom is not None:
                                    cp(a.mom, mom)
                            else:
                                if a.w32 is None:
                                    mean, var = st
                                elif kind in ('adam', 'lamb'):
                                    w32, (mean, var) = st
                                    cp(a.w32, w32)
                                else:
                                    w32, mean, var = st
                                    cp(a.w32, w32)
                                cp(a.mean, mean)
                                cp(a.var, var)
                        # rebind state views to the arena
                        w32v = NDArray(a.w32[off:off + n].view(shape)) if a.w32 is not None else None
                        if kind == 'sgd':
                            momv = NDArray(a.mom[off:off + n].view(shape)) if a.mom is not None else None
                            upd.states[idx] = (momv, w32v) if w32v is not None else momv
                        else:
                            mv = (NDArray(a.mean[off:off + n].view(shape)), NDArray(a.var[off:off + n].view(shape)))
                            upd.states[idx] = mv if w32v is None else ((w32v, mv) if kind in ('adam', 'lamb')
                                                                       else (w32v,) + mv)
        param_dict = {i: param for i, param in enumerate(self._params)}
        self._optimizer.param_dict = param_dict


class _ArenaBuckets(GradBuckets):
    """GradBuckets whose buckets are contiguous slices of the trainer's gradient arenas."""

    def __init__(self, arenas, bucket_bytes=None, tail_bytes=None):
        from ..parallel.buckets import _Bucket
        if bucket_bytes is None:
            from ..parallel.buckets import bucket_bytes_for
            bucket_bytes = bucket_bytes_for(sum(a.g.numel() * a.g.element_size() for a in arenas))
        if tail_bytes is None:
            tail_bytes = int(_env.get('MXAMD_TAIL_BUCKET_MB') * (1 << 20))
        tail_bytes = max(1, min(tail_bytes, bucket_bytes))
        self.overlap = dist.world_size() > 1
        self.average = False
        self.buckets = []
        self._hooks = []
        for a in arenas:
            esz = a.g.element_size()
            # walk parameters from the end of the arena (first to receive grads in backward)
            cur = None
            cur_lo = None
            segs = list(zip(a.params, a.views))[::-1]
            for p, (off, n, shape) in segs:
                # the first layers' gradients (produced last, reduced after backward ends) go into small
                # tail buckets so the un-overlapped final all-reduce stays short
                cap = tail_bytes if (off + n) * esz <= 2 * tail_bytes else bucket_bytes
                if cur is None or (cur_hi - off) * esz > cap:
                    if cur is not None:
                        cur.flat = a.g[cur_lo:cur_hi]
                    cur = _Bucket(a.g.dtype, a.g.device)
                    self.buckets.append(cur)
                    cur_hi = off + n
                cur_lo = off
                cur.params.append(p._all_data()[0])
                cur.count += 1
            if cur is not None:
                cur.flat = a.g[cur_lo:cur_hi]
        if self.overlap:
            for b in self.buckets:
                if any(p._grad_req == 'add' for p in b.params):
                    continue
                for p in b.params:
                    self._hooks.append(p._data.register_post_accumulate_grad_hook(self._make_hook(b)))


class _ArenaSlice:
    """One parameter's segment of a flat arena, shaped like an arena for the torch update paths."""

    def __init__(self, a, off, n, shape):
        def cut(b):
            return None if b is None else b[off:off + n]
        self.w, self.g, self.w32 = cut(a.w), cut(a.g), cut(a.w32)
        self.mom = cut(getattr(a, 'mom', None))
        self.mean, self.var = cut(getattr(a, 'mean', None)), cut(getattr(a, 'var', None))
        self.views = [(0, n, shape)]


@torch.no_grad()
def flat_sgd_update(w, g, mom, w32, lr, wd, momentum, rescale, clip, hp=None, torch_only=False):
    """SGD(-momentum) over flat buffers; fused HIP kernel on gfx950 (``hp``: device lr, graph mode)."""
    if not torch_only and w.is_cuda and _K.available() and _K.enabled() and hasattr(_K, 'flat_sgd'):
        _K.flat_sgd(w, g, mom, w32, lr, wd, momentum, rescale, clip, hp=hp)
        return
    if hp is not None:
        raise RuntimeError('graph-captured updates need the HIP optimizer kernels')
    tgt = w32 if w32 is not None else w
    gg = g.to(tgt.dtype) if g.dtype != tgt.dtype else g.clone()
    if rescale != 1.0:
        gg.mul_(rescale)
    if clip is not None and clip >= 0:
        gg.clamp_(-clip, clip)
    if wd != 0.0:
        gg.add_(tgt, alpha=wd)
    if momentum != 0.0 and mom is not None:
        mom.mul_(momentum).add_(gg, alpha=-lr)
        tgt.add_(mom)
    else:
        tgt.add_(gg, alpha=-lr)
    if w32 is not None:
        w.copy_(w32)


@torch.no_grad()
def flat_adam_update(a, lr, beta1, beta2, eps, wd, rescale, clip, adamw, hp=None, torch_only=False):
    """Adam / AdamW over one arena: fused HIP kernel on gfx950, torch ops elsewhere (same math)."""
    if not torch_only and a.w.is_cuda and _K.available() and _K.enabled() and hasattr(_K, 'flat_adam'):
        _K.flat_adam(a.w, a.g, a.mean, a.var, a.w32, lr, beta1, beta2, eps, wd, rescale, clip, adamw=adamw, hp=hp)
        return
    if hp is not None:
        raise RuntimeError('graph-captured updates need the HIP optimizer kernels')
    w = a.w32 if a.w32 is not None else a.w
    g = a.g.float() * rescale
    if not adamw and wd:
        g = g + wd * w.float()
    if clip is not None and clip >= 0:
        g = g.clamp(-clip, clip)
    a.mean.mul_(beta1).add_(g, alpha=1 - beta1)
    a.var.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    step = lr * a.mean / (a.var.sqrt() + eps)
    if adamw:
        step = step + wd * w.float()
    w.sub_(step.to(w.dtype))
    if a.w32 is not None:
        a.w.copy_(a.w32)


@torch.no_grad()
def lamb_flat_update(a, lr, o, t, wd, clip, hp=None, torch_only=False):
    """LAMB (phase 1 + per-parameter trust ratio + phase 2) over one arena."""
    lb = -1.0 if o.lower_bound is None else o.lower_bound
    ub = -1.0 if o.upper_bound is None else o.upper_bound
    if not torch_only and a.w.is_cuda and _K.available() and _K.enabled() and hasattr(_K, 'lamb_update'):
        _K.lamb_update(a.w, a.g, a.mean, a.var, a.w32, a.upd, a.table, a.nrm, lr, o.beta1, o.beta2, o.epsilon, t,
                       o.bias_correction, wd, o.rescale_grad, clip, lb, ub, hp=hp)
        return
    if hp is not None:
        raise RuntimeError('graph-captured updates need the HIP optimizer kernels')
    from ..ops import optimizer_ops as _oo
    for off, n, _shape in a.views:
        w = a.w[off:off + n]
        w32 = a.w32[off:off + n] if a.w32 is not None else None
        tgt = w32 if w32 is not None else w
        g = _oo._lamb1(tgt, a.g[off:off + n].float(), a.mean[off:off + n], a.var[off:off + n], o.beta1, o.beta2,
                       o.epsilon, t, o.bias_correction, wd, o.rescale_grad, clip)
        r1 = torch.linalg.vector_norm(tgt.float()).reshape(1)
        r2 = torch.linalg.vector_norm(g).reshape(1)
        _oo._lamb2(w, g, r1, r2, lr, lb, ub, w32=w32)
