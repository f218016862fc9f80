"""Optimizers.

Parity: python/mxnet/optimizer/optimizer.py (Optimizer registry/create,
lr/wd multipliers, update counts, multi-precision master weights, Updater,
get_updater; SGD, Signum, FTML, LARS, LBSGD, LAMB, DCASGD, NAG, SGLD, ccSGD,
Adam, AdaGrad, RMSProp, AdaDelta, Ftrl, Adamax, Nadam, Test) and
python/mxnet/optimizer/contrib.py (GroupAdaGrad), plus AdamW
(src/operator/contrib/adamw*).

Updates run in place on the parameter tensors.  ``SGD`` and ``Adam`` accept
lists of indices (``aggregate_num``) and then run as one multi-tensor update:
the fused gfx950 HIP kernel when available, ``torch._foreach_*`` otherwise.
"""
import math
import pickle
import warnings

import numpy as np
import torch

from ..base import MXNetError, torch_dtype
from ..ndarray.ndarray import NDArray
from .. import ndarray as nd
from ..ops import optimizer_ops as _oo
from ..ops import kernels as _K

__all__ = ['Optimizer', 'register', 'create', 'SGD', 'Signum', 'FTML', 'LARS', 'LBSGD', 'LAMB', 'DCASGD', 'NAG',
           'SGLD', 'ccSGD', 'Adam', 'AdamW', 'AdaGrad', 'RMSProp', 'AdaDelta', 'Ftrl', 'Adamax', 'Nadam', 'Test',
           'Updater', 'get_updater', 'GroupAdaGrad']


def _t(x):
    return x._data if isinstance(x, NDArray) else x


class _UpdateCounts:
    """Per-device, per-parameter update counters (the reference counts updates separately on every
    device of a multi-device Module).  ``current`` is the table of the active device."""

    def __init__(self, begin):
        self.begin = begin
        self.tables = {0: {}}
        self.current = self.tables[0]

    def select(self, device_id):
        self.current = self.tables.setdefault(device_id, {})

    def bump(self, indices):
        """Advance the counters of ``indices``; returns the largest resulting count."""
        top = 0
        for idx in indices:
            n = self.current.get(idx, self.begin) + 1
            self.current[idx] = n
            top = max(top, n)
        return top


def _symbol_attr_mults(sym_info, key):
    """``{argument name: float}`` from the ``__lr_mult__`` / ``__wd_mult__`` attributes of a Symbol."""
    if not sym_info:
        return {}
    attrs, names = sym_info
    return {n: float(attrs[n][key]) for n in names if key in attrs.get(n, {})}


class Optimizer:
    """Base class of all optimizers.

    Hyper-parameters are resolved per parameter index: the learning rate comes from the scheduler
    (at the current update count) or ``lr``, the weight decay from ``wd``; both are scaled by a
    multiplier looked up first on the Gluon Parameter (``param_dict``), then by index, then by the
    parameter's name (``idx2name``) in ``lr_mult`` / ``wd_mult``.  By default only ``*_weight`` and
    ``*_gamma`` parameters are decayed.  Subclasses implement ``create_state`` and ``update``.
    """
    opt_registry = {}

    def __init__(self, rescale_grad=1., param_idx2name=None, wd=0., clip_gradient=None, learning_rate=None,
                 lr_scheduler=None, sym=None, begin_num_update=0, multi_precision=False, param_dict=None,
                 aggregate_num=None, use_fused_step=None, **kwargs):
        if param_idx2name is not None and not isinstance(param_idx2name, dict):
            raise AssertionError('param_idx2name should be a dict of param indexes to names.')
        self.rescale_grad = rescale_grad
        self.wd = wd
        self.clip_gradient = clip_gradient
        self.multi_precision = multi_precision
        self.aggregate_num = aggregate_num or 0
        self.allow_np_array = False
        self.lr_scheduler = lr_scheduler
        self.lr = self._initial_lr(learning_rate, lr_scheduler)
        self.begin_num_update = begin_num_update
        self.num_update = begin_num_update
        self._counts = _UpdateCounts(begin_num_update)
        self.idx2name = dict(param_idx2name or {})
        self.sym_info = (sym.attr_dict(), sym.list_arguments()) if sym is not None else ()
        self.param_dict = param_dict or {}
        self.lr_mult, self.wd_mult = {}, {}
        self.set_lr_mult({})
        self.set_wd_mult({})

    @staticmethod
    def _initial_lr(learning_rate, scheduler):
        if scheduler is None:
            return 0.01 if learning_rate is None else learning_rate
        if learning_rate is not None:
            # an explicit learning_rate overrides the scheduler's base_lr
            if scheduler.base_lr != learning_rate:
                warnings.warn('learning rate from ``lr_scheduler`` has been overwritten by ``learning_rate`` '
                              'in optimizer.', UserWarning)
            scheduler.base_lr = learning_rate
        return scheduler.base_lr

    # ------------------------------------------------------------------ registry
    @staticmethod
    def register(klass):
        """Class decorator: make ``klass`` creatable by its lower-cased name."""
        if not isinstance(klass, type):
            raise AssertionError('register expects a class')
        key = klass.__name__.lower()
        old = Optimizer.opt_registry.get(key)
        if old is not None:
            warnings.warn('WARNING: New optimizer %s.%s is overriding existing optimizer %s.%s'
                          % (klass.__module__, klass.__name__, old.__module__, old.__name__))
        Optimizer.opt_registry[key] = klass
        return klass

    @staticmethod
    def create_optimizer(name, **kwargs):
        """Instantiate a registered optimizer by (case-insensitive) name."""
        klass = Optimizer.opt_registry.get(name.lower())
        if klass is None:
            raise ValueError('Cannot find optimizer %s' % name)
        return klass(**kwargs)

    # ------------------------------------------------------------------ update-count bookkeeping
    @property
    def _index_update_count(self):
        return self._counts.current

    @property
    def _all_index_update_counts(self):
        return self._counts.tables

    def _set_current_context(self, device_id):
        self._counts.select(device_id)

    def _update_count(self, index):
        top = self._counts.bump(index if isinstance(index, (list, tuple)) else [index])
        self.num_update = max(self.num_update, top)

    # ------------------------------------------------------------------ learning rate / weight decay
    @property
    def learning_rate(self):
        return self.lr if self.lr_scheduler is None else self.lr_scheduler(self.num_update)

    def set_learning_rate(self, lr):
        if self.lr_scheduler is not None:
            raise UserWarning('LRScheduler of the optimizer has already been defined. Note that '
                              'set_learning_rate can mutate the value of the learning rate of the optimizer only '
                              'when the LRScheduler of the optimizer is undefined.')
        self.lr = lr

    def set_lr_scale(self, args_lrscale):
        raise DeprecationWarning

    def set_lr_mult(self, args_lr_mult):
        """Learning-rate multipliers by name or index (Symbol ``__lr_mult__`` attributes come first)."""
        self.lr_mult = _symbol_attr_mults(self.sym_info, '__lr_mult__')
        self.lr_mult.update(args_lr_mult)

    def set_wd_mult(self, args_wd_mult):
        """Weight-decay multipliers; parameters not named ``*_weight`` / ``*_gamma`` default to 0."""
        self.wd_mult = {n: 0.0 for n in self.idx2name.values() if not n.endswith(('_weight', '_gamma'))}
        self.wd_mult.update(_symbol_attr_mults(self.sym_info, '__wd_mult__'))
        self.wd_mult.update(args_wd_mult)

    def _mult(self, index, table, attr):
        p = self.param_dict.get(index)
        if p is not None:
            return getattr(p, attr)
        if index in table:
            return table[index]
        name = self.idx2name.get(index)
        return table.get(name, 1.0) if name is not None else 1.0

    def _get_lrs(self, indices):
        base = self.learning_rate
        return [base * self._mult(i, self.lr_mult, 'lr_mult') for i in indices]

    def _get_lr(self, index):
        return self._get_lrs([index])[0]

    def _get_wds(self, indices):
        return [self.wd * self._mult(i, self.wd_mult, 'wd_mult') for i in indices]

    def _get_wd(self, index):
        return self._get_wds([index])[0]

    def _clip(self):
        return -1.0 if self.clip_gradient is None else self.clip_gradient

    # ------------------------------------------------------------------ states and updates
    def create_state(self, index, weight):
        return None

    def _wants_master(self, weight):
        return self.multi_precision and weight._data.dtype in (torch.float16, torch.bfloat16)

    def create_state_multi_precision(self, index, weight):
        """With ``multi_precision`` and a half-precision weight: ``(fp32 master copy, state of the
        master)``; otherwise the plain state."""
        if self._wants_master(weight):
            master = NDArray(weight._data.detach().float().clone())
            return (master, self.create_state(index, master))
        if weight._data.dtype in (torch.float16, torch.bfloat16):
            warnings.warn('Accumulating with float16 in optimizer can lead to poor accuracy or slow convergence. '
                          'Consider using multi_precision=True option of the optimizer')
        return self.create_state(index, weight)

    def update(self, index, weight, grad, state):
        raise NotImplementedError()

    def update_multi_precision(self, index, weight, grad, state):
        """``update`` on the fp32 master copy (then rounded into the weight) for half-precision weights
        under ``multi_precision``; lists of indices are updated one by one."""
        if isinstance(index, (list, tuple)):
            for args in zip(index, weight, grad, state):
                self.update_multi_precision(*args)
            return
        if not self._wants_master(weight):
            self.update(index, weight, grad, state)
            return
        master, inner = state
        # sparse gradients keep their storage (lazy row updates need the row indices)
        g32 = grad.astype('float32') if getattr(grad, 'stype', 'default') != 'default' else NDArray(grad._data.float())
        self.update(index, master, g32, inner)
        with torch.no_grad():
            weight._data.copy_(master._data)

    def __getstate__(self):
        state = dict(self.__dict__)
        state.pop('param_dict', None)      # Gluon Parameters do not travel with a pickled optimizer
        return state

    def __setstate__(self, state):
        if '_counts' not in state:        # optimizer states pickled by an older version of this class
            counts = _UpdateCounts(state.get('begin_num_update', 0))
            counts.tables = state.pop('_all_index_update_counts', {0: {}})
            counts.current = state.pop('_index_update_count', counts.tables.setdefault(0, {}))
            state['_counts'] = counts
        self.__dict__ = state
        self.param_dict = {}


register = Optimizer.register
create = Optimizer.create_optimizer


def _as_list(x):
    return x if isinstance(x, (list, tuple)) else [x]


def _zeros(weight, count=1, dtype=None):
    """``count`` zero state arrays shaped like ``weight`` (a single array when ``count == 1``)."""
    made = tuple(NDArray(torch.zeros_like(weight._data, dtype=dtype)) for _ in range(count))
    return made[0] if count == 1 else made


def _is_half(weight):
    return weight._data.dtype in (torch.float16, torch.bfloat16)


def _master_then(opt, weight, make_state):
    """Multi-precision state ``(make_state(master), master)`` -- the SGD-family layout (state first)."""
    if opt.multi_precision and _is_half(weight):
        master = NDArray(weight._data.detach().float().clone())
        return (make_state(master), master)
    return make_state(weight)


class _Stepper(Optimizer):
    """Shared plumbing of the concrete optimizers below: hyper-parameters kept as attributes,
    one call that counts the update and resolves (lr, wd, t), and gradient conditioning."""

    def _hyper(self, **values):
        self.__dict__.update(values)

    def _begin(self, index):
        self._update_count(index)
        return self._get_lr(index), self._get_wd(index), self._index_update_count[index]

    def _conditioned(self, grad, decay_with=None, wd=0.0):
        """``clip(rescale * grad (+ wd * decay_with))`` (decay before clipping when given)."""
        g = grad._data * self.rescale_grad
        if decay_with is not None and wd:
            g = g + wd * decay_with._data
        if self.clip_gradient is not None:
            g = torch.clamp(g, -self.clip_gradient, self.clip_gradient)
        return g


@register
class SGD(_Stepper):
    """SGD with optional momentum and multi-precision (fp32 master weights).

    ``state = momentum * state - lr * (rescale_grad * clip(grad) + wd * weight)``; ``weight += state``.
    Lists of indices (``aggregate_num``) run as one multi-tensor update; row_sparse gradients with
    ``lazy_update`` touch only their rows.
    """

    def __init__(self, momentum=0.0, lazy_update=True, **kwargs):
        super().__init__(**kwargs)
        self._hyper(momentum=momentum, lazy_update=lazy_update,
                    aggregate_num=int(kwargs.get('aggregate_num') or 1 << 30))

    def create_state_multi_precision(self, index, weight):
        if _is_half(weight) and not self.multi_precision:
            warnings.warn('Accumulating with float16 in optimizer can lead to poor accuracy or slow convergence. '
                          'Consider using multi_precision=True option of the SGD optimizer')
        return _master_then(self, weight, lambda w: self.create_state(index, w))

    def create_state(self, index, weight):
        return _zeros(weight) if self.momentum != 0.0 else None

    def _apply(self, indices, weights, grads, states, with_master):
        idx, ws, gs, sts = (list(indices), list(weights), list(grads), list(states)) \
            if isinstance(indices, (list, tuple)) else ([indices], [weights], [grads], [states])
        self._update_count(idx)
        lrs, wds, clip = self._get_lrs(idx), self._get_wds(idx), self._clip()
        split = [(st if with_master else (st, None)) for st in sts]
        moms = [None if m is None else m._data for m, _ in split]
        masters = [None if w32 is None else w32._data for _, w32 in split]
        if self.lazy_update and any(_is_rsp(g) for g in gs):
            for w, g, m, w32, lr, wd in zip(ws, gs, moms, masters, lrs, wds):
                _lazy_sgd_rows(w._data, g, m, w32, lr, wd, self.momentum, self.rescale_grad, clip)
            return
        multi_sgd([w._data for w in ws], [g._data for g in gs], moms, masters if with_master else None,
                  lrs, wds, self.momentum, self.rescale_grad, clip)

    def update(self, index, weight, grad, state):
        self._apply(index, weight, grad, state, False)

    def update_multi_precision(self, index, weight, grad, state):
        self._apply(index, weight, grad, state, self.multi_precision and _is_half(_as_list(weight)[0]))


def _is_rsp(g):
    return getattr(g, 'stype', 'default') == 'row_sparse'


def _rsp_rows_of(g, device):
    """(row ids, fp32 row values) of a row_sparse gradient (compressed storage, no densify)."""
    idx = g._aux_arrays()[0].to(device)
    return idx, g._values().to(device).float()


def _prep_grad(gr, w_rows, wd, rescale, clip):
    gr = gr * rescale
    if clip is not None and clip >= 0:
        gr = gr.clamp(-clip, clip)
    return gr + wd * w_rows if wd else gr


@torch.no_grad()
def _lazy_sgd_rows(w, g, mom, w32, lr, wd, momentum, rescale, clip):
    """SGD(-momentum) touching only the rows a row_sparse gradient holds (reference: lazy_update=True,
    src/operator/optimizer_op-inl.h SGDMomLazyUpdateRspImpl)."""
    idx, gr = _rsp_rows_of(g, w.device)
    if idx.numel() == 0:
        return
    tgt = w32 if w32 is not None else w
    rows = tgt.index_select(0, idx).float()
    step = _prep_grad(gr, rows, wd, rescale, clip)
    if momentum != 0.0 and mom is not None:
        m = mom.index_select(0, idx).float().mul_(momentum).sub_(lr * step)
        mom.index_copy_(0, idx, m.to(mom.dtype))
        rows = rows + m
    else:
        rows = rows - lr * step
    tgt.index_copy_(0, idx, rows.to(tgt.dtype))
    if w32 is not None:
        w.index_copy_(0, idx, rows.to(w.dtype))


@torch.no_grad()
def _lazy_adam_rows(w, g, mean, var, lr, beta1, beta2, eps, wd, rescale, clip):
    """Adam over the rows of a row_sparse gradient only (AdamLazyUpdateRspImpl)."""
    idx, gr = _rsp_rows_of(g, w.device)
    if idx.numel() == 0:
        return
    rows = w.index_select(0, idx).float()
    # Adam's order (AdamDnsRspDnsKernel): weight decay joins the gradient before the clip
    step = gr * rescale + wd * rows if wd else gr * rescale
    if clip is not None and clip >= 0:
        step = step.clamp(-clip, clip)
    m = mean.index_select(0, idx).float().mul_(beta1).add_(step, alpha=1 - beta1)
    v = var.index_select(0, idx).float().mul_(beta2).addcmul_(step, step, value=1 - beta2)
    mean.index_copy_(0, idx, m.to(mean.dtype))
    var.index_copy_(0, idx, v.to(var.dtype))
    w.index_copy_(0, idx, (rows - lr * m / (v.sqrt() + eps)).to(w.dtype))


@torch.no_grad()
def multi_sgd(W, G, M, W32, lrs, wds, momentum, rescale, clip):
    """One fused update over many tensors (SGD / SGD-momentum, optional fp32 masters)."""
    if not W:
        return
    if W[0].is_cuda and _K.available() and _K.enabled() and hasattr(_K, 'multi_sgd_mom_tensors') \
            and (momentum == 0.0 or all(m is not None for m in M)):
        _K.multi_sgd_mom_tensors(W, G, M, W32, lrs, wds, momentum, rescale, clip)
        return
    tgt = W32 if W32 is not None else W
    # group by (lr, wd) so each group is a handful of foreach launches
    groups = {}
    for i, (lr, wd) in enumerate(zip(lrs, wds)):
        groups.setdefault((lr, wd), []).append(i)
    for (lr, wd), idx in groups.items():
        g = [G[i].float() if G[i].dtype != tgt[i].dtype else G[i] for i in idx]
        if rescale != 1.0:
            g = torch._foreach_mul(g, rescale)
        if clip is not None and clip >= 0:
            g = [torch.clamp(x, -clip, clip) for x in g]
        w = [tgt[i] for i in idx]
        if wd != 0.0:
            g = torch._foreach_add(g, w, alpha=wd)
        if momentum != 0.0:
            m = [M[i] for i in idx]
            torch._foreach_mul_(m, momentum)
            torch._foreach_add_(m, g, alpha=-lr)
            torch._foreach_add_(w, m)
        else:
            torch._foreach_add_(w, g, alpha=-lr)
        if W32 is not None:
            for i in idx:
                W[i].copy_(W32[i])


@register
class Signum(_Stepper):
    """signSGD / Signum (Bernstein et al. 2018): step by the sign of the (momentum-averaged) gradient."""

    def __init__(self, learning_rate=0.01, momentum=0.9, wd_lh=0.0, **kwargs):
        super().__init__(learning_rate=learning_rate, **kwargs)
        self._hyper(momentum=momentum, wd_lh=wd_lh)

    def create_state(self, index, weight):
        return _zeros(weight) if self.momentum != 0.0 else None

    def update(self, index, weight, grad, state):
        lr, wd, _ = self._begin(index)
        common = dict(lr=lr, wd=wd, rescale_grad=self.rescale_grad, clip_gradient=self._clip())
        if state is None:
            _oo.signsgd_update(weight._data, grad._data, **common)
        else:
            _oo.signum_update(weight._data, grad._data, state._data, momentum=self.momentum, wd_lh=self.wd_lh,
                              **common)


@register
class FTML(_Stepper):
    """FTML (Zheng & Kwok 2017); state (d, v, z)."""

    def __init__(self, beta1=0.6, beta2=0.999, epsilon=1e-8, **kwargs):
        super().__init__(**kwargs)
        self._hyper(beta1=beta1, beta2=beta2, epsilon=epsilon)

    def create_state(self, index, weight):
        return _zeros(weight, 3)

    def update(self, index, weight, grad, state):
        lr, wd, t = self._begin(index)
        d, v, z = (s._data for s in state)
        _oo.ftml_update(weight._data, grad._data, d, v, z, lr=lr, beta1=self.beta1, beta2=self.beta2,
                        epsilon=self.epsilon, t=t, wd=wd, rescale_grad=self.rescale_grad, clip_grad=self._clip())


_NO_LARS_SUFFIXES = ('gamma', 'beta', 'bias')


@register
class LARS(_Stepper):
    """SGD with layer-wise adaptive rate scaling (You et al. 2017): the learning rate of every
    weight tensor is scaled by ``eta * |w| / (|g| + wd * |w| + eps)``."""

    def __init__(self, momentum=0.0, lazy_update=True, eta=0.001, eps=0, momentum_correction=True, **kwargs):
        super().__init__(**kwargs)
        self._hyper(momentum=momentum, eta=eta, eps=eps, lazy_update=lazy_update)

    def create_state(self, index, weight):
        return _zeros(weight, dtype=torch.float32) if self.momentum != 0.0 else None

    def create_state_multi_precision(self, index, weight):
        return _master_then(self, weight, lambda w: self.create_state(index, w))

    def _trust(self, index, weight, grad, lr, wd):
        if self.idx2name.get(index, '').endswith(_NO_LARS_SUFFIXES):
            return lr
        w_norm = float(torch.linalg.vector_norm(weight._data.float()))
        g_norm = float(torch.linalg.vector_norm(grad._data.float() * self.rescale_grad))
        if w_norm > 0.0 and g_norm > 0.0:
            return lr * self.eta * w_norm / (g_norm + wd * w_norm + self.eps)
        return lr

    def update(self, index, weight, grad, state):
        lr, wd, _ = self._begin(index)
        lr = self._trust(index, weight, grad, lr, wd)
        multi_sgd([weight._data], [grad._data], [None if state is None else state._data], None, [lr], [wd],
                  self.momentum, self.rescale_grad, self._clip())

    def update_multi_precision(self, index, weight, grad, state):
        if not (self.multi_precision and _is_half(weight)):
            self.update(index, weight, grad, state)
            return
        mom, master = state
        self.update(index, master, NDArray(grad._data.float()), mom)
        with torch.no_grad():
            weight._data.copy_(master._data)


def _warmup_multiplier(strategy, done, total, peak):
    """Large-batch warm-up factor after ``done`` of ``total`` warm-up updates (1 -> ``peak``)."""
    if done >= total:
        return peak
    if total <= 1:
        return 1.0
    frac = {'linear': done / total, 'power2': (done * done) / (total * total),
            'sqrt': math.sqrt(float(done) / total)}.get(strategy)
    return 1.0 if frac is None else 1.0 + (peak - 1) * frac


@register
class LBSGD(_Stepper):
    """Large-batch SGD: momentum SGD whose learning rate ramps up to ``batch_scale`` x over
    ``warmup_epochs`` (linear, power2 or sqrt)."""

    def __init__(self, momentum=0.0, multi_precision=False, warmup_strategy='linear', warmup_epochs=5,
                 batch_scale=1, updates_per_epoch=32, begin_epoch=0, num_epochs=60, **kwargs):
        super().__init__(multi_precision=multi_precision, **kwargs)
        self._hyper(momentum=momentum, warmup_strategy=warmup_strategy, warmup_epochs=warmup_epochs,
                    batch_scale=batch_scale, updates_per_epoch=updates_per_epoch,
                    init_updates=begin_epoch * updates_per_epoch, num_epochs=num_epochs,
                    lbmult=1, cumgrads={}, adaptive=False, admult=1)

    def create_state(self, index, weight):
        return _zeros(weight) if self.momentum != 0.0 else None

    def _get_lbmult(self, nup):
        return _warmup_multiplier(self.warmup_strategy, nup, self.warmup_epochs * self.updates_per_epoch,
                                  float(self.batch_scale))

    def update(self, index, weight, grad, state):
        lr, wd, _ = self._begin(index)
        lr *= self._get_lbmult(self.num_update - self.init_updates)
        multi_sgd([weight._data], [grad._data], [None if state is None else state._data], None, [lr], [wd],
                  self.momentum, self.rescale_grad, self._clip())


@register
class LAMB(_Stepper):
    """LAMB (You et al. 2019): Adam-style direction, per-tensor trust ratio ``|w| / |update|``
    clamped to [lower_bound, upper_bound]; phase 1 / phase 2 as in the reference operators."""

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-6, lower_bound=None,
                 upper_bound=None, bias_correction=True, **kwargs):
        super().__init__(learning_rate=learning_rate, **kwargs)
        self._hyper(beta1=beta1, beta2=beta2, epsilon=epsilon, lower_bound=lower_bound, upper_bound=upper_bound,
                    bias_correction=bias_correction)

    def create_state(self, index, weight):
        return _zeros(weight, 2, dtype=torch.float32)

    def _step(self, index, weight, grad, mean, var, w32=None):
        lr, wd, t = self._begin(index)
        target = weight._data if w32 is None else w32
        direction = _oo._lamb1(target, grad._data.float(), mean, var, self.beta1, self.beta2, self.epsilon, t,
                               self.bias_correction, wd, self.rescale_grad, self._clip())
        w_norm = torch.linalg.vector_norm(target.float()).reshape(1)
        d_norm = torch.linalg.vector_norm(direction).reshape(1)
        bounds = [-1.0 if b is None else b for b in (self.lower_bound, self.upper_bound)]
        _oo._lamb2(weight._data, direction, w_norm, d_norm, lr, bounds[0], bounds[1], w32=w32)

    def update(self, index, weight, grad, state):
        self._step(index, weight, grad, state[0]._data, state[1]._data)

    def update_multi_precision(self, index, weight, grad, state):
        """Multi-precision state = (fp32 master, (mean, var)) (the reference layout); lists of indices
        (aggregated updates) are applied tensor by tensor."""
        if isinstance(index, (list, tuple)):
            for args in zip(index, weight, grad, state):
                self.update_multi_precision(*args)
            return
        if not self._wants_master(weight):
            self.update(index, weight, grad, state)
            return
        master, (mean, var) = state
        self._step(index, weight, grad, mean._data, var._data, w32=master._data)


@register
class DCASGD(_Stepper):
    """Delay-compensated async SGD (Zheng et al. 2016): the gradient is corrected by
    ``lamda * g * g * (w - w_prev)``; state (momentum or None, previous weight)."""

    def __init__(self, momentum=0.0, lamda=0.04, **kwargs):
        super().__init__(**kwargs)
        self._hyper(momentum=momentum, lamda=lamda, weight_previous={})

    def create_state(self, index, weight):
        previous = NDArray(weight._data.clone())
        return (_zeros(weight) if self.momentum != 0.0 else None, previous)

    @torch.no_grad()
    def update(self, index, weight, grad, state):
        lr, wd, _ = self._begin(index)
        g = self._conditioned(grad)
        mom, previous = state
        w = weight._data
        delta = -lr * (g + wd * w + self.lamda * g * g * (w - previous._data))
        if mom is not None:
            delta = mom._data.mul_(self.momentum).add_(delta)
        previous._data.copy_(w)
        w.add_(delta)


@register
class NAG(_Stepper):
    """Nesterov accelerated gradient (momentum look-ahead); multi-precision like SGD."""

    def __init__(self, momentum=0.0, **kwargs):
        super().__init__(**kwargs)
        self._hyper(momentum=momentum)

    def create_state_multi_precision(self, index, weight):
        return _master_then(self, weight, lambda w: self.create_state(index, w))

    def create_state(self, index, weight):
        return _zeros(weight) if self.momentum != 0.0 else None

    def _nesterov(self, index, weight, grad, mom, w32=None):
        lr, wd, _ = self._begin(index)
        if mom is None:
            _oo._sgd(weight._data, grad._data, lr, wd, self.rescale_grad, self._clip(), w32=w32)
        else:
            _oo._nag(weight._data, grad._data, mom._data, lr, self.momentum, wd, self.rescale_grad, self._clip(),
                     w32=w32)

    def update(self, index, weight, grad, state):
        self._nesterov(index, weight, grad, state)

    def update_multi_precision(self, index, weight, grad, state):
        if self.multi_precision and _is_half(weight):
            mom, master = state
            self._nesterov(index, weight, NDArray(grad._data.float()), mom, w32=master._data)
        else:
            self.update(index, weight, grad, state)


@register
class SGLD(_Stepper):
    """Stochastic gradient Langevin dynamics: half an SGD step plus N(0, lr) noise."""

    def create_state(self, index, weight):
        return None

    @torch.no_grad()
    def update(self, index, weight, grad, state):
        lr, wd, _ = self._begin(index)
        w = weight._data
        w.add_(-lr / 2 * (self._conditioned(grad) + wd * w) + torch.randn_like(w) * math.sqrt(lr))


@register
class ccSGD(SGD):
    """Deprecated alias of SGD kept for API compatibility."""


@register
class Adam(_Stepper):
    """Adam (Kingma & Ba); bias correction folded into the learning rate like the reference."""

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, lazy_update=True, **kwargs):
        super().__init__(learning_rate=learning_rate, **kwargs)
        self._hyper(beta1=beta1, beta2=beta2, epsilon=epsilon, lazy_update=lazy_update)

    def create_state(self, index, weight):
        return _zeros(weight, 2)

    def update(self, index, weight, grad, state):
        lr, wd, t = self._begin(index)
        lr *= math.sqrt(1. - self.beta2 ** t) / (1. - self.beta1 ** t)
        mean, var = state[0]._data, state[1]._data
        clip = self._clip()
        if self.lazy_update and _is_rsp(grad):
            _lazy_adam_rows(weight._data, grad, mean, var, lr, self.beta1, self.beta2, self.epsilon, wd,
                            self.rescale_grad, clip)
        else:
            _oo.adam_update(weight._data, grad._data, mean, var, lr=lr, beta1=self.beta1, beta2=self.beta2,
                            epsilon=self.epsilon, wd=wd, rescale_grad=self.rescale_grad, clip_gradient=clip)


@register
class AdamW(_Stepper):
    """Adam with decoupled weight decay (contrib adamw_update); mp state = (master, mean, var)."""

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, correct_bias=True, **kwargs):
        super().__init__(learning_rate=learning_rate, **kwargs)
        self._hyper(beta1=beta1, beta2=beta2, epsilon=epsilon, correct_bias=correct_bias)

    def create_state(self, index, weight):
        return _zeros(weight, 2, dtype=torch.float32)

    def create_state_multi_precision(self, index, weight):
        if self.multi_precision and _is_half(weight):
            master = NDArray(weight._data.float())
            return (master,) + self.create_state(index, master)
        return self.create_state(index, weight)

    def _decoupled(self, index, weight, grad, mean, var, w32=None):
        lr, wd, t = self._begin(index)
        if self.correct_bias:
            lr *= math.sqrt(1. - self.beta2 ** t) / (1. - self.beta1 ** t)
        _oo._adamw(weight._data, grad._data.float(), mean._data, var._data, self.rescale_grad, lr,
                   self.beta1, self.beta2, self.epsilon, wd, 1.0, self._clip(), w32=w32)

    def update(self, index, weight, grad, state):
        self._decoupled(index, weight, grad, *state)

    def update_multi_precision(self, index, weight, grad, state):
        if self.multi_precision and _is_half(weight):
            master, mean, var = state
            self._decoupled(index, weight, grad, mean, var, w32=master._data)
        else:
            self.update(index, weight, grad, state)


@register
class AdaGrad(_Stepper):
    """AdaGrad: per-element learning rate ``lr / sqrt(sum g^2 + eps)``."""

    def __init__(self, eps=1e-7, **kwargs):
        super().__init__(**kwargs)
        self._hyper(float_stable_eps=eps)

    def create_state(self, index, weight):
        return _zeros(weight)

    @torch.no_grad()
    def update(self, index, weight, grad, state):
        lr, wd, _ = self._begin(index)
        g = self._conditioned(grad)
        history = state._data.add_(g * g)
        w = weight._data
        w.add_(-lr * (g / torch.sqrt(history + self.float_stable_eps) + wd * w))


@register
class RMSProp(_Stepper):
    """RMSProp (Tieleman & Hinton) and, with ``centered``, the Graves 2013 variant."""

    def __init__(self, learning_rate=0.001, gamma1=0.9, gamma2=0.9, epsilon=1e-8, centered=False,
                 clip_weights=None, **kwargs):
        super().__init__(learning_rate=learning_rate, **kwargs)
        self._hyper(gamma1=gamma1, gamma2=gamma2, centered=centered, epsilon=epsilon, clip_weights=clip_weights)

    def create_state(self, index, weight):
        return _zeros(weight, 3) if self.centered else (_zeros(weight),)

    def update(self, index, weight, grad, state):
        lr, wd, _ = self._begin(index)
        common = dict(lr=lr, gamma1=self.gamma1, epsilon=self.epsilon, wd=wd, rescale_grad=self.rescale_grad,
                      clip_gradient=self._clip(), clip_weights=-1.0 if self.clip_weights is None else self.clip_weights)
        tensors = [s._data for s in state]
        if self.centered:
            _oo.rmspropalex_update(weight._data, grad._data, *tensors, gamma2=self.gamma2, **common)
        else:
            _oo.rmsprop_update(weight._data, grad._data, tensors[0], **common)


@register
class AdaDelta(_Stepper):
    """AdaDelta (Zeiler 2012): running averages of g^2 and of the squared steps."""

    def __init__(self, rho=0.90, epsilon=1e-5, **kwargs):
        super().__init__(**kwargs)
        self._hyper(rho=rho, epsilon=epsilon)

    def create_state(self, index, weight):
        return _zeros(weight, 2)

    @torch.no_grad()
    def update(self, index, weight, grad, state):
        _lr, wd, _ = self._begin(index)
        g = self._conditioned(grad)
        sq_grad, sq_step = state[0]._data, state[1]._data
        keep = self.rho
        sq_grad.mul_(keep).add_((1. - keep) * g * g)
        step = torch.sqrt(sq_step + self.epsilon) / torch.sqrt(sq_grad + self.epsilon) * g
        sq_step.mul_(keep).add_((1. - keep) * step * step)
        weight._data.sub_(step + wd * weight._data)


@register
class Ftrl(_Stepper):
    """FTRL-proximal (McMahan et al. 2013); state (z, n)."""

    def __init__(self, lamda1=0.01, learning_rate=0.1, beta=1, **kwargs):
        super().__init__(learning_rate=learning_rate, **kwargs)
        self._hyper(lamda1=lamda1, beta=beta)

    def create_state(self, index, weight):
        return _zeros(weight, 2)

    def update(self, index, weight, grad, state):
        lr, wd, _ = self._begin(index)
        kw = dict(lr=lr, lamda1=self.lamda1, beta=self.beta, wd=wd, rescale_grad=self.rescale_grad,
                  clip_gradient=self._clip())
        if _is_rsp(grad):
            # a row_sparse gradient updates only its rows (reference: the sparse ftrl_update kernel)
            w = weight._data
            rows, gv = _rsp_rows_of(grad, w.device)
            if rows.numel() == 0:
                return
            z, n = state[0]._data, state[1]._data
            wr, zr, nr = w[rows].clone(), z[rows].clone(), n[rows].clone()
            _oo.ftrl_update(wr, gv.to(w.dtype).reshape(wr.shape), zr, nr, **kw)
            with torch.no_grad():
                w[rows], z[rows], n[rows] = wr, zr, nr
            return
        _oo.ftrl_update(weight._data, grad._data, state[0]._data, state[1]._data, **kw)


@register
class Adamax(_Stepper):
    """AdaMax (Adam with the infinity norm): ``u = max(beta2 * u, |g|)``."""

    def __init__(self, learning_rate=0.002, beta1=0.9, beta2=0.999, **kwargs):
        super().__init__(learning_rate=learning_rate, **kwargs)
        self._hyper(beta1=beta1, beta2=beta2)

    def create_state(self, index, weight):
        return _zeros(weight, 2)

    @torch.no_grad()
    def update(self, index, weight, grad, state):
        lr, wd, t = self._begin(index)
        g = self._conditioned(grad, decay_with=weight, wd=wd)
        first, inf_norm = state[0]._data, state[1]._data
        first.mul_(self.beta1).add_((1. - self.beta1) * g)
        inf_norm.copy_(torch.maximum(self.beta2 * inf_norm, torch.abs(g)))
        weight._data.sub_(lr / (1. - self.beta1 ** t) * first / inf_norm)


@register
class Nadam(_Stepper):
    """Nesterov Adam (Dozat 2016) with the momentum schedule ``beta1 (1 - 0.5 * 0.96^(t * decay))``."""

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, schedule_decay=0.004, **kwargs):
        super().__init__(learning_rate=learning_rate, **kwargs)
        self._hyper(beta1=beta1, beta2=beta2, epsilon=epsilon, schedule_decay=schedule_decay, m_schedule=1.)

    def create_state(self, index, weight):
        return _zeros(weight, 2)

    def _mu(self, step):
        return self.beta1 * (1. - 0.5 * pow(0.96, step * self.schedule_decay))

    @torch.no_grad()
    def update(self, index, weight, grad, state):
        lr, wd, t = self._begin(index)
        g = self._conditioned(grad, decay_with=weight, wd=wd)
        mu_now, mu_next = self._mu(t), self._mu(t + 1)
        self.m_schedule *= mu_now
        first, second = state[0]._data, state[1]._data
        first.mul_(self.beta1).add_((1. - self.beta1) * g)
        second.mul_(self.beta2).add_((1. - self.beta2) * g * g)
        blended = (1. - mu_now) * g / (1. - self.m_schedule) + mu_next * first / (1. - self.m_schedule * mu_next)
        second_hat = second / (1. - pow(self.beta2, t))
        weight._data.sub_(lr * blended / (torch.sqrt(second_hat) + self.epsilon))


@register
class GroupAdaGrad(_Stepper):
    """AdaGrad with one accumulator per row (python/mxnet/optimizer/contrib.py)."""

    def __init__(self, eps=1e-5, **kwargs):
        super().__init__(**kwargs)
        self._hyper(float_stable_eps=eps)

    def create_state(self, index, weight):
        assert len(weight.shape) == 2
        return NDArray(torch.zeros((weight.shape[0], 1), dtype=weight._data.dtype, device=weight._data.device))

    @torch.no_grad()
    def update(self, index, weight, grad, state):
        lr, wd, _ = self._begin(index)
        assert wd == 0, 'Weight decay is not supported for GroupAdaGrad'
        g = self._conditioned(grad)
        state._data.add_((g * g).mean(1, keepdim=True))
        weight._data.sub_(lr * g / torch.sqrt(state._data + self.float_stable_eps))


@register
class Test(_Stepper):
    """Test optimizer: ``weight += rescale_grad * grad``; the state mirrors the weight."""

    def create_state(self, index, weight):
        return _zeros(weight)

    @torch.no_grad()
    def update(self, index, weight, grad, state):
        weight._data.add_(grad._data * self.rescale_grad)
        state._data.copy_(weight._data)


class Updater:
    """Updater for kvstore (applies an Optimizer given index, grad, weight)."""

    def __init__(self, optimizer):
        self.optimizer = optimizer
        self.states = {}
        self.states_synced = {}
        self.aggregate_updates = optimizer.aggregate_num > 0

    def __call__(self, index, grad, weight):
        if not isinstance(index, (list, tuple)):
            indices, grads, weights = [index], [grad], [weight]
        else:
            indices, grads, weights = index, grad, weight
        if weights:
            # one update-count table per device: updaters of different contexts advance it independently
            # (the Trainer numbers its per-context updaters; CPU contexts share one torch device)
            slot = getattr(self, 'device_slot', None)
            self.optimizer._set_current_context(slot if slot is not None else weights[0].context.device_id)
        for i, idx in enumerate(indices):
            if idx not in self.states:
                self.states[idx] = self.optimizer.create_state_multi_precision(idx, weights[i])
                self.states_synced[idx] = True
            elif not self.states_synced[idx]:
                self.states[idx] = self.sync_state_context(self.states[idx], weights[i].context)
                self.states_synced[idx] = True
        if self.aggregate_updates and isinstance(self.optimizer, SGD):
            self.optimizer.update_multi_precision(list(indices), list(weights), list(grads),
                                                  [self.states[i] for i in indices])
        else:
            for i, w, g in zip(indices, weights, grads):
                self.optimizer.update_multi_precision(i, w, g, self.states[i])

    def sync_state_context(self, state, context):
        if isinstance(state, NDArray):
            return state.as_in_context(context)
        if isinstance(state, (tuple, list)):
            synced = [self.sync_state_context(i, context) for i in state]
            return tuple(synced) if isinstance(state, tuple) else synced
        return state

    def set_states(self, states):
        states = pickle.loads(states)
        if isinstance(states, tuple) and len(states) == 2:
            self.states, self.optimizer = states
        else:
            self.states = states
        self.states_synced = dict.fromkeys(self.states.keys(), False)

    def get_states(self, dump_optimizer=False):
        return pickle.dumps((self.states, self.optimizer) if dump_optimizer else self.states)


def get_updater(optimizer):
    return Updater(optimizer)
