"""BucketingModule: one Module per bucket key, all sharing one set of parameters.

API parity: python/mxnet/module/bucketing_module.py.  ``sym_gen(bucket_key)``
returns ``(symbol, data_names, label_names)``.  The default bucket's module owns
the parameters (and optimizer); a module for any other key is created on first
use and bound with ``shared_module=<default>`` so its executors alias the same
parameter / gradient arrays.  Each batch selects its bucket by
``data_batch.bucket_key``.
"""
import logging
import warnings

from .. import context as ctx_mod
from ..initializer import Uniform
from .base_module import BaseModule, _check_input_names
from .module import Module

__all__ = ['BucketingModule']


class BucketingModule(BaseModule):
    def __init__(self, sym_gen, default_bucket_key=None, logger=logging, context=None, work_load_list=None,
                 fixed_param_names=None, state_names=None, group2ctxs=None, compression_params=None):
        super().__init__(logger=logger)
        if default_bucket_key is None:
            raise AssertionError('BucketingModule needs a default_bucket_key')
        self._sym_gen = sym_gen
        self._default_bucket_key = default_bucket_key
        sym, data_names, label_names = self._call_sym_gen(default_bucket_key)
        self._fixed_param_names = list(fixed_param_names or [])
        self._state_names = list(state_names or [])
        for names, kind, strict in ((list(data_names or []), 'data', True), (list(label_names or []), 'label', False),
                                    (self._state_names, 'state', True), (self._fixed_param_names, 'fixed_param', True)):
            _check_input_names(sym, names, kind, strict)
        # construction arguments shared by every per-bucket Module
        self._module_kwargs = dict(logger=logger, context=context if context is not None else ctx_mod.cpu(),
                                   work_load_list=work_load_list, fixed_param_names=self._fixed_param_names,
                                   state_names=self._state_names, group2ctxs=group2ctxs,
                                   compression_params=compression_params)
        self._context = self._module_kwargs['context']
        self._buckets = {}
        self._active = None
        self._active_key = None
        self._dirty = False
        self._monitor = None
        self._grad_req = None
        self._preload = None

    # reference attribute names (tests and user code reach into these)
    _curr_module = property(lambda self: self._active)
    _curr_bucket_key = property(lambda self: self._active_key)

    def _call_sym_gen(self, *args, **kwargs):
        # a fresh name scope per call: every bucket's graph names its auto-named nodes alike
        # (embedding0_weight in each), so parameters are shared by name across buckets
        from ..name import NameManager
        with NameManager():
            return self._sym_gen(*args, **kwargs)

    def _reset_bind(self):
        self.binded = False
        self._buckets = {}
        self._active = None
        self._active_key = None

    def _new_module(self, key):
        sym, data_names, label_names = self._call_sym_gen(key)
        return Module(sym, data_names, label_names, **self._module_kwargs)

    @property
    def _default_module(self):
        return self._buckets[self._default_bucket_key]

    # ---------------------------------------------------------------- names / shapes
    def _default_sym_info(self):
        return self._call_sym_gen(self._default_bucket_key)

    @property
    def data_names(self):
        return self._active.data_names if self.binded else self._default_sym_info()[1]

    @property
    def output_names(self):
        return self._active.output_names if self.binded else self._default_sym_info()[0].list_outputs()

    @property
    def data_shapes(self):
        self._require('binded')
        return self._active.data_shapes

    @property
    def label_shapes(self):
        self._require('binded')
        return self._active.label_shapes

    @property
    def output_shapes(self):
        self._require('binded')
        return self._active.output_shapes

    @property
    def symbol(self):
        self._require('binded')
        return self._active.symbol

    # ---------------------------------------------------------------- parameters
    def get_params(self):
        self._require('binded', 'params_initialized')
        self._active._params_dirty = self._dirty
        out = self._active.get_params()
        self._dirty = False
        return out

    def set_params(self, arg_params, aux_params, allow_missing=False, force_init=True, allow_extra=False):
        if not allow_missing:
            self.init_params(initializer=None, arg_params=arg_params, aux_params=aux_params, allow_missing=False,
                             force_init=force_init)
            return
        if self.params_initialized and not force_init:
            warnings.warn('Parameters already initialized and force_init=False. set_params call ignored.',
                          stacklevel=2)
            return
        self._active.set_params(arg_params, aux_params, allow_missing=True, force_init=force_init,
                                     allow_extra=allow_extra)
        self._dirty = True
        self.params_initialized = True

    def init_params(self, initializer=Uniform(0.01), arg_params=None, aux_params=None, allow_missing=False,
                    force_init=False, allow_extra=False):
        if self.params_initialized and not force_init:
            return
        if not self.binded:
            raise AssertionError('call bind before initializing the parameters')
        self._active.init_params(initializer=initializer, arg_params=arg_params, aux_params=aux_params,
                                      allow_missing=allow_missing, force_init=force_init, allow_extra=allow_extra)
        self._dirty = False
        self.params_initialized = True

    def get_states(self, merge_multi_context=True):
        self._require('binded', 'params_initialized')
        return self._active.get_states(merge_multi_context=merge_multi_context)

    def set_states(self, states=None, value=None):
        self._require('binded', 'params_initialized')
        self._active.set_states(states, value)

    # ---------------------------------------------------------------- binding / buckets
    def bind(self, data_shapes, label_shapes=None, for_training=True, inputs_need_grad=False, force_rebind=False,
             shared_module=None, grad_req='write'):
        saved = self.get_params() if self.params_initialized else None
        if force_rebind:
            self._reset_bind()
        if self.binded:
            self.logger.warning('Already bound, ignoring bind()')
            return
        if shared_module is not None:
            raise AssertionError('shared_module is not supported by BucketingModule')
        self.for_training, self.inputs_need_grad, self._grad_req = for_training, inputs_need_grad, grad_req
        self.binded = True
        mod = self._new_module(self._default_bucket_key)
        mod.bind(data_shapes, label_shapes, for_training, inputs_need_grad, force_rebind=False, shared_module=None,
                 grad_req=grad_req)
        self._buckets[self._default_bucket_key] = mod
        self._active, self._active_key = mod, self._default_bucket_key
        if saved is None and self._preload is not None:      # BucketingModule.load()
            saved, self._preload = self._preload, None
            self.params_initialized = True
        if saved is not None:
            self.set_params(*saved)

    def switch_bucket(self, bucket_key, data_shapes, label_shapes=None):
        """Make ``bucket_key`` current, creating / binding its module on first use."""
        self._require('binded')
        mod = self._buckets.get(bucket_key)
        if mod is None:
            mod = self._new_module(bucket_key)
            self._buckets[bucket_key] = mod
            if self._monitor is not None:
                self._bind_shared(mod, data_shapes, label_shapes)
                mod.install_monitor(self._monitor)
        if not mod.binded:
            self._bind_shared(mod, data_shapes, label_shapes)
        self._active, self._active_key = mod, bucket_key

    def _bind_shared(self, mod, data_shapes, label_shapes):
        if mod.binded:
            return
        cur = self._active
        mod.bind(data_shapes, label_shapes, cur.for_training, cur.inputs_need_grad, force_rebind=False,
                 shared_module=self._default_module, grad_req=self._grad_req)

    def init_optimizer(self, kvstore='local', optimizer='sgd', optimizer_params=(('learning_rate', 0.01),),
                       force_init=False):
        self._require('binded', 'params_initialized')
        if self.optimizer_initialized and not force_init:
            self.logger.warning('optimizer already initialized, ignoring.')
            return
        self._active.init_optimizer(kvstore, optimizer, optimizer_params, force_init=force_init)
        for mod in self._buckets.values():
            if mod is not self._active:
                mod.borrow_optimizer(self._active)
        self.optimizer_initialized = True

    # ---------------------------------------------------------------- computation
    def prepare(self, data_batch, sparse_row_id_fn=None):
        self._require('binded', 'params_initialized')
        home = self._active_key
        self.switch_bucket(data_batch.bucket_key, data_batch.provide_data, data_batch.provide_label)
        self._active.prepare(data_batch, sparse_row_id_fn=sparse_row_id_fn)
        self.switch_bucket(home, None, None)

    def forward(self, data_batch, is_train=None):
        self._require('binded', 'params_initialized')
        self.switch_bucket(data_batch.bucket_key, data_batch.provide_data, data_batch.provide_label)
        self._active.forward(data_batch, is_train=is_train)

    def backward(self, out_grads=None):
        self._require('binded', 'params_initialized')
        self._active.backward(out_grads=out_grads)

    def update(self):
        self._require('binded', 'params_initialized', 'optimizer_initialized')
        self._dirty = True
        self._active.update()

    def get_outputs(self, merge_multi_context=True):
        self._require('binded', 'params_initialized')
        return self._active.get_outputs(merge_multi_context=merge_multi_context)

    def get_input_grads(self, merge_multi_context=True):
        self._require('binded', 'params_initialized', 'inputs_need_grad')
        return self._active.get_input_grads(merge_multi_context=merge_multi_context)

    def update_metric(self, eval_metric, labels, pre_sliced=False):
        self._require('binded', 'params_initialized')
        self._active.update_metric(eval_metric, labels, pre_sliced)

    def install_monitor(self, mon):
        self._require('binded')
        self._monitor = mon
        for mod in self._buckets.values():
            mod.install_monitor(mon)

    # ---------------------------------------------------------------- checkpoints
    def save_checkpoint(self, prefix, epoch, remove_amp_cast=False):
        if not (self.binded and self._buckets):
            raise AssertionError('bind before saving a checkpoint')
        self._active.save_checkpoint(prefix, epoch)

    @staticmethod
    def load(prefix, epoch, sym_gen=None, default_bucket_key=None, **kwargs):
        """A BucketingModule whose parameters are set from ``prefix-%04d.params`` at bind time."""
        from ..model import load_params
        if sym_gen is None or default_bucket_key is None:
            raise AssertionError('BucketingModule.load needs sym_gen and default_bucket_key')
        mod = BucketingModule(sym_gen=sym_gen, default_bucket_key=default_bucket_key, **kwargs)
        mod._preload = load_params(prefix, epoch)
        return mod
