"""SequentialModule: a pipeline of modules, each consuming the previous one's outputs.

API parity: python/mxnet/module/sequential_module.py (``add(module,
take_labels=..., auto_wiring=...)``).  Forward feeds stage i's outputs as stage
i+1's data; backward walks the stages in reverse, feeding each stage's input
gradients to its predecessor as output gradients.
"""
import copy
import logging
from collections import namedtuple

from ..initializer import Uniform
from ..io import DataDesc
from .base_module import BaseModule

__all__ = ['SequentialModule']

_Stage = namedtuple('_Stage', ['module', 'take_labels', 'auto_wiring'])


class SequentialModule(BaseModule):
    META_TAKE_LABELS = 'take_labels'
    META_AUTO_WIRING = 'auto_wiring'
    _METAS = (META_TAKE_LABELS, META_AUTO_WIRING)

    def __init__(self, logger=logging):
        super().__init__(logger=logger)
        self._stages = []
        self._data_shapes = None
        self._label_shapes = None

    @property
    def _modules(self):
        return [s.module for s in self._stages]

    def add(self, module, **kwargs):
        """Append a stage; ``take_labels`` feeds it the batch labels, ``auto_wiring`` renames the
        incoming data to its own data names.  Returns self (chainable)."""
        unknown = set(kwargs) - set(self._METAS)
        if unknown:
            raise AssertionError('unknown SequentialModule meta %s (a typo?)' % sorted(unknown))
        self._stages.append(_Stage(module, bool(kwargs.get(self.META_TAKE_LABELS, False)),
                                   bool(kwargs.get(self.META_AUTO_WIRING, False))))
        self.binded = self.params_initialized = self.optimizer_initialized = False
        return self

    # ---------------------------------------------------------------- names / shapes
    @property
    def data_names(self):
        return self._stages[0].module.data_names if self._stages else []

    @property
    def output_names(self):
        return self._stages[-1].module.output_names if self._stages else []

    @property
    def data_shapes(self):
        self._require('binded')
        return self._stages[0].module.data_shapes

    @property
    def label_shapes(self):
        self._require('binded')
        return self._label_shapes

    @property
    def output_shapes(self):
        self._require('binded')
        return self._stages[-1].module.output_shapes

    @property
    def symbol(self):
        return self._stages[-1].module.symbol if self._stages else None

    # ---------------------------------------------------------------- parameters
    def get_params(self):
        self._require('binded', 'params_initialized')
        args, auxs = {}, {}
        for s in self._stages:
            a, x = s.module.get_params()
            args.update(a)
            auxs.update(x)
        return args, auxs

    def init_params(self, initializer=Uniform(0.01), arg_params=None, aux_params=None, allow_missing=False,
                    force_init=False, allow_extra=False):
        if self.params_initialized and not force_init:
            return
        if not self.binded:
            raise AssertionError('call bind before initializing the parameters')
        for s in self._stages:
            s.module.init_params(initializer=initializer, arg_params=arg_params, aux_params=aux_params,
                                 allow_missing=allow_missing, force_init=force_init, allow_extra=allow_extra)
        # a parameter name may belong to one stage only
        owner = {'arg': {}, 'aux': {}}
        for i, s in enumerate(self._stages):
            for kind, params in zip(('arg', 'aux'), s.module.get_params()):
                for name in params:
                    if name in owner[kind]:
                        j = owner[kind][name]
                        raise AssertionError('Duplicated parameter names: "%s" of stage %d (%s) is already used by '
                                             'stage %d (%s)' % (name, i, type(s.module), j,
                                                                type(self._stages[j].module)))
                    owner[kind][name] = i
        self.params_initialized = True

    # ---------------------------------------------------------------- binding
    def bind(self, data_shapes, label_shapes=None, for_training=True, inputs_need_grad=False, force_rebind=False,
             shared_module=None, grad_req='write'):
        if self.binded and not force_rebind:
            self.logger.warning('Already bound, ignoring bind()')
            return
        if inputs_need_grad and not for_training:
            raise AssertionError('inputs_need_grad requires for_training')
        if shared_module is not None:
            raise AssertionError('shared_module is not supported by SequentialModule')
        if not self._stages:
            raise AssertionError('cannot bind an empty SequentialModule')
        self.binded = True
        feed = data_shapes
        uses_labels = False
        for i, s in enumerate(self._stages):
            if s.auto_wiring:
                names = s.module.data_names
                if len(names) != len(feed):
                    raise AssertionError('auto_wiring: stage %d expects %d inputs, got %d' % (i, len(names), len(feed)))
                feed = [DataDesc(n, getattr(d, 'shape', None) or d[1]) for n, d in zip(names, feed)]
            uses_labels |= s.take_labels
            # every stage after the first must hand gradients back to its predecessor
            s.module.bind(data_shapes=feed, label_shapes=label_shapes if s.take_labels else None,
                          for_training=for_training, inputs_need_grad=bool(inputs_need_grad or (for_training and i)),
                          force_rebind=force_rebind, shared_module=None, grad_req=grad_req)
            feed = s.module.output_shapes
        self._label_shapes = label_shapes if uses_labels else None

    def init_optimizer(self, kvstore='local', optimizer='sgd', optimizer_params=(('learning_rate', 0.01),),
                       force_init=False):
        self._require('binded', 'params_initialized')
        if self.optimizer_initialized and not force_init:
            self.logger.warning('optimizer already initialized, ignoring.')
            return
        for s in self._stages:
            s.module.init_optimizer(kvstore=kvstore, optimizer=optimizer, optimizer_params=optimizer_params,
                                    force_init=force_init)
        self.optimizer_initialized = True

    # ---------------------------------------------------------------- computation
    def forward(self, data_batch, is_train=None):
        self._require('binded', 'params_initialized')
        batch = copy.copy(data_batch)
        last = len(self._stages) - 1
        for i, s in enumerate(self._stages):
            s.module.forward(batch, is_train=is_train)
            if i == last:
                break
            batch.data = s.module.get_outputs()
            if hasattr(batch, 'provide_data'):
                names = [d[0] for d in s.module.output_shapes]
                if len(names) != len(batch.data):
                    raise AssertionError('stage %d output count changed' % i)
                batch.provide_data = [(n, a.shape) for n, a in zip(names, batch.data)]

    def backward(self, out_grads=None):
        self._require('binded', 'params_initialized')
        grads = out_grads
        for i in range(len(self._stages) - 1, -1, -1):
            mod = self._stages[i].module
            mod.backward(out_grads=grads)
            if i:
                grads = mod.get_input_grads()

    def update(self):
        self._require('binded', 'params_initialized', 'optimizer_initialized')
        for s in self._stages:
            s.module.update()

    def get_outputs(self, merge_multi_context=True):
        self._require('binded', 'params_initialized')
        return self._stages[-1].module.get_outputs(merge_multi_context=merge_multi_context)

    def get_input_grads(self, merge_multi_context=True):
        self._require('binded', 'params_initialized', 'inputs_need_grad')
        return self._stages[0].module.get_input_grads(merge_multi_context=merge_multi_context)

    def update_metric(self, eval_metric, labels, pre_sliced=False):
        self._require('binded', 'params_initialized')
        for s in self._stages:
            if s.take_labels:
                s.module.update_metric(eval_metric, labels, pre_sliced)

    def install_monitor(self, mon):
        self._require('binded')
        for s in self._stages:
            s.module.install_monitor(mon)
