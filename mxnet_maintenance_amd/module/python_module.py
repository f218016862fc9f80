"""Modules implemented directly in Python (API parity: python/mxnet/module/python_module.py).

``PythonModule`` is a parameter-free module: subclasses supply
``_compute_output_shapes`` and the forward / backward computation, and get
no-op parameter / optimizer handling.  ``PythonLossModule`` is the typical
use: it passes its input scores through as the output and, in backward,
returns ``grad_func(scores, labels)`` as the gradient of its input.
"""
import logging

from .. import ndarray as nd
from ..initializer import Uniform
from .base_module import BaseModule

__all__ = ['PythonModule', 'PythonLossModule']


def _listify(names):
    return list(names) if isinstance(names, tuple) else names


class PythonModule(BaseModule):
    def __init__(self, data_names, label_names, output_names, logger=logging):
        super().__init__(logger=logger)
        self._data_names = _listify(data_names)
        self._label_names = _listify(label_names)
        self._output_names = list(output_names)
        self._shapes = {'data': None, 'label': None, 'output': None}

    data_names = property(lambda self: self._data_names)
    output_names = property(lambda self: self._output_names)
    data_shapes = property(lambda self: self._shapes['data'])
    label_shapes = property(lambda self: self._shapes['label'])
    output_shapes = property(lambda self: self._shapes['output'])

    # reference attribute names
    _data_shapes = property(lambda self: self._shapes['data'])
    _label_shapes = property(lambda self: self._shapes['label'])

    # a Python module has no parameters and no optimizer
    def get_params(self):
        return {}, {}

    def init_params(self, initializer=Uniform(0.01), arg_params=None, aux_params=None, allow_missing=False,
                    force_init=False, allow_extra=False):
        return None

    def init_optimizer(self, kvstore='local', optimizer='sgd', optimizer_params=(('learning_rate', 0.01),),
                       force_init=False):
        return None

    def update(self):
        return None

    def update_metric(self, eval_metric, labels, pre_sliced=False):
        if self._shapes['label'] is None:
            return
        if pre_sliced:
            raise RuntimeError('PythonModule does not support pre-sliced labels')
        eval_metric.update(labels, self.get_outputs())

    def bind(self, data_shapes, label_shapes=None, for_training=True, inputs_need_grad=False, force_rebind=False,
             shared_module=None, grad_req='write'):
        if self.binded and not force_rebind:
            self.logger.warning('%s is already bound; bind() ignored', type(self).__name__)
            return
        if grad_req != 'write':
            raise AssertionError('PythonModule supports grad_req="write" only')
        if [d[0] for d in data_shapes] != list(self._data_names):
            raise AssertionError('data_shapes %s do not match data_names %s' % (data_shapes, self._data_names))
        if label_shapes is not None and (self._label_names is None or
                                         [d[0] for d in label_shapes] != list(self._label_names)):
            raise AssertionError('label_shapes %s do not match label_names %s' % (label_shapes, self._label_names))
        self.for_training, self.inputs_need_grad = for_training, inputs_need_grad
        self._shapes['data'] = data_shapes
        self._shapes['label'] = label_shapes
        self._shapes['output'] = self._compute_output_shapes()

    def _compute_output_shapes(self):
        raise NotImplementedError('PythonModule subclasses define their output shapes')


class PythonLossModule(PythonModule):
    """Identity forward on the scores; backward input gradient = ``grad_func(scores, labels)``."""

    def __init__(self, name='pyloss', data_names=('data',), label_names=('softmax_label',), logger=logging,
                 grad_func=None):
        if len(data_names) != 1 or len(label_names) != 1:
            raise AssertionError('PythonLossModule takes exactly one data and one label input')
        if grad_func is not None and not callable(grad_func):
            raise AssertionError('grad_func must be callable')
        super().__init__(data_names, label_names, [name + '_output'], logger=logger)
        self._name = name
        self._grad_func = grad_func
        self._pred = self._label_val = self._pred_grad = None

    def _compute_output_shapes(self):
        return [(self._name + '_output', self._shapes['data'][0][1])]

    def forward(self, data_batch, is_train=None):
        train = self.for_training if is_train is None else is_train
        self._pred = data_batch.data[0]
        if train:
            self._label_val = data_batch.label[0]

    def get_outputs(self, merge_multi_context=True):
        if not merge_multi_context:
            raise AssertionError('PythonLossModule has a single context')
        return [self._pred]

    def backward(self, out_grads=None):
        if out_grads is not None:
            raise AssertionError('a loss module takes no output gradients')
        if not self.for_training:
            raise AssertionError('bind with for_training=True to run backward')
        self._backward_impl()

    def _backward_impl(self):
        if self._grad_func is None:
            raise NotImplementedError('PythonLossModule needs grad_func (or override _backward_impl)')
        g = self._grad_func(self._pred, self._label_val)
        self._pred_grad = g if isinstance(g, nd.NDArray) else nd.array(g)

    def get_input_grads(self, merge_multi_context=True):
        if not merge_multi_context:
            raise AssertionError('PythonLossModule has a single context')
        return [self._pred_grad] if self._pred_grad is not None else [None]

    def install_monitor(self, mon):
        raise NotImplementedError('PythonLossModule has no executor to monitor')
