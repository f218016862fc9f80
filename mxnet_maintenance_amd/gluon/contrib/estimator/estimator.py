"""High-level training loop for Gluon (parity: gluon/contrib/estimator/estimator.py).

``Estimator(net, loss, train_metrics, val_metrics, trainer, context).fit(train_data, val_data, epochs)``
runs the loop, dispatching to event handlers sorted by priority:
train_begin -> [epoch_begin -> [batch_begin -> fit_batch -> batch_end]* -> epoch_end]* -> train_end.
"""
import copy
import logging
import sys
import warnings

from .... import metric as metric_mod
from ....context import Context, cpu, num_gpus, gpu
from ....metric import Accuracy, Loss as metric_loss, EvalMetric
from ...loss import Loss as gluon_loss, SoftmaxCrossEntropyLoss
from ...trainer import Trainer
from ...utils import split_and_load
from .batch_processor import BatchProcessor
from .event_handler import (TrainBegin, TrainEnd, EpochBegin, EpochEnd, BatchBegin, BatchEnd, StoppingHandler,
                            MetricHandler, ValidationHandler, LoggingHandler, GradientUpdateHandler,
                            _check_event_handlers)

__all__ = ['Estimator']


def _check_metrics(metrics):
    if isinstance(metrics, CompositeEvalMetric_):
        metrics = [m for metric in metrics.metrics for m in _check_metrics(metric)]
    elif isinstance(metrics, EvalMetric):
        metrics = [metrics]
    else:
        metrics = metrics or []
        if not all(isinstance(metric, EvalMetric) for metric in metrics):
            raise ValueError('metrics must be a Metric or a list of Metric, refer to mxnet.metric.EvalMetric: '
                             '%s' % metrics)
    return metrics


CompositeEvalMetric_ = metric_mod.CompositeEvalMetric


class Estimator:
    logger = None

    def __init__(self, net, loss, train_metrics=None, val_metrics=None, initializer=None, trainer=None,
                 context=None, val_net=None, val_loss=None, batch_processor=None):
        self.net = net
        self.loss = self._check_loss(loss)
        self._train_metrics = _check_metrics(train_metrics)
        self._val_metrics = _check_metrics(val_metrics)
        self._add_default_training_metrics()
        self._add_validation_metrics()
        self.val_loss = self._check_loss(val_loss) if val_loss is not None else self.loss
        self.val_net = val_net if val_net is not None else self.net
        self.logger = logging.Logger(name='Estimator', level=logging.INFO)
        self.logger.addHandler(logging.StreamHandler(sys.stdout))
        self.context = self._check_context(context)
        self._initialize(initializer)
        self.trainer = self._check_trainer(trainer)
        self.batch_processor = batch_processor if batch_processor is not None else BatchProcessor()
        self.max_epoch = None
        self.max_batch = None
        self.batch_axis = 0

    def _check_loss(self, loss):
        if not isinstance(loss, gluon_loss):
            raise ValueError('loss must be a Loss, refer to gluon.loss.Loss:{}'.format(loss))
        return loss

    def _check_context(self, context):
        if context:
            if isinstance(context, Context):
                context = [context]
            elif isinstance(context, list) and all(isinstance(c, Context) for c in context):
                pass
            else:
                raise ValueError('context must be a Context or a list of Context, refer to mxnet.Context: '
                                 '{}'.format(context))
            return context
        return [gpu(i) for i in range(num_gpus())] or [cpu()]

    def _initialize(self, initializer):
        if not self._is_initialized():
            from ....initializer import Uniform
            self.net.initialize(init=initializer or Uniform(), ctx=self.context)
        elif initializer is not None:
            warnings.warn('Network already fully initialized, skipping initialization. You don\'t need to pass '
                          'initializer if you already initialized your net. You can use net.initialize('
                          'force_reinit=True) to re-initialize.')

    def _check_trainer(self, trainer):
        if not trainer:
            warnings.warn('No trainer specified, default SGD optimizer with learning rate 0.001 is used.')
            trainer = Trainer(self.net.collect_params(), 'sgd', {'learning_rate': 0.001})
        elif not isinstance(trainer, Trainer):
            raise ValueError('Trainer must be a Gluon Trainer instance, refer to gluon.Trainer:{}'.format(trainer))
        return trainer

    def _is_initialized(self):
        param_dict = self.net.collect_params()
        for param in param_dict.values():
            try:
                param.list_ctx()
            except Exception:
                return False
        return True

    def _add_default_training_metrics(self):
        if not self._train_metrics:
            suggested = Accuracy() if isinstance(self.loss, SoftmaxCrossEntropyLoss) else None
            self._train_metrics = [suggested] if suggested is not None else []
        loss_name = self.loss.name.rstrip('1234567890')
        self._train_metrics.append(metric_loss(loss_name))
        for metric in self._train_metrics:
            metric.name = 'training ' + metric.name

    def _add_validation_metrics(self):
        if not self._val_metrics:
            self._val_metrics = [copy.deepcopy(metric) for metric in self._train_metrics]
        for metric in self._val_metrics:
            if 'training' in metric.name:
                metric.name = metric.name.replace('training', 'validation')
            elif 'validation' not in metric.name:
                metric.name = 'validation ' + metric.name

    @property
    def train_metrics(self):
        return self._train_metrics

    @property
    def val_metrics(self):
        return self._val_metrics

    def evaluate(self, val_data, batch_axis=0, event_handlers=None):
        for metric in self.val_metrics:
            metric.reset()
        event_handlers = self._prepare_default_validation_handlers(event_handlers)
        _, epoch_begin, batch_begin, batch_end, epoch_end, _ = self._categorize_handlers(event_handlers)
        estimator_ref = self
        for handler in epoch_begin:
            handler.epoch_begin(estimator_ref)
        for _, batch in enumerate(val_data):
            for handler in batch_begin:
                handler.batch_begin(estimator_ref, batch=batch)
            _, label, pred, loss = self.batch_processor.evaluate_batch(estimator_ref, batch, batch_axis)
            for handler in batch_end:
                handler.batch_end(estimator_ref, batch=batch, pred=pred, label=label, loss=loss)
        for handler in epoch_end:
            handler.epoch_end(estimator_ref)

    def fit(self, train_data, val_data=None, epochs=None, event_handlers=None, batches=None, batch_axis=0):
        if not isinstance(train_data, (list, tuple)) and not hasattr(train_data, '__iter__'):
            raise ValueError('train_data must be iterable')
        if not epochs and not batches:
            raise ValueError('Please specify either epochs or batches.')
        if epochs and batches:
            raise ValueError('Only one of epochs and batches can be specified.')
        self.max_epoch = epochs
        self.max_batch = batches
        self.batch_axis = batch_axis
        event_handlers = self._prepare_default_handlers(val_data, event_handlers)
        train_begin, epoch_begin, batch_begin, batch_end, epoch_end, train_end = \
            self._categorize_handlers(event_handlers)
        self._handlers = event_handlers
        estimator_ref = self
        for handler in train_begin:
            handler.train_begin(estimator_ref)
        while True:
            for handler in epoch_begin:
                handler.epoch_begin(estimator_ref)
            stop = False
            for _, batch in enumerate(train_data):
                for handler in batch_begin:
                    handler.batch_begin(estimator_ref, batch=batch)
                _, label, pred, loss = self.batch_processor.fit_batch(estimator_ref, batch, batch_axis)
                batch_end_result = []
                for handler in batch_end:
                    batch_end_result.append(handler.batch_end(estimator_ref, batch=batch, pred=pred, label=label,
                                                              loss=loss))
                if any(batch_end_result):
                    stop = True
                    break
            epoch_end_result = []
            for handler in epoch_end:
                epoch_end_result.append(handler.epoch_end(estimator_ref))
            if stop or any(epoch_end_result):
                break
        for handler in train_end:
            handler.train_end(estimator_ref)

    def _prepare_default_handlers(self, val_data, event_handlers):
        event_handlers = _check_event_handlers(event_handlers)
        added_default_handlers = []
        added_default_handlers.append(StoppingHandler(self.max_epoch, self.max_batch))
        if not any(isinstance(handler, GradientUpdateHandler) for handler in event_handlers):
            added_default_handlers.append(GradientUpdateHandler())
        if not any(isinstance(handler, MetricHandler) for handler in event_handlers):
            added_default_handlers.append(MetricHandler(metrics=self.train_metrics))
        if not any(isinstance(handler, ValidationHandler) for handler in event_handlers):
            if val_data:
                added_default_handlers.append(ValidationHandler(val_data=val_data, eval_fn=self.evaluate))
        if not any(isinstance(handler, LoggingHandler) for handler in event_handlers):
            added_default_handlers.append(LoggingHandler(metrics=self.train_metrics))
        mixing_handlers = event_handlers and added_default_handlers
        event_handlers.extend(added_default_handlers)
        if mixing_handlers:
            known = {id(h) for h in added_default_handlers}
            # make sure every user handler that watches metrics sees the estimator's metrics
            for h in event_handlers:
                if id(h) not in known and isinstance(h, (MetricHandler, LoggingHandler)) and not h.metrics:
                    h.metrics = self.train_metrics
        event_handlers.sort(key=lambda handler: getattr(handler, 'priority', 0))
        return event_handlers

    def _prepare_default_validation_handlers(self, event_handlers):
        event_handlers = _check_event_handlers(event_handlers)
        added = []
        if not any(isinstance(handler, MetricHandler) for handler in event_handlers):
            added.append(MetricHandler(metrics=self.val_metrics))
        if not any(isinstance(handler, LoggingHandler) for handler in event_handlers):
            added.append(LoggingHandler(metrics=self.val_metrics))
        event_handlers.extend(added)
        event_handlers.sort(key=lambda handler: getattr(handler, 'priority', 0))
        return event_handlers

    def _categorize_handlers(self, event_handlers):
        train_begin, epoch_begin, batch_begin, batch_end, epoch_end, train_end = [], [], [], [], [], []
        for handler in event_handlers:
            if isinstance(handler, TrainBegin):
                train_begin.append(handler)
            if isinstance(handler, EpochBegin):
                epoch_begin.append(handler)
            if isinstance(handler, BatchBegin):
                batch_begin.append(handler)
            if isinstance(handler, BatchEnd):
                batch_end.append(handler)
            if isinstance(handler, EpochEnd):
                epoch_end.append(handler)
            if isinstance(handler, TrainEnd):
                train_end.append(handler)
        return train_begin, epoch_begin, batch_begin, batch_end, epoch_end, train_end
