"""Estimator: a handler-driven training loop for Gluon networks.

API parity: gluon/contrib/estimator/estimator.py (``Estimator(net, loss,
train_metrics, val_metrics, initializer, trainer, context, val_net,
val_loss, batch_processor)``, ``fit``, ``evaluate``, ``train_metrics``,
``val_metrics``).

The loop itself only produces events: train_begin -> (epoch_begin ->
(batch_begin -> batch step -> batch_end)* -> epoch_end)* -> train_end.  All
behaviour (gradient update, metrics, logging, validation, stopping) lives in
event handlers, dispatched by ``_EventBus`` in ascending ``priority``.
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
from .batch_processor import BatchProcessor
from .event_handler import (StoppingHandler, MetricHandler, ValidationHandler, LoggingHandler,
                            GradientUpdateHandler, _check_event_handlers, _EVENTS, _MIXIN)

__all__ = ['Estimator']


def _check_metrics(metrics):
    """Flatten a metric / composite / list of metrics into a list of EvalMetric."""
    if isinstance(metrics, metric_mod.CompositeEvalMetric):
        return [leaf for child in metrics.metrics for leaf in _check_metrics(child)]
    if isinstance(metrics, EvalMetric):
        return [metrics]
    metrics = list(metrics or [])
    if any(not isinstance(m, EvalMetric) for m in metrics):
        raise ValueError('metrics must be a Metric or a list of Metric, refer to mxnet.metric.EvalMetric: %s'
                         % metrics)
    return metrics


def _require_loader(data):
    """The Estimator consumes Gluon DataLoaders only (reference estimator.py fit / evaluate): a
    DataIter yields DataBatch objects and a bare NDArray has no (data, label) structure."""
    from ...data import DataLoader
    if not isinstance(data, DataLoader):
        raise ValueError('Estimator only support input as Gluon DataLoader. Alternatively, you can transform '
                         'your DataIter or any NDArray into Gluon DataLoader. Refer to gluon.data.DataLoader')


class _EventBus:
    """Handlers sorted by priority, grouped per event by their hook mix-ins."""

    def __init__(self, handlers):
        self.handlers = sorted(handlers, key=lambda h: getattr(h, 'priority', 0))
        self._by_event = {ev: [h for h in self.handlers if isinstance(h, _MIXIN[ev])] for ev in _EVENTS}

    def fire(self, event, estimator, **kwargs):
        """Call ``event`` on its subscribers; True if any asked to stop (all are still called)."""
        results = [getattr(h, event)(estimator, **kwargs) for h in self._by_event[event]]
        return any(results)


class Estimator:
    logger = None

    def __init__(self, net, loss, train_metrics=None, val_metrics=None, initializer=None, trainer=None,
                 context=None, val_net=None, val_loss=None, batch_processor=None):
        self.net = net
        self.loss = self._check_loss(loss)
        self.val_loss = self._check_loss(val_loss) if val_loss is not None else self.loss
        self.val_net = val_net if val_net is not None else net
        self._train_metrics = self._training_metrics(_check_metrics(train_metrics))
        self._val_metrics = self._validation_metrics(_check_metrics(val_metrics))
        self.logger = logging.Logger(name='Estimator', level=logging.INFO)
        self.logger.addHandler(logging.StreamHandler(sys.stdout))
        self.context = self._check_context(context)
        self._initialize(initializer)
        self.trainer = self._check_trainer(trainer)
        self.batch_processor = batch_processor if batch_processor is not None else BatchProcessor()
        self.max_epoch = self.max_batch = None
        self.batch_axis = 0
        self._handlers = []

    # ---------------------------------------------------------------- set-up checks
    @staticmethod
    def _check_loss(loss):
        if not isinstance(loss, gluon_loss):
            raise ValueError('loss must be a Loss, refer to gluon.loss.Loss:{}'.format(loss))
        return loss

    @staticmethod
    def _check_context(context):
        if not context:
            return [gpu(i) for i in range(num_gpus())] or [cpu()]
        ctxs = [context] if isinstance(context, Context) else context
        if not isinstance(ctxs, list) or any(not isinstance(c, Context) for c in ctxs):
            raise ValueError('context must be a Context or a list of Context, refer to mxnet.Context: {}'
                             .format(context))
        gpus = [gpu(i) for i in range(num_gpus())]
        for c in ctxs:
            if c.device_type != 'cpu' and c not in gpus:
                raise AssertionError('%s is not available, please make sure your context is in one of: mx.cpu(), %s'
                                     % (c, ', '.join(str(g) for g in gpus)))
        return ctxs

    def _is_initialized(self):
        for p in self.net.collect_params().values():
            try:
                p.list_ctx()
            except Exception:   # pylint: disable=broad-except
                return False
        return True

    def _initialize(self, initializer):
        if not self._is_initialized():
            from ....initializer import Uniform
            self.net.initialize(init=initializer or Uniform(), ctx=self.context)
        elif initializer is not None:
            warnings.warn("Network already fully initialized, skipping initialization. You don't need to pass "
                          'initializer if you already initialized your net. You can use '
                          'net.initialize(force_reinit=True) to re-initialize.')

    def _check_trainer(self, trainer):
        if not trainer:
            warnings.warn('No trainer specified, default SGD optimizer with learning rate 0.001 is used.')
            return Trainer(self.net.collect_params(), 'sgd', {'learning_rate': 0.001})
        if not isinstance(trainer, Trainer):
            raise ValueError('Trainer must be a Gluon Trainer instance, refer to gluon.Trainer:{}'.format(trainer))
        return trainer

    def _training_metrics(self, metrics):
        """User metrics (Accuracy for a softmax-CE loss by default) plus the loss, prefixed 'training'."""
        if not metrics and isinstance(self.loss, SoftmaxCrossEntropyLoss):
            metrics = [Accuracy()]
        metrics = metrics + [metric_loss(self.loss.name.rstrip('1234567890'))]
        for m in metrics:
            m.name = 'training ' + m.name
        return metrics

    def _validation_metrics(self, metrics):
        metrics = metrics or [copy.deepcopy(m) for m in self._train_metrics]
        for m in metrics:
            if 'training' in m.name:
                m.name = m.name.replace('training', 'validation')
            elif 'validation' not in m.name:
                m.name = 'validation ' + m.name
        return metrics

    @property
    def train_metrics(self):
        return self._train_metrics

    @property
    def val_metrics(self):
        return self._val_metrics

    # ---------------------------------------------------------------- handler sets
    def _with_defaults(self, handlers, defaults):
        """User handlers plus each default whose type the user did not supply."""
        handlers = _check_event_handlers(handlers)
        added = [d for d in defaults if not any(isinstance(h, type(d)) for h in handlers)]
        if handlers:
            # user metric / logging handlers without metrics watch the estimator's
            for h in handlers:
                if isinstance(h, (MetricHandler, LoggingHandler)) and not h.metrics:
                    h.metrics = self.train_metrics
        return handlers + added

    def _prepare_default_handlers(self, val_data, event_handlers):
        defaults = [GradientUpdateHandler(), MetricHandler(metrics=self.train_metrics)]
        if val_data:
            defaults.append(ValidationHandler(val_data=val_data, eval_fn=self.evaluate))
        defaults.append(LoggingHandler(metrics=self.train_metrics))
        user = _check_event_handlers(event_handlers)
        handlers = self._with_defaults(event_handlers, defaults)
        handlers.append(StoppingHandler(self.max_epoch, self.max_batch))     # always one of ours
        if user:
            # user handlers next to default ones must watch the estimator's own metric objects
            known = set(id(m) for m in self.train_metrics + self.val_metrics)
            for h in handlers:
                for attr in dir(h):
                    if 'metric' not in attr:
                        continue
                    ref = getattr(h, attr, None)
                    for m in (ref if isinstance(ref, list) else [ref] if ref else []):
                        if hasattr(m, 'update') and id(m) not in known:
                            raise ValueError('Event handler %s refers to a metric instance %s outside of the '
                                             'estimator\'s train_metrics / val_metrics' % (type(h).__name__, m))
        return sorted(handlers, key=lambda h: getattr(h, 'priority', 0))

    def _prepare_default_validation_handlers(self, event_handlers):
        handlers = _check_event_handlers(event_handlers)
        defaults = [MetricHandler(metrics=self.val_metrics), LoggingHandler(metrics=self.val_metrics)]
        handlers = handlers + [d for d in defaults if not any(isinstance(h, type(d)) for h in handlers)]
        return sorted(handlers, key=lambda h: getattr(h, 'priority', 0))

    def _categorize_handlers(self, event_handlers):
        bus = _EventBus(event_handlers)
        return tuple(bus._by_event[ev] for ev in _EVENTS)

    # ---------------------------------------------------------------- loops
    def evaluate(self, val_data, batch_axis=0, event_handlers=None):
        """One pass over ``val_data`` updating ``val_metrics`` (through the validation handlers)."""
        _require_loader(val_data)
        for m in self.val_metrics:
            m.reset()
        bus = _EventBus(self._prepare_default_validation_handlers(event_handlers))
        bus.fire('epoch_begin', self)
        for batch in val_data:
            bus.fire('batch_begin', self, batch=batch)
            _, label, pred, loss = self.batch_processor.evaluate_batch(self, batch, batch_axis)
            bus.fire('batch_end', self, batch=batch, pred=pred, label=label, loss=loss)
        bus.fire('epoch_end', self)

    def fit(self, train_data, val_data=None, epochs=None, event_handlers=None, batches=None, batch_axis=0):
        """Train for ``epochs`` epochs or ``batches`` batches (exactly one of them)."""
        _require_loader(train_data)
        if bool(epochs) == bool(batches):
            raise ValueError('Please specify either epochs or batches.' if not epochs else
                             'Only one of epochs and batches can be specified.')
        self.max_epoch, self.max_batch, self.batch_axis = epochs, batches, batch_axis
        self._handlers = self._prepare_default_handlers(val_data, event_handlers)
        bus = _EventBus(self._handlers)
        bus.fire('train_begin', self)
        stop = False
        while not stop:
            bus.fire('epoch_begin', self)
            for batch in train_data:
                bus.fire('batch_begin', self, batch=batch)
                _, label, pred, loss = self.batch_processor.fit_batch(self, batch, batch_axis)
                if bus.fire('batch_end', self, batch=batch, pred=pred, label=label, loss=loss):
                    stop = True
                    break
            stop = bus.fire('epoch_end', self) or stop
        bus.fire('train_end', self)
