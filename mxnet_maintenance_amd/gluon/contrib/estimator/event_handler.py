"""Estimator event handlers (API parity: gluon/contrib/estimator/event_handler.py).

Hook mix-ins (``TrainBegin``, ``TrainEnd``, ``EpochBegin``, ``EpochEnd``,
``BatchBegin``, ``BatchEnd``) mark which events a handler receives; the
Estimator's event bus calls ``handler.<event>(estimator, **kw)`` on every
handler that derives from the matching mix-in, in ``priority`` order.
``batch_end`` / ``epoch_end`` return True to request that training stop.

Shared helpers: ``_Improvement`` (min / max / auto comparison of a monitored
metric, used by checkpointing and early stopping) and ``_metric_text`` (the
"name: value" strings of the logging handler).
"""
import logging
import os
import re
import time
import warnings

import numpy as np

from ....metric import CompositeEvalMetric, EvalMetric
from ....metric import Loss as metric_loss

__all__ = ['TrainBegin', 'TrainEnd', 'EpochBegin', 'EpochEnd', 'BatchBegin', 'BatchEnd', 'StoppingHandler',
           'MetricHandler', 'ValidationHandler', 'LoggingHandler', 'CheckpointHandler', 'EarlyStoppingHandler',
           'GradientUpdateHandler']

_EVENTS = ('train_begin', 'epoch_begin', 'batch_begin', 'batch_end', 'epoch_end', 'train_end')


class EventHandler:
    """Root of all handlers."""


def _check_event_handlers(handlers):
    if isinstance(handlers, EventHandler):
        return [handlers]
    handlers = list(handlers or [])
    bad = [h for h in handlers if not isinstance(h, EventHandler)]
    if bad:
        raise ValueError('event_handlers must be EventHandler instances, got: %s' % bad)
    return handlers


def _hook(event, result=None):
    def method(self, estimator, *args, **kwargs):
        return result
    method.__name__ = event
    return method


class TrainBegin(EventHandler):
    train_begin = _hook('train_begin')


class TrainEnd(EventHandler):
    train_end = _hook('train_end')


class EpochBegin(EventHandler):
    epoch_begin = _hook('epoch_begin')


class EpochEnd(EventHandler):
    epoch_end = _hook('epoch_end', False)


class BatchBegin(EventHandler):
    batch_begin = _hook('batch_begin')


class BatchEnd(EventHandler):
    batch_end = _hook('batch_end', False)


_MIXIN = {'train_begin': TrainBegin, 'epoch_begin': EpochBegin, 'batch_begin': BatchBegin,
          'batch_end': BatchEnd, 'epoch_end': EpochEnd, 'train_end': TrainEnd}


def _metric_text(metrics):
    return ', '.join('%s: %.4f' % m.get() for m in metrics)


class _Improvement:
    """Is a new value of ``metric`` better than the best so far?  ``mode`` 'min' / 'max', or 'auto'
    (higher is better for accuracy / f1 names, lower otherwise)."""

    def __init__(self, metric, mode, what):
        if mode not in ('auto', 'min', 'max'):
            warnings.warn('%s mode %s is unknown, fallback to auto mode.' % (what, mode), RuntimeWarning)
            mode = 'auto'
        if mode == 'auto':
            name = metric.get()[0].lower()
            mode = 'max' if ('acc' in name or 'f1' in name) else 'min'
        self.maximize = mode == 'max'
        self.monitor_op = np.greater if self.maximize else np.less

    def worst(self):
        return -np.inf if self.maximize else np.inf


def _monitor_value(metric):
    name, value = metric.get()
    if np.isnan(value):
        warnings.warn(RuntimeWarning('%s is not updated, make sure you pass one of the metric objects from '
                                     'estimator.train_metrics and estimator.val_metrics as monitor.' % name))
        return name, None
    return name, value


class StoppingHandler(TrainBegin, BatchEnd, EpochEnd):
    """Request a stop once ``max_batch`` batches or ``max_epoch`` epochs have run."""

    def __init__(self, max_epoch=None, max_batch=None):
        self.max_epoch, self.max_batch = max_epoch, max_batch
        self.current_epoch = self.current_batch = 0
        self.stop_training = False

    def train_begin(self, estimator, *args, **kwargs):
        self.max_epoch, self.max_batch = estimator.max_epoch, estimator.max_batch
        self.current_epoch = self.current_batch = 0

    def batch_end(self, estimator, *args, **kwargs):
        self.current_batch += 1
        self.stop_training |= self.current_batch == self.max_batch
        return self.stop_training

    def epoch_end(self, estimator, *args, **kwargs):
        self.current_epoch += 1
        self.stop_training |= self.current_epoch == self.max_epoch
        return self.stop_training


class MetricHandler(EpochBegin, BatchEnd):
    """Reset the metrics each epoch and feed them every batch (loss metrics get the loss)."""

    def __init__(self, metrics, priority=-1000):
        self.metrics = metrics or []
        self.priority = priority

    def epoch_begin(self, estimator, *args, **kwargs):
        for m in self.metrics:
            m.reset()

    def batch_end(self, estimator, *args, **kwargs):
        for m in self.metrics:
            if isinstance(m, metric_loss):
                m.update(0, kwargs['loss'])
            else:
                m.update(kwargs['label'], kwargs['pred'])


class ValidationHandler(TrainBegin, BatchEnd, EpochEnd):
    """Call ``eval_fn(val_data=..., event_handlers=...)`` every ``epoch_period`` epochs and / or
    every ``batch_period`` batches."""

    def __init__(self, val_data, eval_fn, epoch_period=1, batch_period=None, priority=-1000, event_handlers=None):
        self.val_data = val_data
        self.eval_fn = eval_fn
        self.epoch_period, self.batch_period = epoch_period, batch_period
        self.priority = priority
        self.event_handlers = event_handlers
        self.current_epoch = self.current_batch = 0

    def _run(self):
        self.eval_fn(val_data=self.val_data, event_handlers=self.event_handlers)

    def train_begin(self, estimator, *args, **kwargs):
        self.current_epoch = self.current_batch = 0

    def batch_end(self, estimator, *args, **kwargs):
        self.current_batch += 1
        if self.batch_period and not self.current_batch % self.batch_period:
            self._run()

    def epoch_end(self, estimator, *args, **kwargs):
        self.current_epoch += 1
        if self.epoch_period and not self.current_epoch % self.epoch_period:
            self._run()


class LoggingHandler(TrainBegin, TrainEnd, EpochBegin, EpochEnd, BatchBegin, BatchEnd):
    """Log progress at epoch granularity (``log_interval='epoch'``) or every N batches."""

    def __init__(self, log_interval='epoch', metrics=None, priority=np.inf):
        if log_interval != 'epoch' and not isinstance(log_interval, int):
            raise ValueError("log_interval must be either an integer or string 'epoch'")
        self.log_interval = log_interval
        self.metrics = metrics or []
        self.priority = priority
        self.current_epoch = self.batch_index = self.processed_samples = 0
        self.log_interval_time = 0.0
        self._t_train = self._t_epoch = self._t_batch = None

    @property
    def _per_batch(self):
        return isinstance(self.log_interval, int)

    def train_begin(self, estimator, *args, **kwargs):
        self._t_train = time.time()
        tr = estimator.trainer
        estimator.logger.info('Training begin: using optimizer %s with current learning rate %.4f ',
                              type(tr.optimizer).__name__, tr.learning_rate)
        if estimator.max_epoch:
            estimator.logger.info('Train for %d epochs.', estimator.max_epoch)
        else:
            estimator.logger.info('Train for %d batches.', estimator.max_batch)
        self.current_epoch = self.batch_index = self.processed_samples = 0
        self.log_interval_time = 0.0

    def train_end(self, estimator, *args, **kwargs):
        text = _metric_text(self.metrics)
        estimator.logger.info('Train finished using total %ds with %d epochs. %s', time.time() - self._t_train,
                              self.current_epoch, text)

    def batch_begin(self, estimator, *args, **kwargs):
        if self._per_batch:
            self._t_batch = time.time()

    def batch_end(self, estimator, *args, **kwargs):
        if self._per_batch:
            self.log_interval_time += time.time() - self._t_batch
            self.processed_samples += kwargs['batch'][0].shape[0]
            if self.batch_index % self.log_interval == 0:
                estimator.logger.info('[Epoch %d][Batch %d][Samples %s] time/interval: %.3fs %s', self.current_epoch,
                                      self.batch_index, self.processed_samples, self.log_interval_time,
                                      _metric_text(self.metrics))
                self.log_interval_time = 0.0
        self.batch_index += 1

    def epoch_begin(self, estimator, *args, **kwargs):
        self._t_epoch = time.time()
        if any('training' in m.name for m in self.metrics):
            estimator.logger.info('[Epoch %d] Begin, current learning rate: %.4f', self.current_epoch,
                                  estimator.trainer.learning_rate)
        else:
            estimator.logger.info('Validation Begin')

    def epoch_end(self, estimator, *args, **kwargs):
        estimator.logger.info('[Epoch %d] Finished in %.3fs, %s', self.current_epoch, time.time() - self._t_epoch,
                              _metric_text(self.metrics))
        self.current_epoch += 1
        self.batch_index = 0


def _due(period, count):
    """True when the (count+1)-th event completes a ``period`` (a falsy period never fires)."""
    return bool(period) and (count + 1) % period == 0


class CheckpointHandler(TrainBegin, BatchEnd, EpochEnd):
    """Save ``<prefix>-epoch<E>batch<B>.params/.states`` periodically (keeping the newest
    ``max_checkpoints``), optionally ``<prefix>-best`` by a monitored metric, and resume from the
    newest checkpoint on request."""

    _NAME = re.compile(r'.*epoch(\d+)batch(\d+)\.params$')

    def __init__(self, model_dir, model_prefix='model', monitor=None, verbose=0, save_best=False, mode='auto',
                 epoch_period=1, batch_period=None, max_checkpoints=5, resume_from_checkpoint=False):
        if save_best and not isinstance(monitor, EvalMetric):
            raise ValueError('To save best model only, please provide one of the metric objects from '
                             'estimator.train_metrics and estimator.val_metrics as monitor.')
        os.makedirs(model_dir, exist_ok=True)
        self.model_dir, self.model_prefix = model_dir, model_prefix
        self.monitor, self.verbose, self.save_best = monitor, verbose, save_best
        self.epoch_period, self.batch_period = epoch_period, batch_period
        self.max_checkpoints = max_checkpoints
        self.resume_from_checkpoint = resume_from_checkpoint
        self.saved_checkpoints = []
        self.current_epoch = self.current_batch = 0
        if save_best:
            self._better = _Improvement(monitor, mode, 'ModelCheckpoint')
            self.monitor_op = self._better.monitor_op
            self.best = self._better.worst()

    def _path(self, prefix, ext):
        return os.path.join(self.model_dir, prefix + ext)

    def train_begin(self, estimator, *args, **kwargs):
        self.current_epoch = self.current_batch = 0
        if self.save_best:
            self.best = self._better.worst()
        if self.resume_from_checkpoint:
            self._restore_latest(estimator)

    def batch_end(self, estimator, *args, **kwargs):
        if _due(self.batch_period, self.current_batch):
            self._checkpoint_now(estimator)
        self.current_batch += 1

    def epoch_end(self, estimator, *args, **kwargs):
        if _due(self.epoch_period, self.current_epoch):
            self._checkpoint_now(estimator)
        self.current_epoch += 1

    def _checkpoint_now(self, estimator):
        if self.resume_from_checkpoint and self.current_epoch == 0 and self.current_batch == 0:
            return
        prefix = '%s-epoch%dbatch%d' % (self.model_prefix, self.current_epoch, self.current_batch)
        self._write(estimator, prefix)
        if self.verbose > 0:
            estimator.logger.info('[Epoch %d] CheckpointHandler: trained total %d batches, saving model at %s with '
                                  'prefix: %s', self.current_epoch, self.current_batch + 1, self.model_dir, prefix)
        if not self.save_best:
            return
        name, value = _monitor_value(self.monitor)
        if value is not None and self.monitor_op(value, self.best):
            best_prefix = self.model_prefix + '-best'
            self._write(estimator, best_prefix)
            if self.verbose > 0:
                estimator.logger.info('[Epoch %d] CheckpointHandler: %s improved from %0.5f to %0.5f, updating best '
                                      'model at %s with prefix: %s', self.current_epoch, name, self.best, value,
                                      self.model_dir, best_prefix)
            self.best = value

    def _write(self, estimator, file_prefix):
        estimator.net.save_parameters(self._path(file_prefix, '.params'))
        estimator.trainer.save_states(self._path(file_prefix, '.states'))
        if 'best' in file_prefix:
            return
        self.saved_checkpoints.append(file_prefix)
        while len(self.saved_checkpoints) > self.max_checkpoints:
            old = self.saved_checkpoints.pop(0)
            for ext in ('.params', '.states'):
                stale = self._path(old, ext)
                if os.path.exists(stale):
                    os.unlink(stale)

    def _restore_latest(self, estimator):
        found = []
        head = self.model_prefix + '-epoch'
        for fname in sorted(os.listdir(self.model_dir)):
            m = self._NAME.match(fname)
            if m and fname.startswith(head):
                found.append(((int(m.group(1)), int(m.group(2))), fname))
        if not found:
            estimator.logger.info('CheckpointHandler: No checkpoint found, training from scratch for %d epochs'
                                  % (estimator.max_epoch or 0))
            return
        (epoch, batch), latest = max(found)
        estimator.net.load_parameters(os.path.join(self.model_dir, latest))
        states = os.path.join(self.model_dir, latest[:-len('.params')] + '.states')
        if os.path.exists(states):
            estimator.trainer.load_states(states)
        self.current_epoch = epoch + 1 if self.epoch_period else epoch
        self.current_batch = batch
        for h in getattr(estimator, '_handlers', []):
            if isinstance(h, StoppingHandler):
                h.current_epoch, h.current_batch = self.current_epoch, self.current_batch
        estimator.logger.info('CheckpointHandler: resumed from %s', latest)


class EarlyStoppingHandler(TrainBegin, EpochEnd, TrainEnd):
    """Stop when the monitored metric has not improved by ``min_delta`` for ``patience`` epochs."""

    def __init__(self, monitor, min_delta=0, patience=0, mode='auto', baseline=None):
        if not isinstance(monitor, EvalMetric):
            raise ValueError('Please provide one of the metric objects from estimator.train_metrics and '
                             'estimator.val_metrics as monitor.')
        if isinstance(monitor, CompositeEvalMetric):
            raise ValueError('CompositeEvalMetric is not supported for EarlyStoppingHandler, please specify a '
                             'simple metric instead.')
        self.monitor, self.baseline, self.patience = monitor, baseline, patience
        self._better = _Improvement(monitor, mode, 'EarlyStopping')
        self.monitor_op = self._better.monitor_op
        # the required margin points in the direction of improvement
        self.min_delta = min_delta if self._better.maximize else -min_delta
        self.wait = self.stopped_epoch = self.current_epoch = 0
        self.stop_training = False
        self.best = None

    def train_begin(self, estimator, *args, **kwargs):
        self.wait = self.stopped_epoch = self.current_epoch = 0
        self.stop_training = False
        self.best = self.baseline if self.baseline is not None else self._better.worst()

    def epoch_end(self, estimator, *args, **kwargs):
        _name, value = _monitor_value(self.monitor)
        if value is not None:
            if self.monitor_op(value - self.min_delta, self.best):
                self.best, self.wait = value, 0
            else:
                self.wait += 1
                if self.wait >= self.patience:
                    self.stopped_epoch, self.stop_training = self.current_epoch, True
        self.current_epoch += 1
        return self.stop_training

    def train_end(self, estimator, *args, **kwargs):
        if self.stopped_epoch > 0:
            estimator.logger.info('[Epoch %d] EarlyStoppingHanlder: early stopping due to %s not improving'
                                  % (self.stopped_epoch, self.monitor.get()[0]))


class GradientUpdateHandler(BatchEnd):
    """``trainer.step(batch size)`` after every batch; runs before the metric / logging handlers."""

    def __init__(self, priority=-2000):
        self.priority = priority

    def batch_end(self, estimator, *args, **kwargs):
        losses = kwargs['loss'] if isinstance(kwargs['loss'], list) else [kwargs['loss']]
        estimator.trainer.step(sum(l.shape[0] for l in losses))
