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
        self.trained_epoch = self.trained_batch = -1
        if self.save_best:
            self.best = self._better.worst()
        if self.resume_from_checkpoint:
            by_batch = bool(estimator.max_batch)
            if (by_batch and (not self.batch_period or self.epoch_period)) or \
                    (not by_batch and (not self.epoch_period or self.batch_period)):
                raise AssertionError('To use resume from checkpoint, you must only specify the same type of period '
                                     'you used for training (epoch_period for epochs, batch_period for batches).')
            self._resume(estimator)

    def batch_end(self, estimator, *args, **kwargs):
        if self.current_batch == 0:
            self._save_symbol(estimator)
        if self.batch_period and (self.current_batch + 1) % self.batch_period == 0:
            self._checkpoint_now(estimator)
        self.current_batch += 1

    def epoch_end(self, estimator, *args, **kwargs):
        if self.epoch_period and (self.current_epoch + 1) % self.epoch_period == 0:
            self._checkpoint_now(estimator)
        self.current_epoch += 1

    def _numbers(self, estimator):
        """(epoch, batch) the checkpoint is named after: continuing the resumed run's count."""
        if self.trained_epoch < 0:
            return self.current_epoch, self.current_batch
        extra = 0 if estimator.max_epoch else 1
        return self.current_epoch + self.trained_epoch + 1, self.current_batch + self.trained_batch + extra

    def _checkpoint_now(self, estimator):
        epoch, batch = self._numbers(estimator)
        prefix = '%s-epoch%dbatch%d' % (self.model_prefix, epoch, batch)
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

    def _save_symbol(self, estimator):
        """``<prefix>-symbol.json`` of a hybridized network (its cached graph), once per fit."""
        graph = getattr(estimator.net, '_cached_graph', None)
        if graph:
            graph[1].save(self._path(self.model_prefix + '-symbol', '.json'))
        else:
            estimator.logger.info('Model architecture (symbol file) is not saved: hybridize a HybridBlock model '
                                  'before passing it to the Estimator to save it as %s-symbol.json', self.model_prefix)

    def _write(self, estimator, file_prefix):
        estimator.net.save_parameters(self._path(file_prefix, '.params'))
        estimator.trainer.save_states(self._path(file_prefix, '.states'))
        if 'best' in file_prefix:
            return
        self.saved_checkpoints.append(file_prefix)
        while len(self.saved_checkpoints) > self.max_checkpoints:
            old = self.saved_checkpoints.pop(0)
            for fname in os.listdir(self.model_dir):
                if fname.startswith(old):
                    os.unlink(os.path.join(self.model_dir, fname))

    def _latest(self, head, tail):
        """Largest integer between ``head`` and ``tail`` in the model directory's file names, or -1."""
        best = -1
        for fname in os.listdir(self.model_dir):
            if fname.startswith(head) and tail in fname[len(head):]:
                num = fname[len(head):].split(tail, 1)[0]
                if num.isdigit():
                    best = max(best, int(num))
        return best

    def _resume(self, estimator):
        head = self.model_prefix + '-epoch'
        self.trained_epoch = self._latest(head, 'batch')
        if self.trained_epoch < 0:
            estimator.logger.info('CheckpointHandler: No checkpoint found, training from scratch for %s'
                                  % ('%d batches' % estimator.max_batch if estimator.max_batch else
                                     '%d epochs' % (estimator.max_epoch or 0)))
            return
        self.trained_batch = self._latest('%s%d' % (head, self.trained_epoch) + 'batch', '.params')
        if estimator.max_epoch:
            if self.trained_epoch >= estimator.max_epoch - 1:
                raise ValueError('Found checkpoint with maximum number of epoch %d reached, please specify '
                                 'resume_from_checkpoint=False to train from scratch.' % estimator.max_epoch)
            estimator.max_epoch -= self.trained_epoch + 1
        if estimator.max_batch:
            if self.trained_batch >= estimator.max_batch - 1:
                raise ValueError('Found checkpoint with maximum number of batch %d reached, please specify '
                                 'resume_from_checkpoint=False to train from scratch.' % self.trained_batch)
            estimator.max_batch -= self.trained_batch + 1
        stem = '%s-epoch%dbatch%d' % (self.model_prefix, self.trained_epoch, self.trained_batch)
        params, states = self._path(stem, '.params'), self._path(stem, '.states')
        if not (os.path.exists(params) and os.path.exists(states)):
            raise AssertionError('Failed to load checkpoint %s (.params / .states missing)' % stem)
        estimator.net.load_parameters(params, ctx=estimator.context)
        estimator.trainer.load_states(states)
        estimator.logger.warning('CheckpointHandler: Checkpoint resumed from epoch %d batch %d, continue to train '
                                 'for %s', self.trained_epoch, self.trained_batch,
                                 '%d epochs' % estimator.max_epoch if estimator.max_epoch else
                                 '%d batches' % estimator.max_batch)


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
