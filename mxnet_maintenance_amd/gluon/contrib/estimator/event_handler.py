"""Estimator event handlers (parity: gluon/contrib/estimator/event_handler.py).

Mix-in bases (TrainBegin, TrainEnd, EpochBegin, EpochEnd, BatchBegin,
BatchEnd) define the hook points; the concrete handlers implement stopping,
metric updates, periodic validation, logging, checkpointing, early stopping
and the gradient update itself.
"""
import logging
import os
import time
import warnings

import numpy as np

from ....metric import CompositeEvalMetric, EvalMetric
from ....metric import Loss as metric_loss

__all__ = ['TrainBegin', 'TrainEnd', 'EpochBegin', 'EpochEnd', 'BatchBegin', 'BatchEnd', 'StoppingHandler',
           'MetricHandler', 'ValidationHandler', 'LoggingHandler', 'CheckpointHandler', 'EarlyStoppingHandler',
           'GradientUpdateHandler']


class EventHandler:
    pass


def _check_event_handlers(handlers):
    if isinstance(handlers, EventHandler):
        handlers = [handlers]
    else:
        handlers = handlers or []
        if not all(isinstance(h, EventHandler) for h in handlers):
            raise ValueError('event_handlers must be an EventHandler or a list of EventHandlers, got: %s'
                             % handlers)
    return handlers


class TrainBegin(EventHandler):
    def train_begin(self, estimator, *args, **kwargs):
        pass


class TrainEnd(EventHandler):
    def train_end(self, estimator, *args, **kwargs):
        pass


class EpochBegin(EventHandler):
    def epoch_begin(self, estimator, *args, **kwargs):
        pass


class EpochEnd(EventHandler):
    def epoch_end(self, estimator, *args, **kwargs):
        return False


class BatchBegin(EventHandler):
    def batch_begin(self, estimator, *args, **kwargs):
        pass


class BatchEnd(EventHandler):
    def batch_end(self, estimator, *args, **kwargs):
        return False


class StoppingHandler(TrainBegin, BatchEnd, EpochEnd):
    """Stop after ``max_epoch`` epochs or ``max_batch`` batches."""

    def __init__(self, max_epoch=None, max_batch=None):
        self.max_epoch = max_epoch
        self.max_batch = max_batch
        self.current_batch = 0
        self.current_epoch = 0
        self.stop_training = False

    def train_begin(self, estimator, *args, **kwargs):
        self.max_epoch = estimator.max_epoch
        self.max_batch = estimator.max_batch
        self.current_batch = 0
        self.current_epoch = 0

    def batch_end(self, estimator, *args, **kwargs):
        self.current_batch += 1
        if self.current_batch == self.max_batch:
            self.stop_training = True
        return self.stop_training

    def epoch_end(self, estimator, *args, **kwargs):
        self.current_epoch += 1
        if self.current_epoch == self.max_epoch:
            self.stop_training = True
        return self.stop_training


class MetricHandler(EpochBegin, BatchEnd):
    """Reset metrics at epoch start, update them after every batch."""

    def __init__(self, metrics, priority=-1000):
        self.metrics = metrics or []
        self.priority = priority

    def epoch_begin(self, estimator, *args, **kwargs):
        for metric in self.metrics:
            metric.reset()

    def batch_end(self, estimator, *args, **kwargs):
        pred = kwargs['pred']
        label = kwargs['label']
        loss = kwargs['loss']
        for metric in self.metrics:
            if isinstance(metric, metric_loss):
                metric.update(0, loss)
            else:
                metric.update(label, pred)


class ValidationHandler(TrainBegin, BatchEnd, EpochEnd):
    """Run ``eval_fn(val_data)`` every ``epoch_period`` epochs and/or ``batch_period`` batches."""

    def __init__(self, val_data, eval_fn, epoch_period=1, batch_period=None, priority=-1000, event_handlers=None):
        self.val_data = val_data
        self.eval_fn = eval_fn
        self.epoch_period = epoch_period
        self.batch_period = batch_period
        self.current_batch = 0
        self.current_epoch = 0
        self.priority = priority
        self.event_handlers = event_handlers

    def train_begin(self, estimator, *args, **kwargs):
        self.current_batch = 0
        self.current_epoch = 0

    def batch_end(self, estimator, *args, **kwargs):
        self.current_batch += 1
        if self.batch_period and self.current_batch % self.batch_period == 0:
            self.eval_fn(val_data=self.val_data, event_handlers=self.event_handlers)

    def epoch_end(self, estimator, *args, **kwargs):
        self.current_epoch += 1
        if self.epoch_period and self.current_epoch % self.epoch_period == 0:
            self.eval_fn(val_data=self.val_data, event_handlers=self.event_handlers)


class LoggingHandler(TrainBegin, TrainEnd, EpochBegin, EpochEnd, BatchBegin, BatchEnd):
    """Log training progress (per epoch, or every ``log_interval`` batches)."""

    def __init__(self, log_interval='epoch', metrics=None, priority=np.inf):
        super().__init__()
        if not isinstance(log_interval, int) and log_interval != 'epoch':
            raise ValueError('log_interval must be either an integer or string \'epoch\'')
        self.metrics = metrics or []
        self.batch_index = 0
        self.current_epoch = 0
        self.processed_samples = 0
        self.priority = priority
        self.log_interval = log_interval
        self.log_interval_time = 0

    def train_begin(self, estimator, *args, **kwargs):
        self.train_start = time.time()
        trainer = estimator.trainer
        optimizer = trainer.optimizer.__class__.__name__
        lr = trainer.learning_rate
        estimator.logger.info('Training begin: using optimizer %s with current learning rate %.4f ', optimizer, lr)
        if estimator.max_epoch:
            estimator.logger.info('Train for %d epochs.', estimator.max_epoch)
        else:
            estimator.logger.info('Train for %d batches.', estimator.max_batch)
        self.current_epoch = 0
        self.batch_index = 0
        self.processed_samples = 0
        self.log_interval_time = 0

    def train_end(self, estimator, *args, **kwargs):
        train_time = time.time() - self.train_start
        msg = 'Train finished using total %ds with %d epochs. ' % (train_time, self.current_epoch)
        for metric in self.metrics:
            name, value = metric.get()
            msg += '%s: %.4f, ' % (name, value)
        estimator.logger.info(msg.rstrip(', '))

    def batch_begin(self, estimator, *args, **kwargs):
        if isinstance(self.log_interval, int):
            self.batch_start = time.time()

    def batch_end(self, estimator, *args, **kwargs):
        if isinstance(self.log_interval, int):
            batch_time = time.time() - self.batch_start
            msg = '[Epoch %d][Batch %d]' % (self.current_epoch, self.batch_index)
            self.processed_samples += kwargs['batch'][0].shape[0]
            msg += '[Samples %s] ' % self.processed_samples
            self.log_interval_time += batch_time
            if self.batch_index % self.log_interval == 0:
                msg += 'time/interval: %.3fs ' % self.log_interval_time
                self.log_interval_time = 0
                for metric in self.metrics:
                    name, value = metric.get()
                    msg += '%s: %.4f, ' % (name, value)
                estimator.logger.info(msg.rstrip(', '))
        self.batch_index += 1

    def epoch_begin(self, estimator, *args, **kwargs):
        if isinstance(self.log_interval, int) or self.log_interval == 'epoch':
            is_training = False
            for metric in self.metrics:
                if 'training' in metric.name:
                    is_training = True
            self.epoch_start = time.time()
            if is_training:
                estimator.logger.info('[Epoch %d] Begin, current learning rate: %.4f', self.current_epoch,
                                      estimator.trainer.learning_rate)
            else:
                estimator.logger.info('Validation Begin')

    def epoch_end(self, estimator, *args, **kwargs):
        if isinstance(self.log_interval, int) or self.log_interval == 'epoch':
            epoch_time = time.time() - self.epoch_start
            msg = '[Epoch %d] Finished in %.3fs, ' % (self.current_epoch, epoch_time)
            for monitor in self.metrics:
                name, value = monitor.get()
                msg += '%s: %.4f, ' % (name, value)
            estimator.logger.info(msg.rstrip(', '))
        self.current_epoch += 1
        self.batch_index = 0


class CheckpointHandler(TrainBegin, BatchEnd, EpochEnd):
    """Save parameters (and trainer states) periodically; keep the best by a monitored metric."""

    def __init__(self, model_dir, model_prefix='model', monitor=None, verbose=0, save_best=False, mode='auto',
                 epoch_period=1, batch_period=None, max_checkpoints=5, resume_from_checkpoint=False):
        self.monitor = monitor
        self.verbose = verbose
        if not os.path.exists(model_dir):
            os.makedirs(model_dir)
        self.model_dir = model_dir
        self.model_prefix = model_prefix
        self.save_best = save_best
        if self.save_best and not isinstance(self.monitor, EvalMetric):
            raise ValueError('To save best model only, please provide one of the metric objects from '
                             'estimator.train_metrics and estimator.val_metrics as monitor.')
        self.epoch_period = epoch_period
        self.batch_period = batch_period
        self.current_batch = 0
        self.current_epoch = 0
        self.max_checkpoints = max_checkpoints
        self.resume_from_checkpoint = resume_from_checkpoint
        self.saved_checkpoints = []
        if self.save_best:
            if mode not in ['auto', 'min', 'max']:
                warnings.warn('ModelCheckpoint mode %s is unknown, fallback to auto mode. CheckpointHandler will '
                              'use max mode for f1 and accuracy metric comparison and use min mode other wise'
                              % mode, RuntimeWarning)
                mode = 'auto'
            if mode == 'min':
                self.monitor_op = np.less
                self.best = np.inf
            elif mode == 'max':
                self.monitor_op = np.greater
                self.best = -np.inf
            elif 'acc' in self.monitor.get()[0].lower() or 'f1' in self.monitor.get()[0].lower():
                self.monitor_op = np.greater
                self.best = -np.inf
            else:
                self.monitor_op = np.less
                self.best = np.inf

    def train_begin(self, estimator, *args, **kwargs):
        self.current_epoch = 0
        self.current_batch = 0
        if self.save_best:
            self.best = np.inf if self.monitor_op == np.less else -np.inf
        if self.resume_from_checkpoint:
            self._resume_from_checkpoint(estimator)

    def batch_end(self, estimator, *args, **kwargs):
        if self.batch_period and (self.current_batch + 1) % self.batch_period == 0:
            self._save_checkpoint(estimator)
        self.current_batch += 1

    def epoch_end(self, estimator, *args, **kwargs):
        if self.epoch_period and (self.current_epoch + 1) % self.epoch_period == 0:
            self._save_checkpoint(estimator)
        self.current_epoch += 1

    def _save_checkpoint(self, estimator):
        if self.resume_from_checkpoint and self.current_epoch == 0 and self.current_batch == 0:
            return
        prefix = '%s-epoch%dbatch%d' % (self.model_prefix, self.current_epoch, self.current_batch)
        self._save_params_and_trainer(estimator, prefix)
        if self.verbose > 0:
            estimator.logger.info('[Epoch %d] CheckpointHandler: trained total %d batches, saving model at %s '
                                  'with prefix: %s', self.current_epoch, self.current_batch + 1, self.model_dir,
                                  prefix)
        if self.save_best:
            monitor_name, monitor_value = self.monitor.get()
            if np.isnan(monitor_value):
                warnings.warn(RuntimeWarning('%s is not updated, make sure you pass one of the metric objects '
                                             'from estimator.train_metrics and estimator.val_metrics as monitor.'
                                             % monitor_name))
            elif self.monitor_op(monitor_value, self.best):
                prefix = self.model_prefix + '-best'
                self._save_params_and_trainer(estimator, prefix)
                if self.verbose > 0:
                    estimator.logger.info('[Epoch %d] CheckpointHandler: %s improved from %0.5f to %0.5f, updating '
                                          'best model at %s with prefix: %s', self.current_epoch, monitor_name,
                                          self.best, monitor_value, self.model_dir, prefix)
                self.best = monitor_value

    def _save_params_and_trainer(self, estimator, file_prefix):
        param_file = os.path.join(self.model_dir, file_prefix + '.params')
        trainer_file = os.path.join(self.model_dir, file_prefix + '.states')
        estimator.net.save_parameters(param_file)
        estimator.trainer.save_states(trainer_file)
        if 'best' not in file_prefix:
            self.saved_checkpoints.append(file_prefix)
        if len(self.saved_checkpoints) > self.max_checkpoints:
            prefix = self.saved_checkpoints.pop(0)
            for fname in os.listdir(self.model_dir):
                if fname.startswith(prefix + '.'):
                    os.remove(os.path.join(self.model_dir, fname))

    def _resume_from_checkpoint(self, estimator):
        import re
        prefix = self.model_prefix + '-epoch'
        files = [f for f in os.listdir(self.model_dir) if f.startswith(prefix) and f.endswith('.params')]
        if not files:
            estimator.logger.info('CheckpointHandler: No checkpoint found, training from scratch for %d epochs'
                                  % (estimator.max_epoch or 0))
            return

        def key(f):
            m = re.match(r'.*epoch(\d+)batch(\d+)\.params', f)
            return (int(m.group(1)), int(m.group(2))) if m else (-1, -1)
        latest = max(files, key=key)
        epoch, batch = key(latest)
        estimator.net.load_parameters(os.path.join(self.model_dir, latest))
        states = os.path.join(self.model_dir, latest[:-len('.params')] + '.states')
        if os.path.exists(states):
            estimator.trainer.load_states(states)
        self.current_epoch = epoch + 1 if self.epoch_period else epoch
        self.current_batch = batch
        for handler in getattr(estimator, '_handlers', []):
            if isinstance(handler, StoppingHandler):
                handler.current_epoch = self.current_epoch
                handler.current_batch = self.current_batch
        estimator.logger.info('CheckpointHandler: resumed from %s', latest)


class EarlyStoppingHandler(TrainBegin, EpochEnd, TrainEnd):
    """Stop when the monitored metric has not improved by ``min_delta`` for ``patience`` epochs."""

    def __init__(self, monitor, min_delta=0, patience=0, mode='auto', baseline=None):
        super().__init__()
        if not isinstance(monitor, EvalMetric):
            raise ValueError('Please provide one of the metric objects from estimator.train_metrics and '
                             'estimator.val_metrics as monitor.')
        if isinstance(monitor, CompositeEvalMetric):
            raise ValueError('CompositeEvalMetric is not supported for EarlyStoppingHandler, please specify a '
                             'simple metric instead.')
        self.monitor = monitor
        self.baseline = baseline
        self.patience = patience
        self.min_delta = min_delta
        self.wait = 0
        self.stopped_epoch = 0
        self.current_epoch = 0
        self.stop_training = False
        if mode not in ['auto', 'min', 'max']:
            warnings.warn('EarlyStopping mode %s is unknown, fallback to auto mode.' % mode, RuntimeWarning)
            mode = 'auto'
        if mode == 'min':
            self.monitor_op = np.less
        elif mode == 'max':
            self.monitor_op = np.greater
        elif 'acc' in self.monitor.get()[0].lower() or 'f1' in self.monitor.get()[0].lower():
            self.monitor_op = np.greater
        else:
            self.monitor_op = np.less
        if self.monitor_op == np.greater:
            self.min_delta *= 1
        else:
            self.min_delta *= -1

    def train_begin(self, estimator, *args, **kwargs):
        self.wait = 0
        self.stopped_epoch = 0
        self.current_epoch = 0
        self.stop_training = False
        if self.baseline is not None:
            self.best = self.baseline
        else:
            self.best = np.inf if self.monitor_op == np.less else -np.inf

    def epoch_end(self, estimator, *args, **kwargs):
        monitor_name, monitor_value = self.monitor.get()
        if np.isnan(monitor_value):
            warnings.warn(RuntimeWarning('%s is not updated, make sure you pass one of the metric objects from '
                                         'estimator.train_metrics and estimator.val_metrics as monitor.'
                                         % monitor_name))
        else:
            if self.monitor_op(monitor_value - self.min_delta, self.best):
                self.best = monitor_value
                self.wait = 0
            else:
                self.wait += 1
                if self.wait >= self.patience:
                    self.stopped_epoch = self.current_epoch
                    self.stop_training = True
        self.current_epoch += 1
        return self.stop_training

    def train_end(self, estimator, *args, **kwargs):
        if self.stopped_epoch > 0:
            estimator.logger.info('[Epoch %d] EarlyStoppingHanlder: early stopping due to %s not improving'
                                  % (self.stopped_epoch, self.monitor.get()[0]))


class GradientUpdateHandler(BatchEnd):
    """Apply ``trainer.step(batch_size)`` after each batch (priority ordering: before metric/logging)."""

    def __init__(self, priority=-2000):
        self.priority = priority

    def batch_end(self, estimator, *args, **kwargs):
        loss = kwargs['loss']
        batch_size = 0
        if not isinstance(loss, list):
            loss = [loss]
        for l in loss:
            batch_size += l.shape[0]
        estimator.trainer.step(batch_size)
