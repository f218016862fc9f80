"""Training-loop callbacks (API parity: python/mxnet/callback.py).

Two callback shapes exist, as in the reference:

* batch-end: ``cb(param)`` with ``param`` a ``BatchEndParam(epoch, nbatch,
  eval_metric, locals)``;
* epoch-end: ``cb(epoch, symbol, arg_params, aux_params)``.

Periodic behaviour ("every N epochs / batches") is factored into ``_every``.
"""
import logging
import math
import time

__all__ = ['module_checkpoint', 'do_checkpoint', 'log_train_metric', 'Speedometer', 'ProgressBar',
           'LogValidationMetricsCallback']


def _every(period):
    """Predicate on a 0-based epoch index: true on epochs period-1, 2*period-1, ..."""
    period = max(1, int(period))
    return lambda idx: (idx + 1) % period == 0


def module_checkpoint(mod, prefix, period=1, save_optimizer_states=False):
    """Epoch-end callback: ``mod.save_checkpoint(prefix, epoch+1)`` every ``period`` epochs."""
    due = _every(period)

    def on_epoch_end(epoch, sym=None, arg=None, aux=None):
        if due(epoch):
            mod.save_checkpoint(prefix, epoch + 1, save_optimizer_states)
    return on_epoch_end


def do_checkpoint(prefix, period=1):
    """Epoch-end callback: write ``prefix-symbol.json`` + ``prefix-%04d.params`` every ``period`` epochs."""
    due = _every(period)

    def on_epoch_end(epoch, sym, arg, aux):
        if due(epoch):
            from . import model as _model
            _model.save_checkpoint(prefix, epoch + 1, sym, arg, aux)
    return on_epoch_end


def _metric_pairs(metric):
    return list(metric.get_name_value()) if metric is not None else []


def _reset_window(metric):
    """Clear the metric's local (per-window) accumulators."""
    metric.reset_local()


def log_train_metric(period, auto_reset=False):
    """Batch-end callback: log the training metric every ``period`` batches."""
    def on_batch_end(param):
        if param.nbatch % period or param.eval_metric is None:
            return
        for name, value in _metric_pairs(param.eval_metric):
            logging.info('Iter[%d] Batch[%d] Train-%s=%f', param.epoch, param.nbatch, name, value)
        if auto_reset:
            _reset_window(param.eval_metric)
    return on_batch_end


class Speedometer:
    """Batch-end callback: samples/sec (and the metric) over each window of ``frequent`` batches.

    A window starts at the first batch seen (or when the batch counter goes
    backwards, i.e. a new epoch); with ``auto_reset`` the metric's local state
    is cleared after each report so it covers only that window.
    """

    def __init__(self, batch_size, frequent=50, auto_reset=True):
        self.batch_size, self.frequent, self.auto_reset = batch_size, frequent, auto_reset
        self._t0 = None
        self._last = -1

    # reference attribute names, kept for code that inspects them
    @property
    def init(self):
        return self._t0 is not None

    @property
    def tic(self):
        return self._t0 or 0

    @property
    def last_count(self):
        return max(self._last, 0)

    def __call__(self, param):
        n = param.nbatch
        if n < self._last:
            self._t0 = None           # new epoch
        self._last = n
        if self._t0 is None:
            self._t0 = time.time()
            return
        if n % self.frequent:
            return
        elapsed = time.time() - self._t0
        speed = self.frequent * self.batch_size / elapsed if elapsed > 0 else float('inf')
        pairs = _metric_pairs(param.eval_metric)
        if param.eval_metric is None:
            logging.info('Iter[%d] Batch [%d]\tSpeed: %.2f samples/sec', param.epoch, n, speed)
        else:
            first = n - self.frequent if self.auto_reset else 0
            text = ''.join('\t%s=%f' % kv for kv in pairs)
            logging.info('Epoch[%d] Batch [%d-%d]\tSpeed: %.2f samples/sec%s', param.epoch, first, n, speed, text)
            if self.auto_reset:
                _reset_window(param.eval_metric)
        self._t0 = time.time()


class ProgressBar:
    """Batch-end callback drawing a text progress bar of ``total`` batches."""

    def __init__(self, total, length=80):
        self.total = total
        self.bar_len = length

    def __call__(self, param):
        frac = param.nbatch / float(self.total)
        done = int(round(self.bar_len * frac))
        logging.info('[%s] %s%s\r', '=' * done + '-' * (self.bar_len - done), math.ceil(100.0 * frac), '%')


class LogValidationMetricsCallback:
    """Epoch-end (validation) callback logging every metric value."""

    def __call__(self, param):
        for name, value in _metric_pairs(param.eval_metric or None):
            logging.info('Epoch[%d] Validation-%s=%f' % (param.epoch, name, value))
