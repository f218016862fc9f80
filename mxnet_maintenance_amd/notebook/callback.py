"""Training-progress callbacks for notebooks.

Parity: python/mxnet/notebook/callback.py:71-403.  ``PandasLogger`` records
train / eval / epoch statistics into pandas DataFrames through the
``Module.fit`` callbacks.  The live charts render with bokeh, which this image
does not ship: ``LiveBokehChart`` and subclasses raise ``ImportError`` with an
explanation when constructed without it (the logger itself needs only pandas).
"""
import datetime
import time
from collections import defaultdict

__all__ = ['PandasLogger', 'LiveBokehChart', 'LiveTimeSeries', 'LiveLearningCurve', 'args_wrapper']


def _pd():
    import pandas as pd     # pylint: disable=import-outside-toplevel
    return pd


class PandasLogger:
    """Collects metric rows into three DataFrames: 'train' (every ``frequent`` batches), 'eval'
    (once per evaluation) and 'epoch' (timing per epoch)."""

    def __init__(self, batch_size, frequent=50):
        pd = _pd()
        self.batch_size = batch_size
        self.frequent = frequent
        self._dataframes = {k: pd.DataFrame() for k in ('train', 'eval', 'epoch')}
        self.last_time = time.time()
        self.start_time = datetime.datetime.now()
        self.last_epoch_time = self.start_time

    @property
    def train_df(self):
        return self._dataframes['train']

    @property
    def eval_df(self):
        return self._dataframes['eval']

    @property
    def epoch_df(self):
        return self._dataframes['epoch']

    @property
    def all_dataframes(self):
        return self._dataframes

    def elapsed(self):
        """Time since the logger was created."""
        return datetime.datetime.now() - self.start_time

    def append_metrics(self, metrics, df_name):
        """Append one row (a dict of column -> value) to DataFrame ``df_name``."""
        df = self._dataframes[df_name]
        for col in set(metrics) - set(df.columns):
            df[col] = None
        df.loc[len(df)] = metrics

    def _process_batch(self, param, df_name):
        now = time.time()
        row = {}
        if param.eval_metric is not None:
            row.update(dict(param.eval_metric.get_name_value()))
            param.eval_metric.reset()
        dt = now - self.last_time
        rate = self.frequent / dt if dt > 0 else float('inf')
        # column meanings follow the reference (its 'batches_per_sec' is samples per second)
        row['batches_per_sec'] = rate * self.batch_size
        row['records_per_sec'] = rate
        row['elapsed'] = self.elapsed()
        row['minibatch_count'] = param.nbatch
        row['epoch'] = param.epoch
        self.append_metrics(row, df_name)
        self.last_time = now

    def train_cb(self, param):
        if param.nbatch % self.frequent == 0:
            self._process_batch(param, 'train')

    def eval_cb(self, param):
        self._process_batch(param, 'eval')

    def epoch_cb(self, *args):      # Module.fit calls it with (epoch, symbol, arg, aux)
        del args
        now = datetime.datetime.now()
        self.append_metrics({'elapsed': self.elapsed(), 'epoch_time': now - self.last_epoch_time}, 'epoch')
        self.last_epoch_time = now

    def callback_args(self):
        """kwargs for ``Module.fit`` enabling every callback of this logger."""
        return {'batch_end_callback': self.train_cb, 'eval_end_callback': self.eval_cb,
                'epoch_end_callback': self.epoch_cb}


def _require_bokeh():
    try:
        import bokeh  # noqa: F401  pylint: disable=import-outside-toplevel,unused-import
    except ImportError as e:
        raise ImportError('live notebook charts need bokeh, which is not installed in this environment; '
                          'PandasLogger works without it') from e


class LiveBokehChart:
    """Base of the live charts (needs bokeh)."""

    def __init__(self, pandas_logger, metric_name, display_freq=10, batch_size=None, frequent=50):
        _require_bokeh()
        self.pandas_logger = pandas_logger or PandasLogger(batch_size=batch_size, frequent=frequent)
        self.display_freq = display_freq
        self.metric_name = metric_name
        self.last_update = time.time()

    def interval_elapsed(self):
        return time.time() - self.last_update > self.display_freq

    def batch_cb(self, param):
        self.pandas_logger.train_cb(param)

    def eval_cb(self, param):
        self.pandas_logger.eval_cb(param)

    def callback_args(self):
        return {'batch_end_callback': self.batch_cb, 'eval_end_callback': self.eval_cb,
                'epoch_end_callback': self.pandas_logger.epoch_cb}


class LiveTimeSeries(LiveBokehChart):
    def __init__(self, **fig_params):
        _require_bokeh()
        super().__init__(None, None, **fig_params)


class LiveLearningCurve(LiveBokehChart):
    def __init__(self, metric_name, display_freq=10, frequent=50):
        super().__init__(None, metric_name, display_freq, frequent=frequent)


def args_wrapper(*args):
    """Merge the ``callback_args()`` of several callback objects into ``Module.fit`` kwargs."""
    out = defaultdict(list)
    for cb in args:
        for k, v in cb.callback_args().items():
            out[k].append(v)
    return dict(out)
