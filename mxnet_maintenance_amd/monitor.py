"""Executor monitor: periodic statistics of operator outputs, arguments and aux states.

API parity: python/mxnet/monitor.py (``Monitor(interval, stat_func, pattern, sort,
monitor_all)``, ``install``, ``tic``, ``toc``, ``toc_print``).

Design: a ``Monitor`` is a sampling window.  ``tic()`` opens a window on every
``interval``-th batch; while it is open, the executor callback (installed with
``install``) reports each operator output whose name matches ``pattern``.
``toc()`` closes the window, adds the bound arguments / aux states, and returns
``(batch, name, text)`` rows.  Statistics are computed lazily on the GPU (the
callback only stores the stat NDArray); text formatting happens at ``toc``.
"""
import logging
import re

from .ndarray.ndarray import NDArray

__all__ = ['Monitor']


def _rms(arr):
    """Default statistic: ||x||_2 / sqrt(numel), i.e. the root mean square."""
    from . import ndarray as nd
    return nd.norm(arr) / (arr.size ** 0.5)


def _render(stat):
    """Text of a statistic: scalars as numbers, tensors via numpy, lists tab-joined."""
    items = stat if isinstance(stat, (list, tuple)) else [stat]
    out = []
    for v in items:
        if not isinstance(v, NDArray):
            raise AssertionError('monitor statistic must return NDArray(s), got %s' % type(v))
        out.append(str(v.asscalar()) if v.size == 1 and v.ndim <= 1 else str(v.asnumpy()))
    return ''.join(t + '\t' for t in out)


class Monitor:
    """Collect ``stat_func`` of matching arrays every ``interval`` batches."""

    def __init__(self, interval, stat_func=None, pattern='.*', sort=False, monitor_all=False):
        self.interval = interval
        self.stat_func = stat_func if stat_func is not None else _rms
        self.re_prog = re.compile(pattern)
        self.sort = sort
        self.monitor_all = monitor_all
        self.exes = []
        self.step = 0
        self.activated = False
        self.queue = []
        # bound method kept as an attribute: executors hold on to it
        self.stat_helper = self._observe

    def _observe(self, name, array):
        if not isinstance(array, NDArray):
            array = NDArray(array)       # an NDArrayHandle from the executor callback
        if self.activated and self.re_prog.match(name):
            self.queue.append((self.step, name, self.stat_func(array)))

    def install(self, exe):
        """Attach to an executor (every op output goes through ``stat_helper``)."""
        exe.set_monitor_callback(self.stat_helper, self.monitor_all)
        self.exes.append(exe)

    def tic(self):
        """Start of a batch: open a sampling window every ``interval`` batches."""
        if self.step % self.interval == 0:
            self.activated = True
            self.queue = []
        self.step += 1

    def _bound_arrays(self):
        for exe in self.exes:
            sym = exe._symbol
            yield from zip(sym.list_arguments(), exe.arg_arrays)
            yield from zip(sym.list_auxiliary_states(), exe.aux_arrays)

    def toc(self):
        """End of a batch: return ``[(batch, name, stat_text)]`` for an open window, else ``[]``."""
        if not self.activated:
            return []
        bound = list(self._bound_arrays())
        for _name, arr in bound:
            arr.wait_to_read()
        self.queue.extend((self.step, name, self.stat_func(arr)) for name, arr in bound if self.re_prog.match(name))
        self.activated = False
        rows = sorted(self.queue, key=lambda r: r[1]) if self.sort else self.queue
        self.queue = []
        return [(batch, name, _render(stat)) for batch, name, stat in rows]

    def toc_print(self):
        for batch, name, text in self.toc():
            logging.info('Batch: %7d %-30s %s', batch, name, text)
