"""Index samplers for DataLoader (API parity: python/mxnet/gluon/data/sampler.py).

Each sampler is an iterable of dataset indices with a known length.  Index
sequences are produced as numpy arrays (``_indices``) and converted to Python
ints on iteration; ``BatchSampler`` groups any sampler into lists.
"""
import numpy as np

__all__ = ['Sampler', 'SequentialSampler', 'RandomSampler', 'FilterSampler', 'BatchSampler', 'IntervalSampler']

_LAST_BATCH = ('keep', 'discard', 'rollover')


class Sampler:
    """Base class: subclasses define ``_indices()`` (numpy int array) or override ``__iter__``."""

    def _indices(self):
        raise NotImplementedError('%s must define _indices()' % type(self).__name__)

    def __iter__(self):
        return iter(self._indices().tolist())

    def __len__(self):
        raise NotImplementedError('%s must define __len__()' % type(self).__name__)


class SequentialSampler(Sampler):
    """``start, start+1, ..., start+length-1``."""

    def __init__(self, length, start=0):
        self._length = length
        self._start = start

    def _indices(self):
        return np.arange(self._start, self._start + self._length)

    def __len__(self):
        return self._length


class RandomSampler(Sampler):
    """A fresh random permutation of ``range(length)`` per epoch (numpy global RNG)."""

    def __init__(self, length):
        self._length = length

    def _indices(self):
        return np.random.permutation(self._length)

    def __len__(self):
        return self._length


class FilterSampler(Sampler):
    """Indices of the samples of ``dataset`` for which ``fn(sample)`` holds (evaluated once)."""

    def __init__(self, fn, dataset):
        self._fn = fn
        self._dataset = dataset
        self._keep = np.array([i for i in range(len(dataset)) if fn(dataset[i])], dtype=np.int64)

    def _indices(self):
        return self._keep

    def __len__(self):
        return len(self._keep)


class IntervalSampler(Sampler):
    """Strided passes: ``0, k, 2k, ...`` then (with ``rollover``) ``1, 1+k, ...`` up to offset k-1."""

    def __init__(self, length, interval, rollover=True):
        if not interval < length:
            raise AssertionError('interval %d must be smaller than length %d' % (interval, length))
        self._length = length
        self._interval = interval
        self._rollover = rollover

    def _indices(self):
        offsets = range(self._interval) if self._rollover else range(1)
        return np.concatenate([np.arange(o, self._length, self._interval) for o in offsets])

    def __len__(self):
        return self._length


class BatchSampler(Sampler):
    """Group the indices of ``sampler`` into lists of ``batch_size``.

    ``last_batch``: 'keep' yields a short final batch, 'discard' drops it,
    'rollover' carries its indices into the first batch of the next epoch.
    """

    def __init__(self, sampler, batch_size, last_batch='keep'):
        self._sampler = sampler
        self._bsz = batch_size
        self._mode = last_batch
        self._carry = []

    def _check_mode(self):
        if self._mode not in _LAST_BATCH:
            raise ValueError('last_batch must be one of %s, got %r' % (_LAST_BATCH, self._mode))

    def __iter__(self):
        self._check_mode()
        pending, self._carry = list(self._carry), []
        for idx in self._sampler:
            pending.append(idx)
            if len(pending) == self._bsz:
                yield pending
                pending = []
        if not pending:
            return
        mode = self._mode
        if mode == 'rollover':
            self._carry = pending
        elif mode == 'keep':
            yield pending

    def __len__(self):
        self._check_mode()
        n, b, mode = len(self._sampler), self._bsz, self._mode
        if mode == 'rollover':
            return (n + len(self._carry)) // b
        return n // b if mode == 'discard' else -(-n // b)
