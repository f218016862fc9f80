"""Learning-rate schedules (API parity: python/mxnet/lr_scheduler.py).

Every schedule here is a closed-form function of the update counter: a shared
warm-up ramp for ``t < warmup_steps`` and a subclass-defined ``_decayed(t)``
afterwards.  There is no hidden step-by-step state, so a schedule can be
queried for any ``t`` (e.g. after a checkpoint resume) and gives the value the
reference's incremental implementation reaches after the same updates.

``base_lr`` is the peak learning rate reached at the end of warm-up; the
optimizer assigns it when the scheduler is attached.
"""
import bisect
import logging
import math

__all__ = ['LRScheduler', 'FactorScheduler', 'MultiFactorScheduler', 'PolyScheduler', 'CosineScheduler']

_WARMUP_MODES = ('linear', 'constant')


class LRScheduler:
    """Base schedule: warm-up handling; subclasses implement ``_decayed``."""

    def __init__(self, base_lr=0.01, warmup_steps=0, warmup_begin_lr=0, warmup_mode='linear'):
        if not isinstance(warmup_steps, int):
            raise AssertionError('warmup_steps must be an int')
        if warmup_steps < 0:
            raise ValueError('warmup_steps must be >= 0, got %d' % warmup_steps)
        if warmup_mode not in _WARMUP_MODES:
            raise ValueError('warmup_mode must be one of %s, got %r' % (_WARMUP_MODES, warmup_mode))
        if warmup_begin_lr > base_lr:
            raise ValueError('warmup_begin_lr (%g) exceeds base_lr (%g)' % (warmup_begin_lr, base_lr))
        self.base_lr = base_lr
        self.warmup_final_lr = base_lr      # the ramp's target is fixed at construction
        self.warmup_steps = warmup_steps
        self.warmup_begin_lr = warmup_begin_lr
        self.warmup_mode = warmup_mode
        self._last_logged = None

    def get_warmup_lr(self, num_update):
        """Learning rate during warm-up (``num_update < warmup_steps``)."""
        if not num_update < self.warmup_steps:
            raise AssertionError('num_update %d is past warm-up' % num_update)
        if self.warmup_mode == 'constant':
            return self.warmup_begin_lr
        frac = float(num_update) / float(self.warmup_steps)
        return self.warmup_begin_lr + (self.warmup_final_lr - self.warmup_begin_lr) * frac

    def _decayed(self, num_update):
        raise NotImplementedError('schedules implement _decayed(num_update)')

    def __call__(self, num_update):
        if num_update < self.warmup_steps:
            return self.get_warmup_lr(num_update)
        lr = self._decayed(num_update)
        if lr != self._last_logged:
            if self._last_logged is not None:
                logging.info('Update[%d]: learning rate is now %0.5e', num_update, lr)
            self._last_logged = lr
        return lr

    def __repr__(self):
        return '%s(base_lr=%g, warmup_steps=%d)' % (type(self).__name__, self.base_lr, self.warmup_steps)


def _repeat_mul(lr, factor, n):
    """``lr * factor ** n`` as n successive multiplications: bit-identical to a schedule that decays
    its learning rate in place once per period (what user code comparing lr values expects)."""
    for _ in range(n):
        lr *= factor
    return lr


class FactorScheduler(LRScheduler):
    """``base_lr * factor ** k`` after ``k`` completed periods of ``step`` updates, floored at
    ``stop_factor_lr`` (the k-th decay applies once ``num_update > k * step``)."""

    def __init__(self, step, factor=1, stop_factor_lr=1e-8, base_lr=0.01, warmup_steps=0, warmup_begin_lr=0,
                 warmup_mode='linear'):
        super().__init__(base_lr, warmup_steps, warmup_begin_lr, warmup_mode)
        if step < 1:
            raise ValueError('step must be >= 1 update, got %s' % step)
        if factor > 1.0:
            raise ValueError('factor must be <= 1 for a decaying schedule, got %s' % factor)
        self.step = step
        self.factor = factor
        self.stop_factor_lr = stop_factor_lr

    def _decayed(self, num_update):
        periods = max(0, -(-num_update // self.step) - 1)     # ceil(t / step) - 1, never negative
        return max(_repeat_mul(self.base_lr, self.factor, periods), self.stop_factor_lr)


class MultiFactorScheduler(LRScheduler):
    """Multiply by ``factor`` each time ``num_update`` passes one of the increasing ``step`` marks."""

    def __init__(self, step, factor=1, base_lr=0.01, warmup_steps=0, warmup_begin_lr=0, warmup_mode='linear'):
        super().__init__(base_lr, warmup_steps, warmup_begin_lr, warmup_mode)
        if not isinstance(step, list) or not step:
            raise AssertionError('step must be a non-empty list of update counts')
        if any(s < 1 for s in step):
            raise ValueError('every step mark must be >= 1')
        if any(b <= a for a, b in zip(step, step[1:])):
            raise ValueError('step marks must be strictly increasing')
        if factor > 1.0:
            raise ValueError('factor must be <= 1 for a decaying schedule, got %s' % factor)
        self.step = step
        self.factor = factor

    def _decayed(self, num_update):
        passed = bisect.bisect_left(self.step, num_update)      # marks strictly below num_update
        return _repeat_mul(self.base_lr, self.factor, passed)


class _AnnealTo(LRScheduler):
    """Shared shape of Poly/Cosine: anneal from ``base_lr`` to ``final_lr`` over the updates between
    the end of warm-up and ``max_update``, then hold ``final_lr``."""

    def __init__(self, max_update, base_lr, final_lr, warmup_steps, warmup_begin_lr, warmup_mode):
        super().__init__(base_lr, warmup_steps, warmup_begin_lr, warmup_mode)
        if not isinstance(max_update, int):
            raise AssertionError('max_update must be an int')
        if max_update < 1:
            raise ValueError('max_update must be >= 1, got %d' % max_update)
        self.max_update = max_update
        self.final_lr = final_lr
        self.base_lr_orig = base_lr          # annealing starts from the constructor's peak

    @property
    def max_steps(self):
        return self.max_update - self.warmup_steps

    def _shape(self, progress):
        raise NotImplementedError

    def _decayed(self, num_update):
        t = min(num_update, self.max_update) - self.warmup_steps
        progress = float(t) / float(self.max_steps) if self.max_steps > 0 else 1.0
        return self.final_lr + (self.base_lr_orig - self.final_lr) * self._shape(progress)


class PolyScheduler(_AnnealTo):
    """Polynomial decay ``(1 - progress) ** pwr``."""

    def __init__(self, max_update, base_lr=0.01, pwr=2, final_lr=0, warmup_steps=0, warmup_begin_lr=0,
                 warmup_mode='linear'):
        super().__init__(max_update, base_lr, final_lr, warmup_steps, warmup_begin_lr, warmup_mode)
        self.power = pwr

    def _shape(self, progress):
        return (1.0 - progress) ** self.power


class CosineScheduler(_AnnealTo):
    """Half-cosine decay ``(1 + cos(pi * progress)) / 2``."""

    def __init__(self, max_update, base_lr=0.01, final_lr=0, warmup_steps=0, warmup_begin_lr=0,
                 warmup_mode='linear'):
        super().__init__(max_update, base_lr, final_lr, warmup_steps, warmup_begin_lr, warmup_mode)

    def _shape(self, progress):
        return 0.5 * (1.0 + math.cos(math.pi * progress))
