"""Learning-rate schedules.

Parity: python/mxnet/lr_scheduler.py (LRScheduler with warmup, FactorScheduler,
MultiFactorScheduler, PolyScheduler, CosineScheduler).
"""
import logging
from math import cos, pi

__all__ = ['LRScheduler', 'FactorScheduler', 'MultiFactorScheduler', 'PolyScheduler', 'CosineScheduler']


class LRScheduler:
    def __init__(self, base_lr=0.01, warmup_steps=0, warmup_begin_lr=0, warmup_mode='linear'):
        self.base_lr = base_lr
        assert isinstance(warmup_steps, int)
        self.warmup_steps = warmup_steps
        self.warmup_final_lr = base_lr
        self.warmup_begin_lr = warmup_begin_lr
        if self.warmup_begin_lr > self.warmup_final_lr:
            raise ValueError('Base lr has to be higher than warmup_begin_lr')
        if self.warmup_steps < 0:
            raise ValueError('Warmup steps has to be positive or 0')
        if warmup_mode not in ['linear', 'constant']:
            raise ValueError('Supports only linear and constant modes of warmup')
        self.warmup_mode = warmup_mode

    def get_warmup_lr(self, num_update):
        assert num_update < self.warmup_steps
        if self.warmup_mode == 'linear':
            increase = (self.warmup_final_lr - self.warmup_begin_lr) * float(num_update) / float(self.warmup_steps)
            return self.warmup_begin_lr + increase
        if self.warmup_mode == 'constant':
            return self.warmup_begin_lr
        raise ValueError('Invalid warmup mode %s' % self.warmup_mode)

    def __call__(self, num_update):
        raise NotImplementedError('must override this')


class FactorScheduler(LRScheduler):
    """lr = base_lr * factor^(floor(num_update/step)), bounded below by stop_factor_lr."""

    def __init__(self, step, factor=1, stop_factor_lr=1e-8, base_lr=0.01, warmup_steps=0, warmup_begin_lr=0,
                 warmup_mode='linear'):
        super().__init__(base_lr, warmup_steps, warmup_begin_lr, warmup_mode)
        if step < 1:
            raise ValueError('Schedule step must be greater or equal than 1 round')
        if factor > 1.0:
            raise ValueError('Factor must be no more than 1 to make lr reduce')
        self.step = step
        self.factor = factor
        self.stop_factor_lr = stop_factor_lr
        self.count = 0

    def __call__(self, num_update):
        if num_update < self.warmup_steps:
            return self.get_warmup_lr(num_update)
        while num_update > self.count + self.step:
            self.count += self.step
            self.base_lr *= self.factor
            if self.base_lr < self.stop_factor_lr:
                self.base_lr = self.stop_factor_lr
                logging.info('Update[%d]: now learning rate arrived at %0.5e, will not change in the future',
                             num_update, self.base_lr)
            else:
                logging.info('Update[%d]: Change learning rate to %0.5e', num_update, self.base_lr)
        return self.base_lr


class MultiFactorScheduler(LRScheduler):
    def __init__(self, step, factor=1, base_lr=0.01, warmup_steps=0, warmup_begin_lr=0, warmup_mode='linear'):
        super().__init__(base_lr, warmup_steps, warmup_begin_lr, warmup_mode)
        assert isinstance(step, list) and len(step) >= 1
        for i, _step in enumerate(step):
            if i != 0 and step[i] <= step[i - 1]:
                raise ValueError('Schedule step must be an increasing integer list')
            if _step < 1:
                raise ValueError('Schedule step must be greater or equal than 1 round')
        if factor > 1.0:
            raise ValueError('Factor must be no more than 1 to make lr reduce')
        self.step = step
        self.cur_step_ind = 0
        self.factor = factor
        self.count = 0

    def __call__(self, num_update):
        if num_update < self.warmup_steps:
            return self.get_warmup_lr(num_update)
        while self.cur_step_ind <= len(self.step) - 1:
            if num_update > self.step[self.cur_step_ind]:
                self.count = self.step[self.cur_step_ind]
                self.cur_step_ind += 1
                self.base_lr *= self.factor
                logging.info('Update[%d]: Change learning rate to %0.5e', num_update, self.base_lr)
            else:
                return self.base_lr
        return self.base_lr


class PolyScheduler(LRScheduler):
    def __init__(self, max_update, base_lr=0.01, pwr=2, final_lr=0, warmup_steps=0, warmup_begin_lr=0,
                 warmup_mode='linear'):
        super().__init__(base_lr, warmup_steps, warmup_begin_lr, warmup_mode)
        assert isinstance(max_update, int)
        if max_update < 1:
            raise ValueError('maximum number of updates must be strictly positive')
        self.power = pwr
        self.base_lr_orig = self.base_lr
        self.max_update = max_update
        self.final_lr = final_lr
        self.max_steps = self.max_update - self.warmup_steps

    def __call__(self, num_update):
        if num_update < self.warmup_steps:
            return self.get_warmup_lr(num_update)
        if num_update <= self.max_update:
            self.base_lr = self.final_lr + (self.base_lr_orig - self.final_lr) * \
                pow(1 - float(num_update - self.warmup_steps) / float(self.max_steps), self.power)
        return self.base_lr


class CosineScheduler(LRScheduler):
    def __init__(self, max_update, base_lr=0.01, final_lr=0, warmup_steps=0, warmup_begin_lr=0,
                 warmup_mode='linear'):
        super().__init__(base_lr, warmup_steps, warmup_begin_lr, warmup_mode)
        assert isinstance(max_update, int)
        if max_update < 1:
            raise ValueError('maximum number of updates must be strictly positive')
        self.base_lr_orig = base_lr
        self.max_update = max_update
        self.final_lr = final_lr
        self.max_steps = self.max_update - self.warmup_steps

    def __call__(self, num_update):
        if num_update < self.warmup_steps:
            return self.get_warmup_lr(num_update)
        if num_update <= self.max_update:
            self.base_lr = self.final_lr + (self.base_lr_orig - self.final_lr) * \
                (1 + cos(pi * (num_update - self.warmup_steps) / self.max_steps)) / 2
        return self.base_lr
