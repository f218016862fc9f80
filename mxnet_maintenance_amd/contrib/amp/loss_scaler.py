"""Dynamic loss scaling (parity: python/mxnet/contrib/amp/loss_scaler.py).

Start at 2**16; on any non-finite gradient skip the update and halve the
scale; after 2000 clean steps double it (capped at 2**24).  The overflow
check is one fused ``multi_all_finite`` pass (on the flat gradient arena when
the Trainer uses one) and a single device->host read per step.
"""
import logging

import torch

from ... import autograd as ag


class LossScaler:
    def __init__(self, init_scale=2. ** 16, scale_factor=2., scale_window=2000, max_scale=2. ** 24):
        self._loss_scale = init_scale
        self._next_loss_scale = init_scale
        self._max_loss_scale = max_scale
        self._scale_seq_len = scale_window
        self._factor = scale_factor
        self._unskipped = 0

    @property
    def loss_scale(self):
        return self._loss_scale

    def _grads(self, params):
        out = []
        for p in params:
            if getattr(p, 'grad_req', 'write') == 'null' or p._grad is None:
                continue
            for g in p._grad:
                out.append(g._data)
        return out

    def has_overflow(self, params, arenas=None):
        with ag.pause():
            if arenas:
                tensors = [a.g for a in arenas]
            else:
                tensors = self._grads(params)
            if not tensors:
                finite = True
            else:
                flags = torch.stack([torch.isfinite(t).all() for t in tensors])
                finite = bool(flags.all().item())
        has_overflow = not finite
        self._loss_scale = self._next_loss_scale
        if has_overflow:
            self._next_loss_scale = self._loss_scale / self._factor
            self._unskipped = 0
            logging.info('AMP: decreasing loss scale to %f', self._next_loss_scale)
        else:
            self._unskipped += 1
        if self._unskipped == self._scale_seq_len:
            self._unskipped = 0
            self._next_loss_scale = min(self._max_loss_scale, self._loss_scale * self._factor)
            logging.info('AMP: increasing loss scale to %f', self._next_loss_scale)
        return has_overflow
