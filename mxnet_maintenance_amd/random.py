"""Random number generation (mx.random).

Parity: python/mxnet/random.py (seed, uniform, normal, randn, randint,
exponential, gamma, poisson, multinomial, shuffle...).
"""
import random as _pyrandom

import numpy as _np
import torch

from .ndarray.random import *  # noqa: F401,F403
from .ndarray.random import __all__ as _nd_all

__all__ = ['seed'] + list(_nd_all)


def seed(seed_state, ctx='all'):
    """Seed the generators of all devices (or one context)."""
    if not isinstance(seed_state, int):
        raise ValueError('seed_state must be int')
    if ctx == 'all' or getattr(ctx, 'device_type', 'cpu') == 'cpu':
        torch.manual_seed(seed_state)
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        if ctx == 'all':
            torch.cuda.manual_seed_all(seed_state)
        elif getattr(ctx, 'device_type', '') == 'gpu':
            with torch.cuda.device(ctx.device_id):
                torch.cuda.manual_seed(seed_state)
