"""Gluon Estimator: fit/evaluate loop with event handlers (parity: gluon/contrib/estimator)."""
from .estimator import Estimator  # noqa: F401
from .event_handler import *  # noqa: F401,F403
from .batch_processor import BatchProcessor  # noqa: F401
