"""Estimator helper functions (reference: python/mxnet/gluon/contrib/estimator/utils.py)."""
from ...loss import SoftmaxCrossEntropyLoss
from ....metric import Accuracy
from .estimator import _check_metrics  # noqa: F401  (shared with the Estimator)

__all__ = []


def _check_metric_known(handler, metric, known_metrics):
    if metric not in known_metrics:
        raise ValueError('Event handler %s refers to a metric instance %s outside of the known training and '
                         'validation metrics. Please use the metrics from estimator.train_metrics and '
                         'estimator.val_metrics instead.' % (type(handler).__name__, metric))


def _check_handler_metric_ref(handler, known_metrics):
    """Every metric an event handler holds (attributes named *metric*) must be one of the estimator's."""
    for attr in dir(handler):
        if 'metric' not in attr:
            continue
        ref = getattr(handler, attr, None)
        if not ref or callable(ref):
            continue
        for m in (ref if isinstance(ref, list) else [ref]):
            _check_metric_known(handler, m, known_metrics)


def _suggest_metric_for_loss(loss):
    """A default metric for a loss (accuracy for softmax cross-entropy), else None."""
    return Accuracy() if isinstance(loss, SoftmaxCrossEntropyLoss) else None
