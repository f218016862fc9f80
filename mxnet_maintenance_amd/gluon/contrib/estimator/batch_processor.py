"""One training / validation step of the Estimator (API parity: gluon/contrib/estimator/batch_processor.py).

Subclass and override ``fit_batch`` / ``evaluate_batch`` to customise the step;
both return ``(data, label, pred, loss)`` as per-device lists.
"""
from .... import autograd
from ...utils import split_and_load

__all__ = ['BatchProcessor']


class BatchProcessor:
    def _get_data_and_label(self, batch, ctx, batch_axis=0):
        """Split ``(data, label)`` of a batch across the estimator's devices."""
        return tuple(split_and_load(part, ctx_list=ctx, batch_axis=batch_axis) for part in batch[:2])

    @staticmethod
    def _run(net, loss_fn, data, label):
        pred = [net(x) for x in data]
        return pred, [loss_fn(p, y) for p, y in zip(pred, label)]

    def evaluate_batch(self, estimator, val_batch, batch_axis=0):
        data, label = self._get_data_and_label(val_batch, estimator.context, batch_axis)
        pred, loss = self._run(estimator.val_net, estimator.val_loss, data, label)
        return data, label, pred, loss

    def fit_batch(self, estimator, train_batch, batch_axis=0):
        data, label = self._get_data_and_label(train_batch, estimator.context, batch_axis)
        with autograd.record():
            pred, loss = self._run(estimator.net, estimator.loss, data, label)
        autograd.backward(loss)
        return data, label, pred, loss
