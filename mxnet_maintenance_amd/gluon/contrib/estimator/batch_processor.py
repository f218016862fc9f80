"""Per-batch train / evaluate hooks of the Estimator (parity: gluon/contrib/estimator/batch_processor.py)."""
from .... import autograd
from ...utils import split_and_load

__all__ = ['BatchProcessor']


class BatchProcessor:
    """Override ``fit_batch`` / ``evaluate_batch`` to customise one training / validation step."""

    def _get_data_and_label(self, batch, ctx, batch_axis=0):
        data = split_and_load(batch[0], ctx_list=ctx, batch_axis=batch_axis)
        label = split_and_load(batch[1], ctx_list=ctx, batch_axis=batch_axis)
        return data, label

    def evaluate_batch(self, estimator, val_batch, batch_axis=0):
        data, label = self._get_data_and_label(val_batch, estimator.context, batch_axis)
        pred = [estimator.val_net(x) for x in data]
        loss = [estimator.val_loss(y_hat, y) for y_hat, y in zip(pred, label)]
        return data, label, pred, loss

    def fit_batch(self, estimator, train_batch, batch_axis=0):
        data, label = self._get_data_and_label(train_batch, estimator.context, batch_axis)
        with autograd.record():
            pred = [estimator.net(x) for x in data]
            loss = [estimator.loss(y_hat, y) for y_hat, y in zip(pred, label)]
        for l in loss:
            l.backward()
        return data, label, pred, loss
