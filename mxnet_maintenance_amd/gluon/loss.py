"""Loss functions.

Parity: python/mxnet/gluon/loss.py (Loss, L2Loss, L1Loss,
SigmoidBinaryCrossEntropyLoss, SoftmaxCrossEntropyLoss, KLDivLoss, CTCLoss,
HuberLoss, HingeLoss, SquaredHingeLoss, LogisticLoss, TripletLoss,
PoissonNLLLoss, CosineEmbeddingLoss, SDMLLoss).
SoftmaxCrossEntropyLoss with sparse labels on an MI355X runs the fused
row-per-wave HIP kernel (log-softmax + pick + backward in one pass each way).
"""
import numpy as np

from .. import ndarray
from ..base import numeric_types
from .block import HybridBlock

__all__ = ['Loss', 'L2Loss', 'L1Loss', 'SigmoidBinaryCrossEntropyLoss', 'SigmoidBCELoss',
           'SoftmaxCrossEntropyLoss', 'SoftmaxCELoss', 'KLDivLoss', 'CTCLoss', 'HuberLoss', 'HingeLoss',
           'SquaredHingeLoss', 'LogisticLoss', 'TripletLoss', 'PoissonNLLLoss', 'CosineEmbeddingLoss', 'SDMLLoss']


def _apply_weighting(F, loss, weight=None, sample_weight=None):
    """loss * sample_weight (broadcast) * weight (a python number)."""
    out = loss if sample_weight is None else F.broadcast_mul(loss, sample_weight)
    if weight is None:
        return out
    if not isinstance(weight, numeric_types):
        raise AssertionError('weight must be a number')
    return out * weight


def _reshape_like(F, x, y):
    return x.reshape(y.shape) if F is ndarray else F.reshape_like(x, y)


def _batch_mean(F, loss, batch_axis):
    return F.mean(loss, axis=batch_axis, exclude=True)


class Loss(HybridBlock):
    """Base of all losses: ``weight`` (scalar multiplier) and ``batch_axis`` (kept in the output)."""

    def __init__(self, weight, batch_axis, **kwargs):
        super().__init__(**kwargs)
        self._weight = weight
        self._batch_axis = batch_axis

    def __repr__(self):
        return '%s(batch_axis=%s, w=%s)' % (type(self).__name__, self._batch_axis, self._weight)

    def hybrid_forward(self, F, x, *args, **kwargs):
        raise NotImplementedError

    def _finish(self, F, loss, sample_weight, scale=None):
        """Weight (per sample, then by the scalar ``weight``) and average all but the batch axis."""
        w = self._weight if scale is None else scale
        return _batch_mean(F, _apply_weighting(F, loss, w, sample_weight), self._batch_axis)


class _PointwiseLoss(Loss):
    """Losses of the form mean_over_features(f(pred, label)): subclasses define ``_pointwise``."""

    def _pointwise(self, F, pred, label):
        raise NotImplementedError

    def _scale(self):
        return self._weight

    def hybrid_forward(self, F, pred, label, sample_weight=None):
        loss = self._pointwise(F, pred, _reshape_like(F, label, pred))
        return self._finish(F, loss, sample_weight, self._scale())


def _softplus_neg_abs(F, x):
    """log(1 + exp(-|x|)): the numerically safe tail of the logistic losses."""
    return F.Activation(-F.abs(x), act_type='softrelu')


class L2Loss(_PointwiseLoss):
    """0.5 * weight * (label - pred)^2."""

    def __init__(self, weight=1., batch_axis=0, **kwargs):
        super().__init__(weight, batch_axis, **kwargs)

    def _scale(self):
        return self._weight / 2

    def _pointwise(self, F, pred, label):
        return F.square(label - pred)


class L1Loss(_PointwiseLoss):
    """|label - pred|."""

    def __init__(self, weight=None, batch_axis=0, **kwargs):
        super().__init__(weight, batch_axis, **kwargs)

    def _pointwise(self, F, pred, label):
        return F.abs(label - pred)


class SigmoidBinaryCrossEntropyLoss(Loss):
    """Binary cross-entropy on logits (stable form) or on probabilities (``from_sigmoid``),
    with an optional positive-class weight."""

    def __init__(self, from_sigmoid=False, weight=None, batch_axis=0, **kwargs):
        super().__init__(weight, batch_axis, **kwargs)
        self._from_sigmoid = from_sigmoid

    def hybrid_forward(self, F, pred, label, sample_weight=None, pos_weight=None):
        y = _reshape_like(F, label, pred)
        if self._from_sigmoid:
            eps = 1e-12
            pos = F.log(pred + eps) * y
            if pos_weight is not None:
                pos = F.broadcast_mul(pos, pos_weight)
            loss = -(pos + F.log(1. - pred + eps) * (1. - y))
        elif pos_weight is None:
            # max(x, 0) - x*y + log(1 + exp(-|x|))
            loss = F.relu(pred) - pred * y + _softplus_neg_abs(F, pred)
        else:
            scale = 1 + F.broadcast_mul(pos_weight - 1, y)
            loss = pred - pred * y + scale * (_softplus_neg_abs(F, pred) + F.relu(-pred))
        return self._finish(F, loss, sample_weight)


SigmoidBCELoss = SigmoidBinaryCrossEntropyLoss


class SoftmaxCrossEntropyLoss(Loss):
    """-log softmax(pred)[label] (sparse labels) or -sum(label * log softmax(pred)) (dense)."""

    def __init__(self, axis=-1, sparse_label=True, from_logits=False, weight=None, batch_axis=0, **kwargs):
        super().__init__(weight, batch_axis, **kwargs)
        self._axis = axis
        self._sparse_label = sparse_label
        self._from_logits = from_logits

    def _fused_ok(self, F, pred, sample_weight):
        return (F is ndarray and self._sparse_label and not self._from_logits and sample_weight is None
                and self._weight is None and pred.ndim == 2 and self._axis in (-1, 1) and self._batch_axis == 0)

    def hybrid_forward(self, F, pred, label, sample_weight=None):
        if self._fused_ok(F, pred, sample_weight):
            # fused softmax-CE (HIP kernel on gfx950): per-sample loss, fp32 accumulation
            from ..ops import hip_ops
            from ..ndarray.register import _run, _note_leaves
            _note_leaves([pred])
            return ndarray.NDArray(_run(lambda p, l: hip_ops.softmax_ce(p, l).to(p.dtype),
                                        [pred._data, label._data], {}))
        logp = pred if self._from_logits else F.log_softmax(pred, self._axis)
        if self._sparse_label:
            nll = -F.pick(logp, label, axis=self._axis, keepdims=True)
        else:
            nll = -F.sum(logp * _reshape_like(F, label, logp), axis=self._axis, keepdims=True)
        return self._finish(F, nll, sample_weight)


SoftmaxCELoss = SoftmaxCrossEntropyLoss


class KLDivLoss(Loss):
    """sum(label * (log label - log p)); ``pred`` is log-probabilities unless ``from_logits=False``."""

    def __init__(self, from_logits=True, axis=-1, weight=None, batch_axis=0, **kwargs):
        super().__init__(weight, batch_axis, **kwargs)
        self._from_logits = from_logits
        self._axis = axis

    def hybrid_forward(self, F, pred, label, sample_weight=None):
        logp = pred if self._from_logits else F.log_softmax(pred, self._axis)
        return self._finish(F, label * (F.log(label + 1e-12) - logp), sample_weight)


class CTCLoss(Loss):
    """Connectionist temporal classification (blank = last class) over NTC / TNC activations."""

    _LAYOUTS = ('NTC', 'TNC')
    _LABEL_LAYOUTS = ('NT', 'TN')

    def __init__(self, layout='NTC', label_layout='NT', weight=None, **kwargs):
        if layout not in self._LAYOUTS:
            raise AssertionError("Only 'NTC' and 'TNC' layouts for pred are supported. Got: %s" % layout)
        if label_layout not in self._LABEL_LAYOUTS:
            raise AssertionError("Only 'NT' and 'TN' layouts for label are supported. Got: %s" % label_layout)
        self._layout = layout
        self._label_layout = label_layout
        super().__init__(weight, label_layout.index('N'), **kwargs)

    def hybrid_forward(self, F, pred, label, pred_lengths=None, label_lengths=None, sample_weight=None):
        acts = F.swapaxes(pred, 0, 1) if self._layout == 'NTC' else pred          # -> TNC
        lab = F.swapaxes(label, 0, 1) if self._batch_axis == 1 else label          # -> NT
        lengths = [t for t in (pred_lengths, label_lengths) if t is not None]   # the op takes the present ones
        loss = F.CTCLoss(acts, lab, *lengths, use_data_lengths=pred_lengths is not None,
                         use_label_lengths=label_lengths is not None, blank_label='last')
        return _apply_weighting(F, loss, self._weight, sample_weight)


class HuberLoss(_PointwiseLoss):
    """Smooth L1: quadratic below ``rho``, linear above."""

    def __init__(self, rho=1, weight=None, batch_axis=0, **kwargs):
        super().__init__(weight, batch_axis, **kwargs)
        self._rho = rho

    def _pointwise(self, F, pred, label):
        d = F.abs(label - pred)
        return F.where(d > self._rho, d - 0.5 * self._rho, (0.5 / self._rho) * F.square(d))


class HingeLoss(_PointwiseLoss):
    """max(0, margin - pred * label) for labels in {-1, 1}."""

    def __init__(self, margin=1, weight=None, batch_axis=0, **kwargs):
        super().__init__(weight, batch_axis, **kwargs)
        self._margin = margin

    def _pointwise(self, F, pred, label):
        return F.relu(self._margin - pred * label)


class SquaredHingeLoss(HingeLoss):
    """max(0, margin - pred * label)^2."""

    def _pointwise(self, F, pred, label):
        return F.square(super()._pointwise(F, pred, label))


class LogisticLoss(_PointwiseLoss):
    """log(1 + exp(-pred * label)) for signed {-1, 1} or binary {0, 1} labels."""

    def __init__(self, weight=None, batch_axis=0, label_format='signed', **kwargs):
        super().__init__(weight, batch_axis, **kwargs)
        if label_format not in ('signed', 'binary'):
            raise ValueError('label_format can only be signed or binary, recieved %s.' % label_format)
        self._label_format = label_format

    def _pointwise(self, F, pred, label):
        y = (label + 1.0) / 2.0 if self._label_format == 'signed' else label
        return F.relu(pred) - pred * y + _softplus_neg_abs(F, pred)


class TripletLoss(Loss):
    """max(0, ||pred - positive||^2 - ||pred - negative||^2 + margin)."""

    def __init__(self, margin=1, weight=None, batch_axis=0, **kwargs):
        super().__init__(weight, batch_axis, **kwargs)
        self._margin = margin

    def hybrid_forward(self, F, pred, positive, negative, sample_weight=None):
        gap = F.square(_reshape_like(F, positive, pred) - pred) - F.square(_reshape_like(F, negative, pred) - pred)
        loss = F.relu(F.sum(gap, axis=self._batch_axis, exclude=True) + self._margin)
        return _apply_weighting(F, loss, self._weight, sample_weight)


class PoissonNLLLoss(Loss):
    """Poisson negative log-likelihood (optionally with the Stirling term), averaged over everything."""

    def __init__(self, weight=None, from_logits=True, batch_axis=0, compute_full=False, **kwargs):
        super().__init__(weight, batch_axis, **kwargs)
        self._from_logits = from_logits
        self._compute_full = compute_full

    def hybrid_forward(self, F, pred, target, sample_weight=None, epsilon=1e-08):
        t = _reshape_like(F, target, pred)
        loss = F.exp(pred) - t * pred if self._from_logits else pred - t * F.log(pred + epsilon)
        if self._compute_full:
            # Stirling approximation of log(t!), applied where t > 1
            stirling = t * F.log(t) - t + 0.5 * F.log(2 * t * np.pi)
            loss = loss + stirling * (t > 1)
        return F.mean(_apply_weighting(F, loss, self._weight, sample_weight))


class CosineEmbeddingLoss(Loss):
    """1 - cos(x1, x2) for label 1; max(0, cos(x1, x2) - margin) for label -1."""

    def __init__(self, weight=None, batch_axis=0, margin=0, **kwargs):
        super().__init__(weight, batch_axis, **kwargs)
        self._margin = margin

    @staticmethod
    def _const(F, value):
        return F.array([value]) if F is ndarray else F.full((1, 1), value)

    def _cosine_similarity(self, F, x, y, axis=-1):
        col = lambda v: v.reshape((-1, 1))   # noqa: E731
        denom = F.broadcast_maximum(col(F.norm(x, axis=axis)) * col(F.norm(y, axis=axis)), self._const(F, 1e-12))
        return col(F.sum(x * y, axis=axis)) / denom

    def hybrid_forward(self, F, input1, input2, label, sample_weight=None):
        cos = self._cosine_similarity(F, _reshape_like(F, input1, input2), input2)
        y = label.reshape((-1, 1))
        similar = (1 - cos) * (y == 1)
        dissimilar = F.broadcast_maximum(self._const(F, 0), (y == -1) * (cos - self._margin))
        return _apply_weighting(F, similar + dissimilar, self._weight, sample_weight)


class SDMLLoss(Loss):
    """Smoothed deep metric learning loss: KL between a label-smoothed identity and the softmax of
    negative pairwise squared distances within the batch."""

    def __init__(self, smoothing_parameter=0.3, weight=1., batch_axis=0, **kwargs):
        super().__init__(weight, batch_axis, **kwargs)
        self.kl_loss = KLDivLoss(from_logits=True)
        self.smoothing_parameter = smoothing_parameter

    def _compute_distances(self, F, x1, x2):
        diff = F.broadcast_sub(F.expand_dims(x1, 1), F.expand_dims(x2, 0))
        return F.sum(F.square(diff), axis=2)

    def _compute_labels(self, F, batch_size):
        eye = F.eye(batch_size)
        off = self.smoothing_parameter / (batch_size - 1)
        return eye * (1 - self.smoothing_parameter) + (1 - eye) * off

    def hybrid_forward(self, F, x1, x2):
        n = x1.shape[0]
        dist = self._compute_distances(F, x1, x2)
        target = self._compute_labels(F, n).as_in_context(dist.context)
        return self.kl_loss(F.log_softmax(-dist, axis=1), target) * n
