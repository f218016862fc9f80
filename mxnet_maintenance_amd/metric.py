"""Evaluation metrics (API parity: python/mxnet/metric.py).

Public surface as in the reference: ``EvalMetric`` (update / update_dict /
reset / reset_local / get / get_global / get_name_value /
get_global_name_value / get_config), ``CompositeEvalMetric``, ``Accuracy``,
``TopKAccuracy``, ``F1``, ``MCC``, ``Perplexity``, ``MAE``, ``MSE``, ``RMSE``,
``CrossEntropy``, ``NegativeLogLikelihood``, ``PearsonCorrelation``, ``PCC``,
``Loss`` (+ ``Torch`` / ``Caffe``), ``CustomMetric``, ``np``, ``create``,
``register``, ``check_label_shapes``.

Design notes:

* every metric keeps two running (sum, count) pairs -- *local* (since the last
  ``reset_local``) and *global* (since ``reset``) -- updated together by
  ``_accumulate``;
* classification metrics over device tensors reduce ON the device and
  transfer one scalar per batch (argmax / top-k / gather run in torch);
* F1, MCC and PCC share one ``_Confusion`` matrix accumulator (binary F1 /
  MCC use its 2x2 form), with per-batch ("macro") or running ("micro")
  averaging.
"""
import math
from collections import OrderedDict

import numpy
import torch

from .base import numeric_types, string_types
from .ndarray.ndarray import NDArray

__all__ = ['EvalMetric', 'CompositeEvalMetric', 'Accuracy', 'TopKAccuracy', 'F1', 'MCC', 'Perplexity', 'MAE',
           'MSE', 'RMSE', 'CrossEntropy', 'NegativeLogLikelihood', 'PearsonCorrelation', 'PCC', 'Loss', 'Torch',
           'Caffe', 'CustomMetric', 'np', 'create', 'register', 'check_label_shapes']


def check_label_shapes(labels, preds, wrap=False, shape=False):
    """Raise ValueError unless labels and preds agree in length (or full shape); optionally wrap
    single arrays into lists."""
    a, b = (labels.shape, preds.shape) if shape else (len(labels), len(preds))
    if a != b:
        raise ValueError('Shape of labels {} does not match shape of predictions {}'.format(a, b))
    if wrap:
        single = (NDArray, numpy.ndarray)
        labels = [labels] if isinstance(labels, single) else labels
        preds = [preds] if isinstance(preds, single) else preds
    return labels, preds


def _host(x):
    return x.asnumpy() if isinstance(x, NDArray) else numpy.asarray(x)


def _dev(x):
    """A torch tensor view of an NDArray (no copy) or of host data."""
    return x._data if isinstance(x, NDArray) else torch.as_tensor(numpy.asarray(x))


def _pairs(names, values):
    names = names if isinstance(names, list) else [names]
    values = values if isinstance(values, list) else [values]
    return list(zip(names, values))


class EvalMetric:
    """Base metric: ``update`` adds to the running sums, ``get`` reports sum / count."""

    def __init__(self, name, output_names=None, label_names=None, **kwargs):
        self.name = str(name)
        self.output_names = output_names
        self.label_names = label_names
        self._has_global_stats = kwargs.pop('has_global_stats', False)
        self._kwargs = kwargs
        self.reset()

    def __str__(self):
        return 'EvalMetric: {}'.format(dict(self.get_name_value()))

    def get_config(self):
        cfg = dict(self._kwargs)
        cfg.update(metric=type(self).__name__, name=self.name, output_names=self.output_names,
                   label_names=self.label_names)
        return cfg

    # ---------------------------------------------------------------- feeding
    @staticmethod
    def _select(mapping, names):
        return list(mapping.values()) if names is None else [mapping[n] for n in names]

    def update_dict(self, label, pred):
        """Update from ``{name: array}`` dicts, picking ``label_names`` / ``output_names``."""
        self.update(self._select(label, self.label_names), self._select(pred, self.output_names))

    def update(self, labels, preds):
        raise NotImplementedError('%s.update' % type(self).__name__)

    def _accumulate(self, total, count):
        self.sum_metric += total
        self.num_inst += count
        self.global_sum_metric += total
        self.global_num_inst += count

    _add = _accumulate     # short alias used by subclasses written against the older name

    # ---------------------------------------------------------------- state
    def reset_local(self):
        self.sum_metric, self.num_inst = 0.0, 0

    def reset(self):
        self.reset_local()
        self.global_sum_metric, self.global_num_inst = 0.0, 0

    # ---------------------------------------------------------------- reporting
    def _value(self, total, count):
        return float('nan') if count == 0 else total / count

    def get(self):
        return self.name, self._value(self.sum_metric, self.num_inst)

    def get_global(self):
        if not self._has_global_stats:
            return self.get()
        return self.name, self._value(self.global_sum_metric, self.global_num_inst)

    def get_name_value(self):
        return _pairs(*self.get())

    def get_global_name_value(self):
        return _pairs(*self.get_global()) if self._has_global_stats else self.get_name_value()


# ------------------------------------------------------------------------ registry
_METRICS = {}


def register(klass):
    """Class decorator: make ``klass`` creatable by its lower-cased name."""
    _METRICS[klass.__name__.lower()] = klass
    return klass


def alias(*aliases):
    def deco(klass):
        _METRICS.update({a.lower(): klass for a in aliases})
        return klass
    return deco


def create(metric, *args, **kwargs):
    """Metric from a name, class, instance, callable (CustomMetric) or list (composite)."""
    if isinstance(metric, EvalMetric):
        return metric
    if isinstance(metric, list):
        return CompositeEvalMetric([create(m, *args, **kwargs) for m in metric])
    if isinstance(metric, type) and issubclass(metric, EvalMetric):
        return metric(*args, **kwargs)
    if callable(metric):
        return CustomMetric(metric, *args, **kwargs)
    if isinstance(metric, dict) or (isinstance(metric, str) and metric.lstrip()[:1] in ('{', '[')):
        # serialised form: get_config() (dict or JSON) {"metric": name, ...}, or JSON [name, {kwargs}]
        import json
        cfg = metric if isinstance(metric, dict) else json.loads(metric)
        if isinstance(cfg, list):
            name, extra = cfg[0], (cfg[1] if len(cfg) > 1 else {})
        else:
            extra = dict(cfg)
            name = extra.pop('metric')
        return create(name, *args, **dict(extra, **kwargs))
    try:
        return _METRICS[metric.lower()](*args, **kwargs)
    except KeyError:
        raise ValueError('unknown metric %r; registered: %s' % (metric, sorted(_METRICS))) from None


# ------------------------------------------------------------------------ composite
@register
@alias('composite')
class CompositeEvalMetric(EvalMetric):
    """Several metrics updated together; ``get`` returns parallel name / value lists."""

    def __init__(self, metrics=None, name='composite', output_names=None, label_names=None):
        self.metrics = []
        super().__init__(name, output_names=output_names, label_names=label_names, has_global_stats=True)
        self.metrics = [create(m) for m in (metrics or [])]

    def add(self, metric):
        self.metrics.append(create(metric))

    def get_metric(self, index):
        if not -len(self.metrics) <= index < len(self.metrics):
            return ValueError('Metric index {} is out of range 0 and {}'.format(index, len(self.metrics)))
        return self.metrics[index]

    def update_dict(self, labels, preds):
        keep = lambda d, names: d if names is None else OrderedDict((k, v) for k, v in d.items() if k in names)  # noqa
        labels, preds = keep(labels, self.label_names), keep(preds, self.output_names)
        for m in self.metrics:
            m.update_dict(labels, preds)

    def update(self, labels, preds):
        for m in self.metrics:
            m.update(labels, preds)

    def reset(self):
        for m in getattr(self, 'metrics', []):
            m.reset()

    def reset_local(self):
        for m in getattr(self, 'metrics', []):
            m.reset_local()

    @staticmethod
    def _gather(results):
        names, values = [], []
        for n, v in results:
            names.extend([n] if isinstance(n, string_types) else n)
            values.extend([v] if isinstance(v, numeric_types) else v)
        return names, values

    def get(self):
        return self._gather(m.get() for m in self.metrics)

    def get_global(self):
        return self._gather(m.get_global() for m in self.metrics)

    def get_config(self):
        cfg = super().get_config()
        cfg['metrics'] = [m.get_config() for m in self.metrics]
        return cfg


# ------------------------------------------------------------------------ classification
@register
@alias('acc')
class Accuracy(EvalMetric):
    """Fraction of correct predictions; class scores are arg-maxed over ``axis``."""

    def __init__(self, axis=1, name='accuracy', output_names=None, label_names=None):
        super().__init__(name, axis=axis, output_names=output_names, label_names=label_names,
                         has_global_stats=True)
        self.axis = axis

    def update(self, labels, preds):
        labels, preds = check_label_shapes(labels, preds, True)
        for label, pred in zip(labels, preds):
            p, l = _dev(pred), _dev(label)
            if p.shape != l.shape:
                p = torch.argmax(p, dim=self.axis)
            p = p.reshape(-1).to(torch.int64)
            l = l.reshape(-1).to(device=p.device, dtype=torch.int64)
            if p.numel() != l.numel():
                raise ValueError('Shape of labels {} does not match shape of predictions {}'.format(
                    tuple(l.shape), tuple(p.shape)))
            self._accumulate(int((p == l).sum()), int(l.numel()))


@register
@alias('top_k_accuracy', 'top_k_acc')
class TopKAccuracy(EvalMetric):
    """A prediction counts as correct when the label is among the ``top_k`` highest scores."""

    def __init__(self, top_k=1, name='top_k_accuracy', output_names=None, label_names=None):
        if not top_k > 1:
            raise AssertionError('Please use Accuracy if top_k is no more than 1')
        super().__init__('%s_%d' % (name, top_k), top_k=top_k, output_names=output_names, label_names=label_names,
                         has_global_stats=True)
        self.top_k = top_k

    def update(self, labels, preds):
        labels, preds = check_label_shapes(labels, preds, True)
        for label, pred in zip(labels, preds):
            p = _dev(pred).float()
            if p.dim() > 2:
                raise AssertionError('Predictions should be no more than 2 dims')
            l = _dev(label).to(device=p.device, dtype=torch.int64).reshape(-1)
            check_label_shapes(l, p)
            if p.dim() == 1:
                hits = int((p.to(torch.int64) == l).sum())
            else:
                k = min(self.top_k, p.shape[1])
                top = torch.topk(p, k, dim=1).indices
                hits = int((top == l.unsqueeze(1)).any(dim=1).sum())
            self._accumulate(hits, p.shape[0])


class _Confusion:
    """Running k x k confusion matrices (rows: predicted class, cols: true class), local + global."""

    def __init__(self, k=2):
        self.k = k
        self.local = numpy.zeros((k, k))
        self.glob = numpy.zeros((k, k))

    def grow(self, k):
        if k > self.k:
            pad = ((0, k - self.k), (0, k - self.k))
            self.local = numpy.pad(self.local, pad)
            self.glob = numpy.pad(self.glob, pad)
            self.k = k

    def add(self, pred, label):
        self.grow(int(max(pred.max(initial=0), label.max(initial=0))) + 1)
        cm = numpy.zeros((self.k, self.k))
        numpy.add.at(cm, (pred, label), 1)
        self.local += cm
        self.glob += cm

    def clear_local(self):
        self.local = numpy.zeros((self.k, self.k))

    def clear(self):
        self.clear_local()
        self.glob = numpy.zeros((self.k, self.k))


def _binary_counts(cm):
    """(tp, fp, fn, tn) of a 2x2 confusion matrix (class 1 = positive)."""
    return cm[1, 1], cm[1, 0], cm[0, 1], cm[0, 0]


def _f1_of(cm):
    tp, fp, fn, _tn = _binary_counts(cm)
    prec = tp / (tp + fp) if tp + fp > 0 else 0.0
    rec = tp / (tp + fn) if tp + fn > 0 else 0.0
    return 2 * prec * rec / (prec + rec) if prec + rec > 0 else 0.0


def _mcc_binary_of(cm):
    if cm.sum() == 0:
        return 0.0
    tp, fp, fn, tn = _binary_counts(cm)
    denom = 1.0
    for t in (tp + fp, tp + fn, tn + fp, tn + fn):
        if t != 0:
            denom *= t
    return (tp * tn - fp * fn) / math.sqrt(denom)


def _mcc_multiclass_of(cm):
    n = cm.sum()
    pred_tot, true_tot = cm.sum(axis=1), cm.sum(axis=0)
    cov_pp = numpy.sum(pred_tot * (n - pred_tot))
    cov_tt = numpy.sum(true_tot * (n - true_tot))
    if cov_pp == 0 or cov_tt == 0:
        return float('nan')
    cov_pt = numpy.sum(cm.diagonal() * n - pred_tot * true_tot)
    return cov_pt / math.sqrt(cov_pp * cov_tt)


class _BinaryScore(EvalMetric):
    """F1 / MCC over a binary confusion matrix.  'macro': mean of per-batch scores; 'micro': the
    score of all examples seen so far."""

    _score = None

    def __init__(self, name, output_names, label_names, average):
        self.average = average
        self._cm = _Confusion(2)
        super().__init__(name=name, output_names=output_names, label_names=label_names, has_global_stats=True)

    def update(self, labels, preds):
        labels, preds = check_label_shapes(labels, preds, True)
        for label, pred in zip(labels, preds):
            p, l = _host(pred), _host(label).astype('int32').ravel()
            check_label_shapes(l, p)
            if len(numpy.unique(l)) > 2:
                raise ValueError('%s currently only supports binary classification.' % type(self).__name__)
            cls = numpy.argmax(p, axis=1).astype('int64')
            self._cm.grow(2)
            cm = numpy.zeros((2, 2))
            numpy.add.at(cm, ((cls == 1).astype('int64'), (l == 1).astype('int64')), 1)
            self._cm.local += cm
            self._cm.glob += cm
        score = type(self)._score
        if self.average == 'macro':
            self._accumulate(score(self._cm.local), 1)    # local == global here: both hold this batch
            self._cm.clear()
        else:
            nl, ng = self._cm.local.sum(), self._cm.glob.sum()
            self.sum_metric, self.num_inst = score(self._cm.local) * nl, nl
            self.global_sum_metric, self.global_num_inst = score(self._cm.glob) * ng, ng

    def reset_local(self):
        super().reset_local()
        if hasattr(self, '_cm'):
            self._cm.clear_local()

    def reset(self):
        super().reset()
        if hasattr(self, '_cm'):
            self._cm.clear()


@register
class F1(_BinaryScore):
    _score = staticmethod(_f1_of)

    def __init__(self, name='f1', output_names=None, label_names=None, average='macro'):
        super().__init__(name, output_names, label_names, average)


@register
class MCC(_BinaryScore):
    _score = staticmethod(_mcc_binary_of)

    def __init__(self, name='mcc', output_names=None, label_names=None, average='macro'):
        super().__init__(name, output_names, label_names, average)


@register
class PCC(EvalMetric):
    """Multi-class Matthews correlation (Gorodkin's R_K) over a growing confusion matrix."""

    def __init__(self, name='pcc', output_names=None, label_names=None, has_global_stats=True):
        self._cm = _Confusion(2)
        super().__init__(name=name, output_names=output_names, label_names=label_names,
                         has_global_stats=has_global_stats)

    @property
    def k(self):
        return self._cm.k

    def update(self, labels, preds):
        labels, preds = check_label_shapes(labels, preds, True)
        for label, pred in zip(labels, preds):
            l = _host(label).astype('int32', copy=False).ravel()
            p = _host(pred)
            if p.shape != l.shape:
                p = (p.ravel() > 0.5) if p.shape[-1] == 1 else p.argmax(axis=1)
            self._cm.add(p.astype('int64').ravel(), l.astype('int64'))
        self.num_inst += 1
        self.global_num_inst += 1

    # sums are derived from the confusion matrices, never assigned
    sum_metric = property(lambda self: _mcc_multiclass_of(self._cm.local) * self.num_inst, lambda self, v: None)
    global_sum_metric = property(lambda self: _mcc_multiclass_of(self._cm.glob) * self.global_num_inst,
                                 lambda self, v: None)

    def reset_local(self):
        self.num_inst = 0
        if hasattr(self, '_cm'):
            self._cm.clear_local()

    def reset(self):
        self.reset_local()
        self.global_num_inst = 0
        if hasattr(self, '_cm'):
            self._cm.clear()


# ------------------------------------------------------------------------ probabilistic
@register
class Perplexity(EvalMetric):
    """exp(mean negative log-likelihood of the labels), ignoring ``ignore_label`` positions."""

    def __init__(self, ignore_label, axis=-1, name='perplexity', output_names=None, label_names=None):
        super().__init__(name, ignore_label=ignore_label, output_names=output_names, label_names=label_names,
                         has_global_stats=True)
        self.ignore_label = ignore_label
        self.axis = axis

    def update(self, labels, preds):
        if len(labels) != len(preds):
            raise AssertionError('labels and preds differ in length')
        nll, count = 0.0, 0
        for label, pred in zip(labels, preds):
            p = _dev(pred)
            if label.size != p.numel() // p.shape[-1]:
                raise AssertionError('shape mismatch: %s vs. %s' % (label.shape, tuple(p.shape)))
            l = _dev(label).to(p.device).reshape(-1).to(torch.int64)
            # pick() semantics of the reference (mode='clip'): out-of-range labels read the edge class
            prob = p.reshape(-1, p.shape[-1]).float().gather(
                1, l.clamp(min=0, max=p.shape[-1] - 1).unsqueeze(1)).squeeze(1)
            keep = torch.ones_like(prob, dtype=torch.bool) if self.ignore_label is None else l != self.ignore_label
            prob = torch.where(keep, prob, torch.ones_like(prob))
            nll -= float(torch.log(prob.clamp(min=1e-10)).sum())
            count += int(keep.sum())
        self._accumulate(nll, count)

    def _value(self, total, count):
        return float('nan') if count == 0 else math.exp(total / count)


class _PickedNLL(EvalMetric):
    """Sum of -log(p[label] + eps) over examples (CrossEntropy / NLL)."""

    def __init__(self, eps, name, output_names, label_names):
        super().__init__(name, eps=eps, output_names=output_names, label_names=label_names, has_global_stats=True)
        self.eps = eps

    def update(self, labels, preds):
        labels, preds = check_label_shapes(labels, preds, True)
        for label, pred in zip(labels, preds):
            p = _dev(pred)
            l = _dev(label).reshape(-1).to(device=p.device, dtype=torch.int64)
            if l.shape[0] != p.shape[0]:
                raise AssertionError('labels (%d) and predictions (%d) differ in count' % (l.shape[0], p.shape[0]))
            picked = p.double()[torch.arange(l.shape[0], device=p.device), l]
            self._accumulate(float(-torch.log(picked + self.eps).sum()), int(l.shape[0]))


@register
@alias('ce')
class CrossEntropy(_PickedNLL):
    def __init__(self, eps=1e-12, name='cross-entropy', output_names=None, label_names=None):
        super().__init__(eps, name, output_names, label_names)


@register
@alias('nll_loss')
class NegativeLogLikelihood(_PickedNLL):
    def __init__(self, eps=1e-12, name='nll-loss', output_names=None, label_names=None):
        super().__init__(eps, name, output_names, label_names)


# ------------------------------------------------------------------------ regression
class _Regression(EvalMetric):
    """Per-batch error statistic of (label, pred) as 2-D column arrays, averaged over batches."""

    def _stat(self, diff):
        raise NotImplementedError

    def __init__(self, name, output_names, label_names):
        super().__init__(name, output_names=output_names, label_names=label_names, has_global_stats=True)

    def update(self, labels, preds):
        labels, preds = check_label_shapes(labels, preds, True)
        for label, pred in zip(labels, preds):
            l, p = _host(label), _host(pred)
            l = l.reshape(l.shape[0], 1) if l.ndim == 1 else l
            p = p.reshape(p.shape[0], 1) if p.ndim == 1 else p
            self._accumulate(self._stat(l - p), 1)


@register
class MAE(_Regression):
    def __init__(self, name='mae', output_names=None, label_names=None):
        super().__init__(name, output_names, label_names)

    def _stat(self, diff):
        return numpy.abs(diff).mean()


@register
class MSE(_Regression):
    def __init__(self, name='mse', output_names=None, label_names=None):
        super().__init__(name, output_names, label_names)

    def _stat(self, diff):
        return numpy.square(diff).mean()


@register
class RMSE(_Regression):
    def __init__(self, name='rmse', output_names=None, label_names=None):
        super().__init__(name, output_names, label_names)

    def _stat(self, diff):
        return numpy.sqrt(numpy.square(diff).mean())


@register
@alias('pearsonr')
class PearsonCorrelation(EvalMetric):
    """Pearson r.  'macro': mean of per-batch correlations; 'micro': one correlation over all
    values seen, from running (Welford) means / second moments and co-moment."""

    def __init__(self, name='pearsonr', output_names=None, label_names=None, average='macro'):
        self.average = average
        super().__init__(name, output_names=output_names, label_names=label_names, has_global_stats=True)

    def _reset_moments(self):
        self._n = 0
        self._mean_l = self._mean_p = 0.0
        self._m2_l = self._m2_p = 0.0
        self._co = 0.0

    def reset(self):
        super().reset()
        if self.average == 'micro':
            self._reset_moments()

    reset_micro = _reset_moments

    @staticmethod
    def _welford(x, n, mean, m2):
        n2 = n + len(x)
        d = x - mean
        mean2 = mean + numpy.sum(d / n2)
        return n2, mean2, m2 + numpy.sum(d * (x - mean2))

    def update(self, labels, preds):
        labels, preds = check_label_shapes(labels, preds, True)
        for label, pred in zip(labels, preds):
            check_label_shapes(label, pred, False, True)
            l = _host(label).ravel().astype(numpy.float64)
            p = _host(pred).ravel().astype(numpy.float64)
            if self.average == 'macro':
                self._accumulate(numpy.corrcoef(p, l)[0, 1], 1)
                continue
            self.num_inst += 1
            self.global_num_inst += 1
            n, self._mean_l, self._m2_l = self._welford(l, self._n, self._mean_l, self._m2_l)
            # co-moment against the label mean AFTER this batch and the prediction mean BEFORE it
            self._co += numpy.sum((l - self._mean_l) * (p - self._mean_p))
            _, self._mean_p, self._m2_p = self._welford(p, self._n, self._mean_p, self._m2_p)
            self._n = n

    def get(self):
        if self.num_inst == 0:
            return self.name, float('nan')
        if self.average == 'macro':
            return self.name, self.sum_metric / self.num_inst
        dof = self._n - 1
        return self.name, self._co / (dof * numpy.sqrt(self._m2_p / dof) * numpy.sqrt(self._m2_l / dof))


# ------------------------------------------------------------------------ losses / custom
@register
class Loss(EvalMetric):
    """Mean of the loss values given as predictions (labels are ignored)."""

    def __init__(self, name='loss', output_names=None, label_names=None):
        super().__init__(name, output_names=output_names, label_names=label_names, has_global_stats=True)

    def update(self, _, preds):
        for pred in ([preds] if isinstance(preds, NDArray) else preds):
            total = float(pred._data.detach().double().sum()) if isinstance(pred, NDArray) else float(numpy.sum(pred))
            self._accumulate(total, pred.size)


@register
class Torch(Loss):
    def __init__(self, name='torch', output_names=None, label_names=None):
        super().__init__(name, output_names=output_names, label_names=label_names)


@register
class Caffe(Loss):
    def __init__(self, name='caffe', output_names=None, label_names=None):
        super().__init__(name, output_names=output_names, label_names=label_names)


@register
class CustomMetric(EvalMetric):
    """Metric from ``feval(label_np, pred_np)`` returning a value or ``(sum, count)``."""

    def __init__(self, feval, name=None, allow_extra_outputs=False, output_names=None, label_names=None):
        if name is None:
            name = feval.__name__
            name = 'custom(%s)' % name if '<' in name else name
        super().__init__(name, feval=feval, allow_extra_outputs=allow_extra_outputs, output_names=output_names,
                         label_names=label_names, has_global_stats=True)
        self._feval = feval
        self._allow_extra_outputs = allow_extra_outputs

    def update(self, labels, preds):
        if not self._allow_extra_outputs:
            labels, preds = check_label_shapes(labels, preds, True)
        for pred, label in zip(preds, labels):
            res = self._feval(_host(label), _host(pred))
            self._accumulate(*(res if isinstance(res, tuple) else (res, 1)))

    def get_config(self):
        raise NotImplementedError('CustomMetric cannot be serialized')


def np(numpy_feval, name=None, allow_extra_outputs=False):
    """CustomMetric from a function of numpy arrays."""
    def feval(label, pred):
        return numpy_feval(label, pred)
    feval.__name__ = numpy_feval.__name__
    return CustomMetric(feval, name, allow_extra_outputs)
