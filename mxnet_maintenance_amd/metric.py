"""Evaluation metrics.

Parity: python/mxnet/metric.py (EvalMetric, CompositeEvalMetric, Accuracy,
TopKAccuracy, F1, MCC, Perplexity, MAE, MSE, RMSE, CrossEntropy,
NegativeLogLikelihood, PearsonCorrelation, PCC, Loss, Torch, Caffe,
CustomMetric, np, create, register, check_label_shapes).
Accuracy/TopK reduce on the device and transfer one scalar per update.
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
    if not shape:
        label_shape, pred_shape = len(labels), len(preds)
    else:
        label_shape, pred_shape = labels.shape, preds.shape
    if label_shape != pred_shape:
        raise ValueError('Shape of labels {} does not match shape of predictions {}'.format(label_shape, pred_shape))
    if wrap:
        if isinstance(labels, (NDArray, numpy.ndarray)):
            labels = [labels]
        if isinstance(preds, (NDArray, numpy.ndarray)):
            preds = [preds]
    return labels, preds


def _np(x):
    if isinstance(x, NDArray):
        return x.asnumpy()
    return numpy.asarray(x)


class EvalMetric:
    """Base class for all evaluation metrics."""

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
        config = self._kwargs.copy()
        config.update({'metric': self.__class__.__name__, 'name': self.name, 'output_names': self.output_names,
                       'label_names': self.label_names})
        return config

    def update_dict(self, label, pred):
        if self.output_names is not None:
            pred = [pred[name] for name in self.output_names]
        else:
            pred = list(pred.values())
        if self.label_names is not None:
            label = [label[name] for name in self.label_names]
        else:
            label = list(label.values())
        self.update(label, pred)

    def update(self, labels, preds):
        raise NotImplementedError()

    def reset(self):
        self.num_inst = 0
        self.sum_metric = 0.0
        self.global_num_inst = 0
        self.global_sum_metric = 0.0

    def reset_local(self):
        self.num_inst = 0
        self.sum_metric = 0.0

    def get(self):
        if self.num_inst == 0:
            return (self.name, float('nan'))
        return (self.name, self.sum_metric / self.num_inst)

    def get_global(self):
        if self._has_global_stats:
            if self.global_num_inst == 0:
                return (self.name, float('nan'))
            return (self.name, self.global_sum_metric / self.global_num_inst)
        return self.get()

    def get_name_value(self):
        name, value = self.get()
        if not isinstance(name, list):
            name = [name]
        if not isinstance(value, list):
            value = [value]
        return list(zip(name, value))

    def get_global_name_value(self):
        if self._has_global_stats:
            name, value = self.get_global()
            if not isinstance(name, list):
                name = [name]
            if not isinstance(value, list):
                value = [value]
            return list(zip(name, value))
        return self.get_name_value()

    def _add(self, s, n):
        self.sum_metric += s
        self.global_sum_metric += s
        self.num_inst += n
        self.global_num_inst += n


_METRICS = {}


def register(klass):
    _METRICS[klass.__name__.lower()] = klass
    return klass


def alias(*aliases):
    def reg(klass):
        for a in aliases:
            _METRICS[a.lower()] = klass
        return klass
    return reg


def create(metric, *args, **kwargs):
    if callable(metric) and not isinstance(metric, type):
        return CustomMetric(metric, *args, **kwargs)
    if isinstance(metric, list):
        composite_metric = CompositeEvalMetric()
        for child_metric in metric:
            composite_metric.add(create(child_metric, *args, **kwargs))
        return composite_metric
    if isinstance(metric, EvalMetric):
        return metric
    if isinstance(metric, type) and issubclass(metric, EvalMetric):
        return metric(*args, **kwargs)
    return _METRICS[metric.lower()](*args, **kwargs)


@register
@alias('composite')
class CompositeEvalMetric(EvalMetric):
    def __init__(self, metrics=None, name='composite', output_names=None, label_names=None):
        super().__init__(name, output_names=output_names, label_names=label_names, has_global_stats=True)
        if metrics is None:
            metrics = []
        self.metrics = [create(i) for i in metrics]

    def add(self, metric):
        self.metrics.append(create(metric))

    def get_metric(self, index):
        try:
            return self.metrics[index]
        except IndexError:
            return ValueError('Metric index {} is out of range 0 and {}'.format(index, len(self.metrics)))

    def update_dict(self, labels, preds):
        if self.label_names is not None:
            labels = OrderedDict([i for i in labels.items() if i[0] in self.label_names])
        if self.output_names is not None:
            preds = OrderedDict([i for i in preds.items() if i[0] in self.output_names])
        for metric in self.metrics:
            metric.update_dict(labels, preds)

    def update(self, labels, preds):
        for metric in self.metrics:
            metric.update(labels, preds)

    def reset(self):
        try:
            for metric in self.metrics:
                metric.reset()
        except AttributeError:
            pass

    def reset_local(self):
        try:
            for metric in self.metrics:
                metric.reset_local()
        except AttributeError:
            pass

    def get(self):
        names, values = [], []
        for metric in self.metrics:
            name, value = metric.get()
            if isinstance(name, string_types):
                name = [name]
            if isinstance(value, numeric_types):
                value = [value]
            names.extend(name)
            values.extend(value)
        return (names, values)

    def get_global(self):
        names, values = [], []
        for metric in self.metrics:
            name, value = metric.get_global()
            if isinstance(name, string_types):
                name = [name]
            if isinstance(value, numeric_types):
                value = [value]
            names.extend(name)
            values.extend(value)
        return (names, values)

    def get_config(self):
        config = super().get_config()
        config.update({'metrics': [i.get_config() for i in self.metrics]})
        return config


@register
@alias('acc')
class Accuracy(EvalMetric):
    def __init__(self, axis=1, name='accuracy', output_names=None, label_names=None):
        super().__init__(name, axis=axis, output_names=output_names, label_names=label_names,
                         has_global_stats=True)
        self.axis = axis

    def update(self, labels, preds):
        labels, preds = check_label_shapes(labels, preds, True)
        for label, pred_label in zip(labels, preds):
            if isinstance(pred_label, NDArray) and isinstance(label, NDArray):
                p = pred_label._data
                l = label._data
                if p.shape != l.shape:
                    p = torch.argmax(p, dim=self.axis)
                p = p.reshape(-1).to(torch.int64)
                l = l.reshape(-1).to(torch.int64).to(p.device)
                if p.numel() != l.numel():
                    raise ValueError('Shape of labels {} does not match shape of predictions {}'.format(
                        l.shape, p.shape))
                correct = int((p == l).sum())
                self._add(correct, int(l.numel()))
                continue
            pred_label = _np(pred_label)
            label = _np(label)
            if pred_label.shape != label.shape:
                pred_label = numpy.argmax(pred_label, axis=self.axis)
            pred_label = pred_label.astype('int64').flat
            label = label.astype('int64').flat
            check_label_shapes(label, pred_label)
            num_correct = (numpy.asarray(pred_label) == numpy.asarray(label)).sum()
            self._add(num_correct, len(pred_label))


@register
@alias('top_k_accuracy', 'top_k_acc')
class TopKAccuracy(EvalMetric):
    def __init__(self, top_k=1, name='top_k_accuracy', output_names=None, label_names=None):
        super().__init__(name, top_k=top_k, output_names=output_names, label_names=label_names,
                         has_global_stats=True)
        self.top_k = top_k
        assert self.top_k > 1, 'Please use Accuracy if top_k is no more than 1'
        self.name += '_%d' % self.top_k

    def update(self, labels, preds):
        labels, preds = check_label_shapes(labels, preds, True)
        for label, pred_label in zip(labels, preds):
            assert len(pred_label.shape) <= 2, 'Predictions should be no more than 2 dims'
            pred_label = numpy.argpartition(_np(pred_label).astype('float32'), -self.top_k)
            label = _np(label).astype('int32')
            check_label_shapes(label, pred_label)
            num_samples = pred_label.shape[0]
            num_dims = len(pred_label.shape)
            if num_dims == 1:
                self._add((pred_label.flat == label.flat).sum(), num_samples)
            elif num_dims == 2:
                num_classes = pred_label.shape[1]
                top_k = min(num_classes, self.top_k)
                s = 0
                for j in range(top_k):
                    s += (pred_label[:, num_classes - 1 - j].flat == label.flat).sum()
                self._add(s, num_samples)


class _BinaryClassificationMetrics:
    def __init__(self):
        self.true_positives = 0
        self.false_negatives = 0
        self.false_positives = 0
        self.true_negatives = 0
        self.global_true_positives = 0
        self.global_false_negatives = 0
        self.global_false_positives = 0
        self.global_true_negatives = 0

    def update_binary_stats(self, label, pred):
        pred = _np(pred)
        label = _np(label).astype('int32')
        pred_label = numpy.argmax(pred, axis=1)
        check_label_shapes(label, pred)
        if len(numpy.unique(label)) > 2:
            raise ValueError('%s currently only supports binary classification.' % self.__class__.__name__)
        pred_true = (pred_label == 1)
        pred_false = 1 - pred_true
        label_true = (label == 1)
        label_false = 1 - label_true
        tp = (pred_true * label_true).sum()
        fp = (pred_true * label_false).sum()
        fn = (pred_false * label_true).sum()
        tn = (pred_false * label_false).sum()
        self.true_positives += tp
        self.global_true_positives += tp
        self.false_positives += fp
        self.global_false_positives += fp
        self.false_negatives += fn
        self.global_false_negatives += fn
        self.true_negatives += tn
        self.global_true_negatives += tn

    @property
    def precision(self):
        d = self.true_positives + self.false_positives
        return float(self.true_positives) / d if d > 0 else 0.

    @property
    def global_precision(self):
        d = self.global_true_positives + self.global_false_positives
        return float(self.global_true_positives) / d if d > 0 else 0.

    @property
    def recall(self):
        d = self.true_positives + self.false_negatives
        return float(self.true_positives) / d if d > 0 else 0.

    @property
    def global_recall(self):
        d = self.global_true_positives + self.global_false_negatives
        return float(self.global_true_positives) / d if d > 0 else 0.

    @property
    def fscore(self):
        if self.precision + self.recall > 0:
            return 2 * self.precision * self.recall / (self.precision + self.recall)
        return 0.

    @property
    def global_fscore(self):
        if self.global_precision + self.global_recall > 0:
            return 2 * self.global_precision * self.global_recall / (self.global_precision + self.global_recall)
        return 0.

    def matthewscc(self, use_global=False):
        if use_global:
            if not self.global_total_examples:
                return 0.
            tp, fp, fn, tn = map(float, (self.global_true_positives, self.global_false_positives,
                                         self.global_false_negatives, self.global_true_negatives))
        else:
            if not self.total_examples:
                return 0.
            tp, fp, fn, tn = map(float, (self.true_positives, self.false_positives, self.false_negatives,
                                         self.true_negatives))
        terms = [(tp + fp), (tp + fn), (tn + fp), (tn + fn)]
        denom = 1.
        for t in filter(lambda t: t != 0., terms):
            denom *= t
        return ((tp * tn) - (fp * fn)) / math.sqrt(denom)

    @property
    def total_examples(self):
        return self.false_negatives + self.false_positives + self.true_negatives + self.true_positives

    @property
    def global_total_examples(self):
        return (self.global_false_negatives + self.global_false_positives + self.global_true_negatives +
                self.global_true_positives)

    def local_reset_stats(self):
        self.false_positives = 0
        self.false_negatives = 0
        self.true_positives = 0
        self.true_negatives = 0

    def reset_stats(self):
        self.local_reset_stats()
        self.global_false_positives = 0
        self.global_false_negatives = 0
        self.global_true_positives = 0
        self.global_true_negatives = 0


@register
class F1(EvalMetric):
    def __init__(self, name='f1', output_names=None, label_names=None, average='macro'):
        self.average = average
        self.metrics = _BinaryClassificationMetrics()
        super().__init__(name=name, output_names=output_names, label_names=label_names, has_global_stats=True)

    def update(self, labels, preds):
        labels, preds = check_label_shapes(labels, preds, True)
        for label, pred in zip(labels, preds):
            self.metrics.update_binary_stats(label, pred)
        if self.average == 'macro':
            self.sum_metric += self.metrics.fscore
            self.global_sum_metric += self.metrics.global_fscore
            self.num_inst += 1
            self.global_num_inst += 1
            self.metrics.reset_stats()
        else:
            self.sum_metric = self.metrics.fscore * self.metrics.total_examples
            self.global_sum_metric = self.metrics.global_fscore * self.metrics.global_total_examples
            self.num_inst = self.metrics.total_examples
            self.global_num_inst = self.metrics.global_total_examples

    def reset(self):
        self.sum_metric = 0.
        self.num_inst = 0
        self.global_num_inst = 0
        self.global_sum_metric = 0.0
        self.metrics.reset_stats()

    def reset_local(self):
        self.sum_metric = 0.
        self.num_inst = 0
        self.metrics.local_reset_stats()


@register
class MCC(EvalMetric):
    def __init__(self, name='mcc', output_names=None, label_names=None, average='macro'):
        self._average = average
        self._metrics = _BinaryClassificationMetrics()
        super().__init__(name=name, output_names=output_names, label_names=label_names, has_global_stats=True)

    def update(self, labels, preds):
        labels, preds = check_label_shapes(labels, preds, True)
        for label, pred in zip(labels, preds):
            self._metrics.update_binary_stats(label, pred)
        if self._average == 'macro':
            self.sum_metric += self._metrics.matthewscc()
            self.global_sum_metric += self._metrics.matthewscc(use_global=True)
            self.num_inst += 1
            self.global_num_inst += 1
            self._metrics.reset_stats()
        else:
            self.sum_metric = self._metrics.matthewscc() * self._metrics.total_examples
            self.global_sum_metric = self._metrics.matthewscc(use_global=True) * self._metrics.global_total_examples
            self.num_inst = self._metrics.total_examples
            self.global_num_inst = self._metrics.global_total_examples

    def reset(self):
        self.sum_metric = 0.
        self.num_inst = 0.
        self.global_sum_metric = 0.
        self.global_num_inst = 0.
        self._metrics.reset_stats()

    def reset_local(self):
        self.sum_metric = 0.
        self.num_inst = 0.
        self._metrics.local_reset_stats()


@register
class Perplexity(EvalMetric):
    def __init__(self, ignore_label, axis=-1, name='perplexity', output_names=None, label_names=None):
        super().__init__(name, ignore_label=ignore_label, output_names=output_names, label_names=label_names,
                         has_global_stats=True)
        self.ignore_label = ignore_label
        self.axis = axis

    def update(self, labels, preds):
        assert len(labels) == len(preds)
        loss = 0.
        num = 0
        for label, pred in zip(labels, preds):
            assert label.size == pred.size / pred.shape[-1], \
                'shape mismatch: %s vs. %s' % (label.shape, pred.shape)
            p = pred._data if isinstance(pred, NDArray) else torch.as_tensor(numpy.asarray(pred))
            l = label._data if isinstance(label, NDArray) else torch.as_tensor(numpy.asarray(label))
            l = l.to(p.device).reshape(-1).to(torch.int64)
            prob = torch.gather(p.reshape(-1, p.shape[-1]).float(), 1, l.clamp(min=0).unsqueeze(1)).reshape(-1)
            if self.ignore_label is not None:
                ignore = (l == self.ignore_label).to(prob.dtype)
                num -= int(ignore.sum())
                prob = prob * (1 - ignore) + ignore
            loss -= float(torch.sum(torch.log(torch.clamp(prob, min=1e-10))))
            num += prob.numel()
        self._add(loss, num)

    def get(self):
        if self.num_inst == 0:
            return (self.name, float('nan'))
        return (self.name, math.exp(self.sum_metric / self.num_inst))

    def get_global(self):
        if self.global_num_inst == 0:
            return (self.name, float('nan'))
        return (self.name, math.exp(self.global_sum_metric / self.global_num_inst))


def _reg_metric(fn):
    def update(self, labels, preds):
        labels, preds = check_label_shapes(labels, preds, True)
        for label, pred in zip(labels, preds):
            label = _np(label)
            pred = _np(pred)
            if len(label.shape) == 1:
                label = label.reshape(label.shape[0], 1)
            if len(pred.shape) == 1:
                pred = pred.reshape(pred.shape[0], 1)
            self._add(fn(label, pred), 1)
    return update


@register
class MAE(EvalMetric):
    def __init__(self, name='mae', output_names=None, label_names=None):
        super().__init__(name, output_names=output_names, label_names=label_names, has_global_stats=True)

    update = _reg_metric(lambda l, p: numpy.abs(l - p).mean())


@register
class MSE(EvalMetric):
    def __init__(self, name='mse', output_names=None, label_names=None):
        super().__init__(name, output_names=output_names, label_names=label_names, has_global_stats=True)

    update = _reg_metric(lambda l, p: ((l - p) ** 2.0).mean())


@register
class RMSE(EvalMetric):
    def __init__(self, name='rmse', output_names=None, label_names=None):
        super().__init__(name, output_names=output_names, label_names=label_names, has_global_stats=True)

    update = _reg_metric(lambda l, p: numpy.sqrt(((l - p) ** 2.0).mean()))


@register
@alias('ce')
class CrossEntropy(EvalMetric):
    def __init__(self, eps=1e-12, name='cross-entropy', output_names=None, label_names=None):
        super().__init__(name, eps=eps, output_names=output_names, label_names=label_names, has_global_stats=True)
        self.eps = eps

    def update(self, labels, preds):
        labels, preds = check_label_shapes(labels, preds, True)
        for label, pred in zip(labels, preds):
            label = _np(label)
            pred = _np(pred)
            label = label.ravel()
            assert label.shape[0] == pred.shape[0]
            prob = pred[numpy.arange(label.shape[0]), numpy.int64(label)]
            self._add((-numpy.log(prob + self.eps)).sum(), label.shape[0])


@register
@alias('nll_loss')
class NegativeLogLikelihood(EvalMetric):
    def __init__(self, eps=1e-12, name='nll-loss', output_names=None, label_names=None):
        super().__init__(name, eps=eps, output_names=output_names, label_names=label_names, has_global_stats=True)
        self.eps = eps

    def update(self, labels, preds):
        labels, preds = check_label_shapes(labels, preds, True)
        for label, pred in zip(labels, preds):
            label = _np(label)
            pred = _np(pred)
            label = label.ravel()
            num_examples = pred.shape[0]
            assert label.shape[0] == num_examples, (label.shape[0], num_examples)
            prob = pred[numpy.arange(num_examples, dtype=numpy.int64), numpy.int64(label)]
            self._add((-numpy.log(prob + self.eps)).sum(), num_examples)


@register
@alias('pearsonr')
class PearsonCorrelation(EvalMetric):
    def __init__(self, name='pearsonr', output_names=None, label_names=None, average='macro'):
        self.average = average
        super().__init__(name, output_names=output_names, label_names=label_names, has_global_stats=True)
        if self.average == 'micro':
            self.reset_micro()

    def reset_micro(self):
        self._sse_p = 0
        self._mean_p = 0
        self._sse_l = 0
        self._mean_l = 0
        self._pred_nums = 0
        self._label_nums = 0
        self._conv = 0

    def reset(self):
        self.num_inst = 0
        self.sum_metric = 0.0
        self.global_num_inst = 0
        self.global_sum_metric = 0.0
        if self.average == 'micro':
            self.reset_micro()

    def update_variance(self, new_values, *aggregate):
        count, mean, m_2 = aggregate
        count += len(new_values)
        delta = new_values - mean
        mean += numpy.sum(delta / count)
        delta_2 = new_values - mean
        m_2 += numpy.sum(delta * delta_2)
        return count, mean, m_2

    def update_cov(self, label, pred):
        self._conv = self._conv + numpy.sum((label - self._mean_l) * (pred - self._mean_p))

    def update(self, labels, preds):
        labels, preds = check_label_shapes(labels, preds, True)
        for label, pred in zip(labels, preds):
            check_label_shapes(label, pred, False, True)
            label = _np(label).ravel().astype(numpy.float64)
            pred = _np(pred).ravel().astype(numpy.float64)
            if self.average == 'macro':
                pearson_corr = numpy.corrcoef(pred, label)[0, 1]
                self._add(pearson_corr, 1)
            else:
                self.global_num_inst += 1
                self.num_inst += 1
                self._label_nums, self._mean_l, self._sse_l = self.update_variance(
                    label, self._label_nums, self._mean_l, self._sse_l)
                self.update_cov(label, pred)
                self._pred_nums, self._mean_p, self._sse_p = self.update_variance(
                    pred, self._pred_nums, self._mean_p, self._sse_p)

    def get(self):
        if self.num_inst == 0:
            return (self.name, float('nan'))
        if self.average == 'macro':
            return (self.name, self.sum_metric / self.num_inst)
        n = self._label_nums
        pearsonr = self._conv / ((n - 1) * numpy.sqrt(self._sse_p / (n - 1)) * numpy.sqrt(self._sse_l / (n - 1)))
        return (self.name, pearsonr)


@register
class PCC(EvalMetric):
    def __init__(self, name='pcc', output_names=None, label_names=None, has_global_stats=True):
        self.k = 2
        super().__init__(name=name, output_names=output_names, label_names=label_names,
                         has_global_stats=has_global_stats)

    def _grow(self, inc):
        self.lcm = numpy.pad(self.lcm, ((0, inc), (0, inc)), 'constant', constant_values=(0))
        self.gcm = numpy.pad(self.gcm, ((0, inc), (0, inc)), 'constant', constant_values=(0))
        self.k += inc

    def _calc_mcc(self, cmat):
        n = cmat.sum()
        x = cmat.sum(axis=1)
        y = cmat.sum(axis=0)
        cov_xx = numpy.sum(x * (n - x))
        cov_yy = numpy.sum(y * (n - y))
        if cov_xx == 0 or cov_yy == 0:
            return float('nan')
        i = cmat.diagonal()
        cov_xy = numpy.sum(i * n - x * y)
        return cov_xy / (cov_xx * cov_yy) ** 0.5

    def update(self, labels, preds):
        labels, preds = check_label_shapes(labels, preds, True)
        for label, pred in zip(labels, preds):
            label = _np(label).astype('int32', copy=False).ravel()
            pred = _np(pred)
            if pred.shape != label.shape:
                if pred.shape[-1] == 1:
                    pred = (pred.ravel() > 0.5).astype('int32')
                else:
                    pred = pred.argmax(axis=1)
            pred = pred.astype('int32', copy=False).ravel()
            n = max(pred.max(), label.max())
            if n >= self.k:
                self._grow(n + 1 - self.k)
            bcm = numpy.zeros((self.k, self.k))
            for i, j in zip(pred, label):
                bcm[i, j] += 1
            self.lcm += bcm
            self.gcm += bcm
        self.num_inst += 1
        self.global_num_inst += 1

    @property
    def sum_metric(self):
        return self._calc_mcc(self.lcm) * self.num_inst

    @sum_metric.setter
    def sum_metric(self, v):
        pass

    @property
    def global_sum_metric(self):
        return self._calc_mcc(self.gcm) * self.global_num_inst

    @global_sum_metric.setter
    def global_sum_metric(self, v):
        pass

    def reset(self):
        self.global_num_inst = 0.
        self.gcm = numpy.zeros((self.k, self.k))
        self.reset_local()

    def reset_local(self):
        self.num_inst = 0.
        self.lcm = numpy.zeros((self.k, self.k))


@register
class Loss(EvalMetric):
    """Mean of the given loss values."""

    def __init__(self, name='loss', output_names=None, label_names=None):
        super().__init__(name, output_names=output_names, label_names=label_names, has_global_stats=True)

    def update(self, _, preds):
        if isinstance(preds, NDArray):
            preds = [preds]
        for pred in preds:
            if isinstance(pred, NDArray):
                loss = float(pred._data.detach().float().sum())
            else:
                loss = float(numpy.sum(pred))
            self._add(loss, pred.size)


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
    def __init__(self, feval, name=None, allow_extra_outputs=False, output_names=None, label_names=None):
        if name is None:
            name = feval.__name__
            if name.find('<') != -1:
                name = 'custom(%s)' % name
        super().__init__(name, feval=feval, allow_extra_outputs=allow_extra_outputs, output_names=output_names,
                         label_names=label_names, has_global_stats=True)
        self._feval = feval
        self._allow_extra_outputs = allow_extra_outputs

    def update(self, labels, preds):
        if not self._allow_extra_outputs:
            labels, preds = check_label_shapes(labels, preds, True)
        for pred, label in zip(preds, labels):
            label = _np(label)
            pred = _np(pred)
            reval = self._feval(label, pred)
            if isinstance(reval, tuple):
                (sum_metric, num_inst) = reval
                self._add(sum_metric, num_inst)
            else:
                self._add(reval, 1)

    def get_config(self):
        raise NotImplementedError('CustomMetric cannot be serialized')


def np(numpy_feval, name=None, allow_extra_outputs=False):
    def feval(label, pred):
        return numpy_feval(label, pred)
    feval.__name__ = numpy_feval.__name__
    return CustomMetric(feval, name, allow_extra_outputs)
