"""BaseModule: the intermediate-level (symbolic) training interface.

API parity: python/mxnet/module/base_module.py.  A concrete module provides the
primitive operations (``bind``, ``init_params``, ``init_optimizer``,
``forward``, ``backward``, ``update``, ``get_outputs``, ``update_metric``, ...);
this base class builds the driver loops on top of them:

* ``_walk`` -- the shared "iterate an eval iterator for at most N batches,
  preparing and forwarding each" generator behind ``score``,
  ``iter_predict`` and ``predict``;
* ``fit`` -- bind / init / optimizer set-up, then ``_train_epoch`` per epoch
  (which prefetches the next batch and calls ``prepare`` on it while the
  current one is being consumed) and the epoch-end bookkeeping.
"""
import logging
import time

import numpy as np

from .. import metric
from .. import ndarray as nd
from ..initializer import Uniform
from ..model import BatchEndParam
from ..ndarray.ndarray import NDArray

__all__ = ['BaseModule', 'BatchEndParam']


def _as_list(obj):
    return obj if isinstance(obj, list) else [obj]


def _fire(callbacks, *args):
    for cb in _as_list(callbacks) if callbacks is not None else ():
        cb(*args)


def _warn_or_raise(msg, throw):
    if throw:
        raise ValueError(msg)
    logging.warning(msg)


def _looks_like_param(name):
    return name.endswith(('_weight', '_bias', '_gamma', '_beta'))


def _check_input_names(symbol, names, typename, throw):
    """Every declared input name must be an argument of ``symbol``; suggest the plausible ones."""
    args = symbol.list_arguments()
    for name in names:
        if name not in args:
            hints = '\n\t'.join(a for a in args if not _looks_like_param(a))
            _warn_or_raise("Module(..., %s_names=%s): input '%s' is not an argument of the symbol. "
                           'Did you mean one of:\n\t%s' % (typename, list(names), name, hints), throw)


def _check_names_match(expected, descs, kind, throw):
    got = [d[0] for d in descs]
    if sorted(expected) != sorted(got):
        _warn_or_raise('%s_shapes %s do not match the declared %s_names %s' % (kind, descs, kind, list(expected)),
                       throw)


def _as_descs(shapes):
    from ..io import DataDesc
    return None if shapes is None else [s if isinstance(s, DataDesc) else DataDesc(*s) for s in shapes]


def _parse_data_desc(data_names, label_names, data_shapes, label_shapes):
    """Normalise (name, shape) pairs to DataDesc and validate them against the declared names."""
    data_shapes = _as_descs(data_shapes)
    label_shapes = _as_descs(label_shapes)
    _check_names_match(data_names, data_shapes, 'data', True)
    _check_names_match(label_names, label_shapes or [], 'label', False)
    return data_shapes, label_shapes


def _batch_labels(batch):
    """(labels, pre_sliced) of a batch, or of a list of per-device batches."""
    if isinstance(batch, list):
        return [b.label for b in batch], True
    return batch.label, False


class _SimpleBatch:
    """Minimal DataBatch used by ``predict`` on a bare array."""

    def __init__(self, data, label=None):
        self.data = data
        self.label = label
        self.pad = 0
        self.bucket_key = None
        self.provide_data = None
        self.provide_label = None


class BaseModule:
    """Abstract module; see the module docstring for the split of responsibilities."""

    def __init__(self, logger=logging):
        self.logger = logger
        self.binded = False
        self.for_training = False
        self.inputs_need_grad = False
        self.params_initialized = False
        self.optimizer_initialized = False
        self._symbol = None
        self._total_exec_bytes = 0

    def _require(self, *flags):
        for f in flags:
            if not getattr(self, f):
                raise AssertionError('%s: module is not %s' % (type(self).__name__, f.replace('_', ' ')))

    # ---------------------------------------------------------------- evaluation loops
    def _walk(self, data_iter, num_batch, reset, sparse_row_id_fn):
        self._require('binded', 'params_initialized')
        if reset:
            data_iter.reset()
        for nbatch, batch in enumerate(data_iter):
            if num_batch is not None and nbatch >= num_batch:
                return
            self.prepare(batch, sparse_row_id_fn=sparse_row_id_fn)
            self.forward(batch, is_train=False)
            yield nbatch, batch

    def _unpadded_outputs(self, batch, copy):
        outs = self.get_outputs()
        n = lambda o: o.shape[0] - batch.pad    # noqa: E731
        return [o[0:n(o)].copy() if copy else o[0:n(o)] for o in outs]

    def forward_backward(self, data_batch):
        self.forward(data_batch, is_train=True)
        self.backward()

    def score(self, eval_data, eval_metric, num_batch=None, batch_end_callback=None, score_end_callback=None,
              reset=True, epoch=0, sparse_row_id_fn=None):
        """Run ``eval_data`` through the model and return ``eval_metric``'s (name, value) pairs."""
        if not isinstance(eval_metric, metric.EvalMetric):
            eval_metric = metric.create(eval_metric)
        eval_metric.reset()
        seen = 0
        for nbatch, batch in self._walk(eval_data, num_batch, reset, sparse_row_id_fn):
            labels, pre_sliced = _batch_labels(batch)
            self.update_metric(eval_metric, labels, pre_sliced=pre_sliced)
            _fire(batch_end_callback, BatchEndParam(epoch, nbatch, eval_metric, locals()))
            seen += 1
        _fire(score_end_callback, BatchEndParam(epoch, seen, eval_metric, locals()))
        return eval_metric.get_name_value()

    def iter_predict(self, eval_data, num_batch=None, reset=True, sparse_row_id_fn=None):
        """Yield ``(outputs, batch_index, batch)`` with padding rows removed."""
        for nbatch, batch in self._walk(eval_data, num_batch, reset, sparse_row_id_fn):
            yield self._unpadded_outputs(batch, copy=False), nbatch, batch

    def predict(self, eval_data, num_batch=None, merge_batches=True, reset=True, always_output_list=False,
                sparse_row_id_fn=None):
        """Outputs for a data iterator (concatenated over batches), or for one array."""
        self._require('binded', 'params_initialized')
        if isinstance(eval_data, (NDArray, np.ndarray)):
            arr = eval_data if isinstance(eval_data, NDArray) else nd.array(eval_data)
            self.forward(_SimpleBatch([arr]))
            return self.get_outputs()[0]
        per_batch = [self._unpadded_outputs(batch, copy=True)
                     for _, batch in self._walk(eval_data, num_batch, reset, sparse_row_id_fn)]
        if not per_batch or not merge_batches:
            return per_batch
        width = len(per_batch[0])
        if any(len(outs) != width for outs in per_batch):
            raise AssertionError('cannot merge batches with different numbers of outputs (bucketing?)')
        merged = [nd.concat(*[outs[i] for outs in per_batch], dim=0) for i in range(width)]
        return merged[0] if width == 1 and not always_output_list else merged

    # ---------------------------------------------------------------- training loop
    def fit(self, train_data, eval_data=None, eval_metric='acc', epoch_end_callback=None, batch_end_callback=None,
            kvstore='local', optimizer='sgd', optimizer_params=(('learning_rate', 0.01),), eval_end_callback=None,
            eval_batch_end_callback=None, initializer=Uniform(0.01), arg_params=None, aux_params=None,
            allow_missing=False, force_rebind=False, force_init=False, begin_epoch=0, num_epoch=None,
            validation_metric=None, monitor=None, sparse_row_id_fn=None):
        """Train for epochs ``[begin_epoch, num_epoch)``; optionally score ``eval_data`` after each."""
        if num_epoch is None:
            raise AssertionError('fit() needs num_epoch')
        self.bind(data_shapes=train_data.provide_data, label_shapes=train_data.provide_label, for_training=True,
                  force_rebind=force_rebind)
        if monitor is not None:
            self.install_monitor(monitor)
        self.init_params(initializer=initializer, arg_params=arg_params, aux_params=aux_params,
                         allow_missing=allow_missing, force_init=force_init)
        self.init_optimizer(kvstore=kvstore, optimizer=optimizer, optimizer_params=optimizer_params)
        validation_metric = validation_metric if validation_metric is not None else eval_metric
        train_metric = eval_metric if isinstance(eval_metric, metric.EvalMetric) else metric.create(eval_metric)
        for epoch in range(begin_epoch, num_epoch):
            t0 = time.time()
            results = self._train_epoch(epoch, train_data, train_metric, monitor, batch_end_callback,
                                        sparse_row_id_fn)
            for name, val in results:
                self.logger.info('Epoch[%d] Train-%s=%f', epoch, name, val)
            self.logger.info('Epoch[%d] Time cost=%.3f', epoch, time.time() - t0)
            # pull the trained values back into arg/aux dicts (and re-broadcast to every device)
            args, auxs = self.get_params()
            self.set_params(args, auxs)
            _fire(epoch_end_callback, epoch, self.symbol, args, auxs)
            if eval_data is not None:
                for name, val in self.score(eval_data, validation_metric, score_end_callback=eval_end_callback,
                                            batch_end_callback=eval_batch_end_callback, epoch=epoch):
                    self.logger.info('Epoch[%d] Validation-%s=%f', epoch, name, val)
            train_data.reset()

    def _train_epoch(self, epoch, train_data, train_metric, monitor, batch_end_callback, sparse_row_id_fn):
        train_metric.reset()
        it = iter(train_data)
        batch = next(it)
        nbatch = 0
        while batch is not None:
            if monitor is not None:
                monitor.tic()
            self.forward_backward(batch)
            self.update()
            labels, pre_sliced = _batch_labels(batch)
            self.update_metric(train_metric, labels, pre_sliced=pre_sliced)
            upcoming = next(it, None)
            if upcoming is not None:
                self.prepare(upcoming, sparse_row_id_fn=sparse_row_id_fn)
            if monitor is not None:
                monitor.toc_print()
            results = train_metric.get_global_name_value() if upcoming is None else None
            _fire(batch_end_callback, BatchEndParam(epoch, nbatch, train_metric, locals()))
            batch = upcoming
            nbatch += 1
        return results or []

    # ---------------------------------------------------------------- properties
    @property
    def symbol(self):
        return self._symbol

    def _unimplemented(self, *_a, **_k):
        raise NotImplementedError('%s does not implement this operation' % type(self).__name__)

    data_names = property(_unimplemented)
    output_names = property(_unimplemented)
    data_shapes = property(_unimplemented)
    label_shapes = property(_unimplemented)
    output_shapes = property(_unimplemented)

    # ---------------------------------------------------------------- parameters
    def get_params(self):
        self._unimplemented()

    def init_params(self, initializer=Uniform(0.01), arg_params=None, aux_params=None, allow_missing=False,
                    force_init=False, allow_extra=False):
        self._unimplemented()

    def set_params(self, arg_params, aux_params, allow_missing=False, force_init=True, allow_extra=False):
        self.init_params(initializer=None, arg_params=arg_params, aux_params=aux_params,
                         allow_missing=allow_missing, force_init=force_init, allow_extra=allow_extra)

    def save_params(self, fname):
        """Write ``arg:<name>`` / ``aux:<name>`` arrays (host copies) to an MXNet ``.params`` file."""
        from ..context import cpu
        args, auxs = self.get_params()
        blob = {}
        for prefix, params in (('arg', args), ('aux', auxs)):
            blob.update({'%s:%s' % (prefix, k): v.as_in_context(cpu()) for k, v in params.items()})
        nd.save(fname, blob)

    def load_params(self, fname):
        parts = {'arg': {}, 'aux': {}}
        for key, value in nd.load(fname).items():
            kind, _, name = key.partition(':')
            if kind not in parts or not name:
                raise ValueError('Invalid param file %s (key %r)' % (fname, key))
            parts[kind][name] = value
        self.set_params(parts['arg'], parts['aux'])

    def get_states(self, merge_multi_context=True):
        self._require('binded', 'params_initialized')
        if merge_multi_context:
            raise AssertionError('this module has no states to merge')
        return []

    def set_states(self, states=None, value=None):
        self._require('binded', 'params_initialized')
        if states or value:
            raise AssertionError('this module has no states')

    def install_monitor(self, mon):
        self._unimplemented()

    def prepare(self, data_batch, sparse_row_id_fn=None):
        """Hook run before a batch is forwarded (row-sparse pulls in Module)."""
        if sparse_row_id_fn is not None and not (self.binded and self.params_initialized
                                                 and self.optimizer_initialized):
            self.logger.warning('sparse_row_id_fn ignored: module not bound / initialised / optimised yet.')

    # ---------------------------------------------------------------- computation (abstract)
    def forward(self, data_batch, is_train=None):
        self._unimplemented()

    def backward(self, out_grads=None):
        self._unimplemented()

    def get_outputs(self, merge_multi_context=True):
        self._unimplemented()

    def get_input_grads(self, merge_multi_context=True):
        self._unimplemented()

    def update(self):
        self._unimplemented()

    def update_metric(self, eval_metric, labels, pre_sliced=False):
        self._unimplemented()

    def bind(self, data_shapes, label_shapes=None, for_training=True, inputs_need_grad=False, force_rebind=False,
             shared_module=None, grad_req='write'):
        self._unimplemented()

    def init_optimizer(self, kvstore='local', optimizer='sgd', optimizer_params=(('learning_rate', 0.01),),
                       force_init=False):
        self._unimplemented()
