"""Checkpointing and the legacy FeedForward model API (parity: python/mxnet/model.py).

``save_checkpoint`` / ``load_checkpoint`` write and read ``prefix-symbol.json``
+ ``prefix-%04d.params`` (``arg:``/``aux:`` prefixed NDArray dict in the MXNet
binary format); the kvstore helpers are shared with ``mx.mod.Module``.
"""
import logging
import os
import time
from collections import namedtuple

import numpy as np

from . import io as mxio
from . import kvstore as kvs
from . import metric
from . import ndarray as nd
from . import optimizer as opt
from . import symbol as sym_mod
from .base import MXNetError
from .context import Context, cpu
from .initializer import Uniform

BatchEndParam = namedtuple('BatchEndParams', ['epoch', 'nbatch', 'eval_metric', 'locals'])

__all__ = ['BatchEndParam', 'save_checkpoint', 'load_checkpoint', 'load_params', 'FeedForward']


def _create_kvstore(kvstore, num_device, arg_params):
    """(kvstore or None, update_on_kvstore) for Module / FeedForward.

    One device in one process needs no store; 'local' stores keep the update on the workers when a
    parameter exceeds 16M elements (the store would serialise a huge update); a store that cannot
    run optimizers never updates on itself.  MXNET_UPDATE_ON_KVSTORE=0 disables store updates."""
    if kvstore is not None and not isinstance(kvstore, (kvs.KVStoreBase, str)):
        raise TypeError('kvstore must be KVStore, str or None')
    if isinstance(kvstore, str):
        kv = kvs.create(kvstore) if (num_device > 1 or 'dist' in kvstore) else None
    else:
        kv = kvstore
    if kv is None or not kv.is_capable(kvs.KVStoreBase.OPTIMIZER):
        return kv, False
    on_store = bool(int(os.getenv('MXNET_UPDATE_ON_KVSTORE', '1')))
    biggest = max((int(np.prod(p.shape)) for p in arg_params.values()), default=0) if arg_params else 0
    if kvstore == 'local' and biggest > (16 << 20):
        on_store = False
    return kv, on_store


def _initialize_kvstore(kvstore, param_arrays, arg_params, param_names, update_on_kvstore):
    """Seed the store with every parameter; with store-side updates the device copies are
    broadcast from it (sparse parameters are only initialised)."""
    for name, replicas in zip(param_names, param_arrays):
        value = arg_params[name]
        if update_on_kvstore and value.stype == 'default':
            kvstore.broadcast(name, value, out=replicas)
        else:
            kvstore.init(name, value)


def _update_params_on_kvstore(param_arrays, grad_arrays, kvstore, param_names):
    """Store-side update: push each gradient set, pull the updated weights (priority = -index so
    the first layers, needed first by the next forward, are served first)."""
    for pos, (name, replicas, grads) in enumerate(zip(param_names, param_arrays, grad_arrays)):
        if grads[0] is not None:
            kvstore.push(name, grads, priority=-pos)
            kvstore.pull(name, replicas, priority=-pos)


def _update_params(param_arrays, grad_arrays, updater, num_device, kvstore=None, param_names=None):
    """Worker-side update: optional gradient all-reduce through the store, then ONE aggregated
    updater call per device (updater keys ``index * num_device + device``)."""
    per_device = [([], [], []) for _ in range(num_device)]
    for pos, (replicas, grads) in enumerate(zip(param_arrays, grad_arrays)):
        if grads[0] is None:
            continue
        if kvstore:
            kvstore.pushpull(param_names[pos], grads, grads, priority=-pos)
        for dev, (w, g) in enumerate(zip(replicas, grads)):
            keys, gs, ws = per_device[dev]
            keys.append(pos * num_device + dev)
            gs.append(g)
            ws.append(w)
    for keys, gs, ws in per_device:
        if keys:
            updater(keys, gs, ws)


def _multiple_callbacks(callbacks, *args, **kwargs):
    for cb in (callbacks if isinstance(callbacks, list) else [callbacks] if callbacks else []):
        cb(*args, **kwargs)


def save_checkpoint_symbol(prefix, symbol, remove_amp_cast=True):
    """Write ``prefix-symbol.json`` (nothing for ``symbol=None``)."""
    if symbol is not None:
        symbol.save('%s-symbol.json' % prefix, remove_amp_cast=remove_amp_cast)


def save_checkpoint(prefix, epoch, symbol, arg_params, aux_params, remove_amp_cast=True):
    """Write ``prefix-symbol.json`` and ``prefix-%04d.params`` (``arg:`` / ``aux:`` keyed, host copies)."""
    save_checkpoint_symbol(prefix, symbol, remove_amp_cast)
    tagged = {}
    for tag, table in (('arg', arg_params), ('aux', aux_params)):
        tagged.update({'%s:%s' % (tag, k): v.as_in_context(cpu()) for k, v in table.items()})
    path = '%s-%04d.params' % (prefix, epoch)
    nd.save(path, tagged)
    logging.info('Saved checkpoint to "%s"', path)


def load_params(prefix, epoch):
    """(arg_params, aux_params) from ``prefix-%04d.params``."""
    path = '%s-%04d.params' % (prefix, epoch)
    saved = nd.load(path)
    tables = {'arg': {}, 'aux': {}}
    if not saved:
        logging.warning('Params file "%s" is empty', path)
    for key, value in (saved or {}).items():
        tag, name = key.split(':', 1)
        if tag in tables:
            tables[tag][name] = value
    return tables['arg'], tables['aux']


def load_checkpoint(prefix, epoch):
    """(symbol, arg_params, aux_params) of a checkpoint written by ``save_checkpoint``."""
    return (sym_mod.load('%s-symbol.json' % prefix),) + load_params(prefix, epoch)


class FeedForward:
    """Legacy feed-forward model (deprecated in the reference; kept for API parity) built on Module."""

    def __init__(self, symbol, ctx=None, num_epoch=None, epoch_size=None, optimizer='sgd', initializer=Uniform(0.01),
                 numpy_batch_size=128, arg_params=None, aux_params=None, allow_extra_params=False,
                 begin_epoch=0, **kwargs):
        self.symbol = symbol
        if ctx is None:
            ctx = [cpu()]
        elif isinstance(ctx, Context):
            ctx = [ctx]
        self.ctx = ctx
        self.num_epoch = num_epoch
        self.epoch_size = epoch_size
        self.kwargs = kwargs.copy()
        self.optimizer = optimizer
        self.initializer = initializer
        self.numpy_batch_size = numpy_batch_size
        self.arg_params = arg_params
        self.aux_params = aux_params
        self.allow_extra_params = allow_extra_params
        self.begin_epoch = begin_epoch
        self._mod = None

    def _label_names(self):
        return [n for n in self.symbol.list_arguments() if n.endswith('label')]

    def _init_iter(self, X, y, is_train):
        if isinstance(X, (np.ndarray, nd.NDArray)):
            if y is None:
                if is_train:
                    raise ValueError('y must be specified when X is numpy.ndarray')
                y = np.zeros(X.shape[0])
            if not isinstance(y, (np.ndarray, nd.NDArray)):
                raise TypeError('y must be ndarray when X is numpy.ndarray')
            if X.shape[0] != y.shape[0]:
                raise ValueError('The numbers of data points and labels not equal')
            if y.ndim == 2 and y.shape[1] == 1:
                y = y.flatten()
            if y.ndim != 1:
                raise ValueError('Label must be 1D or 2D (with 2nd dimension being 1)')
            if is_train:
                return mxio.NDArrayIter(X, y, min(X.shape[0], self.numpy_batch_size), shuffle=is_train,
                                        last_batch_handle='roll_over')
            return mxio.NDArrayIter(X, y, min(X.shape[0], self.numpy_batch_size), shuffle=False)
        if not isinstance(X, mxio.DataIter):
            raise TypeError('X must be DataIter, NDArray or numpy.ndarray')
        return X

    def _module(self, data_iter, for_training):
        from .module import Module
        data_names = [d[0] for d in data_iter.provide_data]
        label_names = [l[0] for l in data_iter.provide_label]
        mod = Module(self.symbol, data_names=data_names, label_names=label_names, context=self.ctx)
        mod.bind(data_iter.provide_data, data_iter.provide_label, for_training=for_training)
        mod.init_params(self.initializer, self.arg_params, self.aux_params, allow_missing=True,
                        allow_extra=self.allow_extra_params)
        return mod

    def fit(self, X, y=None, eval_data=None, eval_metric='acc', epoch_end_callback=None, batch_end_callback=None,
            kvstore='local', logger=None, work_load_list=None, monitor=None, eval_end_callback=None,
            eval_batch_end_callback=None):
        data = self._init_iter(X, y, is_train=True)
        if isinstance(eval_data, tuple):
            eval_data = self._init_iter(eval_data[0], eval_data[1], is_train=True)
        from .module import Module
        data_names = [d[0] for d in data.provide_data]
        label_names = [l[0] for l in data.provide_label]
        self._mod = Module(self.symbol, data_names=data_names, label_names=label_names, context=self.ctx,
                           work_load_list=work_load_list, logger=logger or logging)
        self._mod.fit(data, eval_data=eval_data, eval_metric=eval_metric, epoch_end_callback=epoch_end_callback,
                      batch_end_callback=batch_end_callback, kvstore=kvstore, optimizer=self.optimizer,
                      optimizer_params=self.kwargs, initializer=self.initializer, arg_params=self.arg_params,
                      aux_params=self.aux_params, allow_missing=True, begin_epoch=self.begin_epoch,
                      num_epoch=self.num_epoch, monitor=monitor, eval_end_callback=eval_end_callback,
                      eval_batch_end_callback=eval_batch_end_callback)
        self.arg_params, self.aux_params = self._mod.get_params()

    def predict(self, X, num_batch=None, return_data=False, reset=True):
        X = self._init_iter(X, None, is_train=False)
        mod = self._module(X, for_training=False)
        out = mod.predict(X, num_batch=num_batch, reset=reset)
        if isinstance(out, list):
            out = [o.asnumpy() for o in out]
        else:
            out = out.asnumpy()
        if return_data:
            X.reset()
            data, label = [], []
            for b in X:
                data.append(b.data[0].asnumpy()[:b.data[0].shape[0] - b.pad])
                label.append(b.label[0].asnumpy()[:b.label[0].shape[0] - b.pad])
            return out, np.concatenate(data), np.concatenate(label)
        return out

    def score(self, X, eval_metric='acc', num_batch=None, batch_end_callback=None, reset=True):
        X = self._init_iter(X, None, is_train=False)
        mod = self._module(X, for_training=False)
        res = mod.score(X, eval_metric, num_batch=num_batch, batch_end_callback=batch_end_callback, reset=reset)
        return res[0][1]

    def save(self, prefix, epoch=None, remove_amp_cast=True):
        if epoch is None:
            epoch = self.num_epoch
        assert epoch is not None
        save_checkpoint(prefix, epoch, self.symbol, self.arg_params, self.aux_params, remove_amp_cast)

    @staticmethod
    def load(prefix, epoch, ctx=None, **kwargs):
        symbol, arg_params, aux_params = load_checkpoint(prefix, epoch)
        return FeedForward(symbol, ctx=ctx, arg_params=arg_params, aux_params=aux_params, begin_epoch=epoch,
                           **kwargs)

    @staticmethod
    def create(symbol, X, y=None, ctx=None, num_epoch=None, epoch_size=None, optimizer='sgd',
               initializer=Uniform(0.01), eval_data=None, eval_metric='acc', epoch_end_callback=None,
               batch_end_callback=None, kvstore='local', logger=None, work_load_list=None,
               eval_end_callback=None, eval_batch_end_callback=None, **kwargs):
        model = FeedForward(symbol, ctx=ctx, num_epoch=num_epoch, epoch_size=epoch_size, optimizer=optimizer,
                            initializer=initializer, **kwargs)
        model.fit(X, y, eval_data=eval_data, eval_metric=eval_metric, epoch_end_callback=epoch_end_callback,
                  batch_end_callback=batch_end_callback, kvstore=kvstore, logger=logger,
                  work_load_list=work_load_list, eval_end_callback=eval_end_callback,
                  eval_batch_end_callback=eval_batch_end_callback)
        return model
