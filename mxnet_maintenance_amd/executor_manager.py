"""Data-parallel executor management for the legacy ``FeedForward`` model API.

Parity: python/mxnet/executor_manager.py:30-443 (``_split_input_slice``,
``_check_arguments``, ``DataParallelExecutorGroup``,
``DataParallelExecutorManager``).  One executor per context is bound with
``simple_bind`` on that context's share of the batch; parameter arrays of the
same name across executors are kept as lists (reduced by the caller's kvstore
/ updater), data batches are sliced into the per-context input arrays.
Bucketing (``sym_gen``) binds one executor group per bucket key, sharing the
default group's memory.
"""
import logging

from . import ndarray as nd
from .context import cpu
from .base import mx_real_t
from .io import DataDesc

__all__ = ['DataParallelExecutorGroup', 'DataParallelExecutorManager']


def _split_input_slice(batch_size, work_load_list):
    """Contiguous batch slices proportional to ``work_load_list`` (the rounding remainder goes to
    the last device); raises ValueError when a slice would be empty."""
    total = float(sum(work_load_list))
    sizes = [int(round(w * batch_size / total)) for w in work_load_list]
    sizes[-1] += batch_size - sum(sizes)
    out, start = [], 0
    for n in sizes:
        lo = min(start, batch_size)
        hi = min(lo + n, batch_size)
        if hi <= lo:
            raise ValueError('Too many slices. Some splits are empty.')
        out.append(slice(lo, hi))
        start = hi
    return out


def _check_arguments(symbol):
    """Reject symbols whose argument or auxiliary names repeat (a weight shared by accident)."""
    for kind, names in (('argument', symbol.list_arguments()), ('auxiliary param', symbol.list_auxiliary_states())):
        seen = set()
        for n in names:
            if n in seen:
                raise ValueError('Find duplicated %s name "%s", please make the weight name non-duplicated '
                                 '(using name arguments), names are %s' % (kind, n, str(names)))
            seen.add(n)


def _load_general(data, targets):
    """Copy each source array into its target: a whole array, or [(slice, array)] per device."""
    for src, dst in zip(data, targets):
        if isinstance(dst, nd.NDArray):
            src.copyto(dst)
            continue
        if dst[-1][0].stop != src.shape[0]:
            raise AssertionError('Batch size miss match. Expected %d, got %d' % (dst[-1][0].stop, src.shape[0]))
        for sl, arr in dst:
            src[sl].copyto(arr)


def _load_data(batch, targets):
    _load_general(batch.data, targets)


def _load_label(batch, targets):
    _load_general(batch.label, targets)


def _desc_name_shape_type(desc):
    if isinstance(desc, DataDesc):
        return desc.name, tuple(desc.shape), desc.dtype
    return desc[0], tuple(desc[1]), mx_real_t


class DataParallelExecutorGroup:
    """One bound executor per context over the context's slice of the batch."""

    def __init__(self, sym, arg_names, param_names, ctx, slices, train_data, shared_group=None):
        _check_arguments(sym)
        self.shared_data_arrays = ([{} for _ in ctx] if shared_group is None else shared_group.shared_data_arrays)
        self.data_names = [_desc_name_shape_type(d)[0] for d in train_data.provide_data]
        self.label_names = [_desc_name_shape_type(d)[0] for d in train_data.provide_label]
        self.aux_names = sym.list_auxiliary_states()
        self.param_idx = [i for i, n in enumerate(arg_names) if n in param_names]
        self.param_names = [arg_names[i] for i in self.param_idx]
        self.slices = slices
        params = set(self.param_names)
        self.train_execs = []
        for i, c in enumerate(ctx):
            shapes, types = {}, {}
            for d in list(train_data.provide_data) + list(train_data.provide_label):
                name, shape, dtype = _desc_name_shape_type(d)
                shapes[name] = (slices[i].stop - slices[i].start,) + shape[1:]
                types[name] = dtype
            grad_req = {n: ('write' if n in params else 'null') for n in sym.list_arguments()}
            shared = None if shared_group is None else shared_group.train_execs[i]
            ex = sym.simple_bind(c, grad_req=grad_req, type_dict=types, shared_exec=shared,
                                 shared_buffer=self.shared_data_arrays[i], **shapes)
            self.train_execs.append(ex)
        self.data_arrays = [[(slices[i], e.arg_dict[n]) for i, e in enumerate(self.train_execs)]
                            for n in self.data_names]
        self.label_arrays = [[(slices[i], e.arg_dict[n]) for i, e in enumerate(self.train_execs)]
                             for n in self.label_names]
        self.param_arrays = [[e.arg_arrays[i] for e in self.train_execs] for i in self.param_idx]
        self.grad_arrays = [[e.grad_arrays[i] for e in self.train_execs] for i in self.param_idx]
        self.aux_arrays = [[e.aux_arrays[i] for e in self.train_execs] for i in range(len(self.aux_names))]

    def load_data_batch(self, data_batch):
        _load_data(data_batch, self.data_arrays)
        _load_label(data_batch, self.label_arrays)

    def forward(self, is_train=False):
        for ex in self.train_execs:
            ex.forward(is_train=is_train)

    def backward(self):
        for ex in self.train_execs:
            ex.backward()

    def update_metric(self, metric, labels, pre_sliced=False):
        for k, (ex, sl) in enumerate(zip(self.train_execs, self.slices)):
            lab = labels[k] if pre_sliced else [l[sl] for l in labels]
            metric.update(lab, ex.outputs)


class DataParallelExecutorManager:
    """Executor groups for data-parallel training on ``ctx`` (optionally per bucket key)."""

    def __init__(self, symbol, ctx, train_data, arg_names, param_names, aux_names, work_load_list=None,
                 logger=None, sym_gen=None):
        logger = logger or logging
        logger.info('Start training with %s', str(ctx))
        if work_load_list is None:
            work_load_list = [1] * len(ctx)
        if not isinstance(work_load_list, list) or len(work_load_list) != len(ctx):
            raise AssertionError('Invalid settings for work load. ')
        self.slices = _split_input_slice(train_data.batch_size, work_load_list)
        self.arg_names, self.param_names, self.aux_names = arg_names, param_names, aux_names
        self.ctx = ctx
        self.symbol = symbol
        self.execgrp = DataParallelExecutorGroup(symbol, arg_names, param_names, ctx, self.slices, train_data)
        self.sym_gen = sym_gen
        self.curr_execgrp = None
        if sym_gen is not None:
            self.execgrp_bucket = {train_data.default_bucket_key: self.execgrp}

    def install_monitor(self, monitor):
        if self.sym_gen is not None:
            raise NotImplementedError('Monitoring is not implemented for bucketing')
        for ex in self.execgrp.train_execs:
            monitor.install(ex)

    def set_params(self, arg_params, aux_params):
        for ex in self.execgrp.train_execs:
            ex.copy_params_from(arg_params, aux_params)

    def copy_to(self, arg_params, aux_params):
        """Average the replicas of every parameter / auxiliary state into the given dicts."""
        for name, block in zip(self.param_names, self.param_arrays):
            avg = sum(w.copyto(cpu()) for w in block) / len(block)
            avg.astype(arg_params[name].dtype).copyto(arg_params[name])
        for name, block in zip(self.aux_names, self.aux_arrays):
            avg = sum(w.copyto(cpu()) for w in block) / len(block)
            avg.astype(aux_params[name].dtype).copyto(aux_params[name])

    @property
    def param_arrays(self):
        return self.execgrp.param_arrays

    @property
    def grad_arrays(self):
        return self.execgrp.grad_arrays

    @property
    def aux_arrays(self):
        return self.execgrp.aux_arrays

    def load_data_batch(self, data_batch):
        if self.sym_gen is not None:
            key = data_batch.bucket_key
            grp = self.execgrp_bucket.get(key)
            if grp is None:
                grp = DataParallelExecutorGroup(self.sym_gen(key), self.arg_names, self.param_names, self.ctx,
                                                self.slices, data_batch, shared_group=self.execgrp)
                self.execgrp_bucket[key] = grp
            self.curr_execgrp = grp
        else:
            self.curr_execgrp = self.execgrp
        self.curr_execgrp.load_data_batch(data_batch)

    def forward(self, is_train=False):
        self.curr_execgrp.forward(is_train=is_train)

    def backward(self):
        self.curr_execgrp.backward()

    def update_metric(self, metric, labels, pre_sliced=False):
        self.curr_execgrp.update_metric(metric, labels, pre_sliced)
