"""Data-parallel executor group (parity: python/mxnet/module/executor_group.py).

Binds one Executor per context with the batch split by ``workload``;
parameters are replicated (one array per context), inputs/labels are sliced
along the batch axis, outputs are concatenated back.  On an MI355X node the
usual deployment is one process per GPU (one context here) with gradient
reduction through the kvstore; several contexts in one process are
supported for parity.
"""
import logging

import numpy as np

from .. import ndarray as nd
from ..base import MXNetError
from ..io import DataDesc
from ..ndarray.ndarray import NDArray

__all__ = ['DataParallelExecutorGroup']


def _split_input_slice(batch_size, work_load_list):
    total = sum(work_load_list)
    batch_num_list = [round(w * batch_size / total) for w in work_load_list]
    delta = batch_size - sum(batch_num_list)
    batch_num_list[-1] += delta
    slices = []
    end = 0
    for n in batch_num_list:
        begin = int(min(end, batch_size))
        end = int(min(begin + n, batch_size))
        if begin >= end:
            raise ValueError('Too many slices. Some splits are empty.')
        slices.append(slice(begin, end))
    return slices


def _load_general(data, targets, major_axis):
    for d_src, d_targets in zip(data, targets):
        if isinstance(d_targets, NDArray):
            d_src.copyto(d_targets)
        elif isinstance(d_src, (list, tuple)):
            for src, dst in zip(d_src, d_targets):
                src.copyto(dst)
        else:
            for slice_idx, d_dst in d_targets:
                if major_axis >= 0 and d_src.shape[major_axis] != d_dst.shape[major_axis]:
                    d_src_slice = nd.slice_axis(d_src, axis=major_axis, begin=slice_idx.start,
                                                end=slice_idx.stop)
                else:
                    d_src_slice = d_src
                d_dst[:] = d_src_slice.astype(d_dst.dtype).as_in_context(d_dst.context)


def _merge_multi_context(outputs, major_axis):
    rets = []
    for tensors, axis in zip(outputs, major_axis):
        if axis >= 0:
            if len(tensors) == 1:
                rets.append(tensors[0])
            else:
                rets.append(nd.concat(*[t.as_in_context(tensors[0].context) for t in tensors], dim=axis))
        else:
            rets.append(tensors[0])
    return rets


class DataParallelExecutorGroup:
    def __init__(self, symbol, contexts, workload, data_shapes, label_shapes, param_names, for_training,
                 inputs_need_grad, shared_group=None, logger=logging, fixed_param_names=None, grad_req='write',
                 state_names=None, group2ctxs=None):
        self.param_names = param_names
        self.arg_names = symbol.list_arguments()
        self.aux_names = symbol.list_auxiliary_states()
        self.symbol = symbol
        self.contexts = contexts
        self.workload = workload or [1] * len(contexts)
        self.for_training = for_training
        self.inputs_need_grad = inputs_need_grad
        self.logger = logger
        self.fixed_param_names = fixed_param_names or []
        self.state_names = state_names or []
        self.shared_group = shared_group
        self.execs = []
        self.batch_size = None
        self.slices = None
        self.data_shapes = None
        self.label_shapes = None
        self.grad_req = {}
        data_names = [x.name if isinstance(x, DataDesc) else x[0] for x in data_shapes]
        if isinstance(grad_req, str):
            for k in self.arg_names:
                if k in self.param_names:
                    self.grad_req[k] = 'null' if k in self.fixed_param_names else grad_req
                elif k in data_names:
                    self.grad_req[k] = grad_req if self.inputs_need_grad else 'null'
                else:
                    self.grad_req[k] = 'null'
        elif isinstance(grad_req, (list, tuple)):
            self.grad_req = dict(zip(self.arg_names, grad_req))
        elif isinstance(grad_req, dict):
            for k in self.arg_names:
                if k in self.param_names:
                    self.grad_req[k] = 'null' if k in self.fixed_param_names else 'write'
                elif k in data_names:
                    self.grad_req[k] = 'write' if self.inputs_need_grad else 'null'
                else:
                    self.grad_req[k] = 'null'
            self.grad_req.update(grad_req)
        if not for_training:
            self.grad_req = {k: 'null' for k in self.arg_names}
        self.bind_exec(data_shapes, label_shapes, shared_group)

    # ------------------------------------------------------------ binding
    def decide_slices(self, data_shapes):
        major_axis = [DataDesc.get_batch_axis(getattr(x, 'layout', 'NCHW')) for x in data_shapes]
        for desc, axis in zip(data_shapes, major_axis):
            if axis == -1:
                continue
            batch_size = desc.shape[axis]
            if self.batch_size is not None:
                assert batch_size == self.batch_size, \
                    'all data must have the same batch size: batch_size = %d, but %s has shape %s' % (
                        self.batch_size, desc.name, desc.shape)
            else:
                self.batch_size = batch_size
                self.slices = _split_input_slice(self.batch_size, self.workload)
        return major_axis

    def _sliced_shape(self, shapes, i, major_axis):
        sliced = []
        for desc, axis in zip(shapes, major_axis):
            shape = list(desc.shape)
            if axis >= 0:
                shape[axis] = self.slices[i].stop - self.slices[i].start
            sliced.append(DataDesc(desc.name, tuple(shape), desc.dtype, getattr(desc, 'layout', 'NCHW')))
        return sliced

    def bind_exec(self, data_shapes, label_shapes, shared_group=None, reshape=False):
        data_shapes = [x if isinstance(x, DataDesc) else DataDesc(*x) for x in data_shapes]
        if label_shapes is not None:
            label_shapes = [x if isinstance(x, DataDesc) else DataDesc(*x) for x in label_shapes]
        self.batch_size = None
        self.data_layouts = self.decide_slices(data_shapes)
        self.label_layouts = self.decide_slices(label_shapes) if label_shapes is not None else None
        old_execs = self.execs
        self.execs = []
        for i, ctx in enumerate(self.contexts):
            shapes = {d.name: d.shape for d in self._sliced_shape(data_shapes, i, self.data_layouts)}
            types = {d.name: d.dtype for d in data_shapes}
            if label_shapes is not None:
                shapes.update({d.name: d.shape for d in self._sliced_shape(label_shapes, i, self.label_layouts)})
                types.update({d.name: d.dtype for d in label_shapes})
            shapes = {k: v for k, v in shapes.items() if k in self.arg_names}
            types = {k: v for k, v in types.items() if k in self.arg_names}
            exe = self.symbol.simple_bind(ctx, grad_req=self.grad_req, type_dict=types, **shapes)
            # share parameters with an existing group (bucketing) or keep values across reshape
            src = None
            if shared_group is not None:
                src = shared_group.execs[i]
            elif reshape and old_execs:
                src = old_execs[i]
            if src is not None:
                for name in self.param_names:
                    if name in src.arg_dict and src.arg_dict[name].shape == exe.arg_dict[name].shape:
                        j = self.arg_names.index(name)
                        exe.arg_arrays[j] = src.arg_dict[name]
                        if exe.grad_arrays[j] is not None and src.grad_dict.get(name) is not None:
                            exe.grad_arrays[j] = src.grad_dict[name]
                for j, name in enumerate(self.aux_names):
                    if name in src.aux_dict and src.aux_dict[name].shape == exe.aux_arrays[j].shape:
                        exe.aux_arrays[j] = src.aux_dict[name]
            self.execs.append(exe)
        self.data_shapes = data_shapes
        self.label_shapes = label_shapes
        self.data_names = [d.name for d in data_shapes]
        self.label_names = [d.name for d in label_shapes] if label_shapes is not None else []
        self._collect_arrays()

    def reshape(self, data_shapes, label_shapes):
        if data_shapes == self.data_shapes and label_shapes == self.label_shapes:
            return
        self.bind_exec(data_shapes, label_shapes, reshape=True)

    def _collect_arrays(self):
        self.data_arrays = [[(self.slices[i], e.arg_dict[name]) for i, e in enumerate(self.execs)]
                            for name in self.data_names if name in self.arg_names]
        self.label_arrays = [[(self.slices[i], e.arg_dict[name]) for i, e in enumerate(self.execs)]
                             for name in self.label_names if name in self.arg_names]
        self.param_arrays = [[e.arg_arrays[i] for e in self.execs] for i, name in enumerate(self.arg_names)
                             if name in self.param_names]
        if self.for_training:
            self.grad_arrays = [[e.grad_arrays[i] for e in self.execs] for i, name in enumerate(self.arg_names)
                                if name in self.param_names]
        else:
            self.grad_arrays = None
        data_names = [x[0] for x in self.data_shapes]
        if self.inputs_need_grad:
            self.input_grad_arrays = [[e.grad_arrays[self.arg_names.index(name)] for e in self.execs]
                                      for name in data_names if name in self.arg_names]
        else:
            self.input_grad_arrays = None
        self.aux_arrays = [[e.aux_arrays[i] for e in self.execs] for i in range(len(self.aux_names))]

    # ------------------------------------------------------------ params
    def set_params(self, arg_params, aux_params, allow_extra=False):
        for exe in self.execs:
            exe.copy_params_from(arg_params, aux_params, allow_extra_params=allow_extra)

    def get_params(self, arg_params, aux_params):
        for name, block in zip(self.param_names, self.param_arrays):
            weight = sum(w.copyto(_cpu()) for w in block) / len(block)
            weight.astype(arg_params[name].dtype).copyto(arg_params[name])
        for name, block in zip(self.aux_names, self.aux_arrays):
            weight = sum(w.copyto(_cpu()) for w in block) / len(block)
            weight.astype(aux_params[name].dtype).copyto(aux_params[name])

    # ------------------------------------------------------------ compute
    def forward(self, data_batch, is_train=None):
        _load_general(data_batch.data, self.data_arrays, self.data_layouts[0] if self.data_layouts else 0)
        if is_train is None:
            is_train = self.for_training
        if self.label_arrays and data_batch.label:
            _load_general(data_batch.label, self.label_arrays,
                          self.label_layouts[0] if self.label_layouts else 0)
        for exe in self.execs:
            exe.forward(is_train=is_train)

    def get_output_shapes(self):
        # shapes of the whole (unsliced) batch, from shape inference (valid before any forward)
        shapes = {d.name: d.shape for d in self.data_shapes}
        if self.label_shapes is not None:
            shapes.update({d.name: d.shape for d in self.label_shapes})
        shapes = {k: v for k, v in shapes.items() if k in self.arg_names}
        _, out_shapes, _ = self.symbol.infer_shape(**shapes)
        return list(zip(self.symbol.list_outputs(), [tuple(s) for s in out_shapes]))

    def get_outputs(self, merge_multi_context=True, begin=0, end=None):
        if end is None:
            end = len(self.execs[0].outputs)
        outputs = [[exe.outputs[i] for exe in self.execs] for i in range(begin, end)]
        if merge_multi_context:
            outputs = _merge_multi_context(outputs, [0] * len(outputs))
        return outputs

    def get_states(self, merge_multi_context=True):
        assert not merge_multi_context
        return [[exe.arg_dict[name] for exe in self.execs] for name in self.state_names]

    def set_states(self, states=None, value=None):
        if states is not None:
            assert value is None
            _load_general(states, self.get_states(False), -1)
        else:
            for d_dst in self.get_states(False):
                for dst in d_dst:
                    dst[:] = value

    def get_input_grads(self, merge_multi_context=True):
        assert self.inputs_need_grad
        if merge_multi_context:
            return _merge_multi_context(self.input_grad_arrays, [0] * len(self.input_grad_arrays))
        return self.input_grad_arrays

    def backward(self, out_grads=None):
        assert self.for_training, 're-bind with for_training=True to run backward'
        if out_grads is None:
            out_grads = []
        for i, exe in enumerate(self.execs):
            out_grads_slice = []
            for grad in out_grads:
                sl = self.slices[i]
                og = nd.slice_axis(grad, axis=0, begin=sl.start, end=sl.stop)
                out_grads_slice.append(og.as_in_context(self.contexts[i]))
            exe.backward(out_grads=out_grads_slice or None)

    def update_metric(self, eval_metric, labels, pre_sliced=False):
        for current_exec, (texec, islice) in enumerate(zip(self.execs, self.slices)):
            if not pre_sliced:
                labels_slice = []
                for label in labels:
                    if label.shape[0] == self.batch_size and len(self.execs) > 1:
                        labels_slice.append(nd.slice_axis(label, axis=0, begin=islice.start, end=islice.stop))
                    else:
                        labels_slice.append(label)
            else:
                labels_slice = labels[current_exec]
            labels_ = dict(zip(self.label_names, labels_slice))
            preds = dict(zip(self.symbol.list_outputs(), texec.outputs))
            eval_metric.update_dict(labels_, preds)

    def install_monitor(self, mon):
        for exe in self.execs:
            mon.install(exe)


def _cpu():
    from ..context import cpu
    return cpu()
