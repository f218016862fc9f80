"""Data-parallel executor group: one bound Executor per context.

API parity: python/mxnet/module/executor_group.py (``DataParallelExecutorGroup``
with ``param_arrays`` / ``grad_arrays`` / ``aux_arrays`` as per-parameter lists
of per-device arrays, ``forward`` / ``backward`` / ``get_outputs`` /
``update_metric`` / ``reshape`` / ``set_params`` / ``get_params``).

Design: the group is a list of ``_Shard`` records (context, batch slice,
executor).  Per-parameter views (``param_arrays`` etc.) are derived from the
shards after every (re)bind.  On an MI355X node the normal deployment is one
process per GPU, i.e. a single shard, with cross-GPU reduction done by the
kvstore over RCCL; several contexts per process still work (batch split by
``workload``) for parity and CPU tests.
"""
import logging

from .. import ndarray as nd
from ..io import DataDesc
from ..ndarray.ndarray import NDArray

__all__ = ['DataParallelExecutorGroup']


def _split_input_slice(batch_size, work_load_list):
    """Contiguous batch slices proportional to ``work_load_list`` (last slice takes the rounding)."""
    total = float(sum(work_load_list))
    sizes = [int(round(w * batch_size / total)) for w in work_load_list]
    sizes[-1] += batch_size - sum(sizes)
    out, start = [], 0
    for n in sizes:
        stop = min(start + n, batch_size)
        if stop <= start:
            raise ValueError('batch of %d cannot be split over workloads %s: empty slice'
                             % (batch_size, work_load_list))
        out.append(slice(start, stop))
        start = stop
    return out


def _copy_into(src, dst, sl, axis):
    """dst[...] = src (sliced along ``axis`` by ``sl`` when src holds the whole batch)."""
    if axis >= 0 and src.shape[axis] != dst.shape[axis]:
        src = nd.slice_axis(src, axis=axis, begin=sl.start, end=sl.stop)
    dst[:] = src.astype(dst.dtype).as_in_context(dst.context)


def _load_general(data, targets, major_axis):
    """Copy a batch's arrays into per-device targets.

    ``targets[i]`` is either a single NDArray, a list of per-device arrays (src
    then also per-device), or a list of ``(slice, array)`` pairs to slice into.
    """
    for src, tgt in zip(data, targets):
        if isinstance(tgt, NDArray):
            src.copyto(tgt)
        elif isinstance(src, (list, tuple)):
            for s, d in zip(src, tgt):
                s.copyto(d)
        else:
            for sl, dst in tgt:
                _copy_into(src, dst, sl, major_axis)


def _merge_multi_context(outputs, major_axis):
    """Concatenate per-device pieces along each output's batch axis (axis < 0: take device 0's)."""
    merged = []
    for pieces, axis in zip(outputs, major_axis):
        if axis < 0 or len(pieces) == 1:
            merged.append(pieces[0])
        else:
            home = pieces[0].context
            merged.append(nd.concat(*[p.as_in_context(home) for p in pieces], dim=axis))
    return merged


def _resolve_grad_req(grad_req, arg_names, param_names, data_names, fixed, inputs_need_grad, for_training):
    """Per-argument gradient request: parameters get ``grad_req`` (fixed ones 'null'), data inputs
    only when input gradients are wanted, everything else 'null'."""
    if not for_training:
        return {k: 'null' for k in arg_names}
    if isinstance(grad_req, (list, tuple)):
        return dict(zip(arg_names, grad_req))
    default = grad_req if isinstance(grad_req, str) else 'write'

    def req(name):
        if name in param_names:
            return 'null' if name in fixed else default
        if name in data_names:
            return default if inputs_need_grad else 'null'
        return 'null'
    out = {k: req(k) for k in arg_names}
    if isinstance(grad_req, dict):
        out.update(grad_req)
    return out


class _Shard:
    __slots__ = ('ctx', 'slice', 'exe')

    def __init__(self, ctx, sl, exe):
        self.ctx = ctx
        self.slice = sl
        self.exe = exe


class DataParallelExecutorGroup:
    """Executors for ``symbol`` on ``contexts`` sharing one logical batch."""

    def __init__(self, symbol, contexts, workload, data_shapes, label_shapes, param_names, for_training,
                 inputs_need_grad, shared_group=None, logger=logging, fixed_param_names=None, grad_req='write',
                 state_names=None, group2ctxs=None):
        self.symbol = symbol
        self.contexts = list(contexts)
        self.workload = list(workload) if workload else [1] * len(self.contexts)
        self.param_names = list(param_names)
        self.arg_names = symbol.list_arguments()
        self.aux_names = symbol.list_auxiliary_states()
        self.fixed_param_names = list(fixed_param_names or [])
        self.state_names = list(state_names or [])
        self.for_training = for_training
        self.inputs_need_grad = inputs_need_grad
        self.shared_group = shared_group
        self.logger = logger
        self.shards = []
        self.batch_size = None
        self.slices = None
        self.data_shapes = self.label_shapes = None
        self.group2ctxs = group2ctxs
        # per device: the non-parameter argument arrays (inputs, labels, states), shared by name
        # with (and extended into) the shared group's, as the reference's executor group does
        self.shared_data_arrays = (shared_group.shared_data_arrays if shared_group is not None
                                   else [{} for _ in self.contexts])
        data_names = [d.name if isinstance(d, DataDesc) else d[0] for d in data_shapes]
        self.grad_req = _resolve_grad_req(grad_req, self.arg_names, self.param_names, data_names,
                                          self.fixed_param_names, inputs_need_grad, for_training)
        self.bind_exec(data_shapes, label_shapes, shared_group)

    @property
    def execs(self):
        return [s.exe for s in self.shards]

    # ---------------------------------------------------------------- binding
    def decide_slices(self, descs):
        """Batch axis per input; fixes ``batch_size`` / ``slices`` from the first batched input."""
        axes = [DataDesc.get_batch_axis(getattr(d, 'layout', 'NCHW')) for d in descs]
        for d, axis in zip(descs, axes):
            if axis < 0:
                continue
            n = d.shape[axis]
            if self.batch_size is None:
                self.batch_size = n
                self.slices = _split_input_slice(n, self.workload)
            elif n != self.batch_size:
                raise AssertionError('inputs disagree on the batch size: %d vs %s of shape %s'
                                     % (self.batch_size, d.name, d.shape))
        return axes

    def _shapes_for(self, descs, axes, sl):
        out = {}
        for d, axis in zip(descs, axes):
            shape = list(d.shape)
            if axis >= 0:
                shape[axis] = sl.stop - sl.start
            out[d.name] = (tuple(shape), d.dtype)
        return out

    def bind_exec(self, data_shapes, label_shapes, shared_group=None, reshape=False):
        data_shapes = [d if isinstance(d, DataDesc) else DataDesc(*d) for d in data_shapes]
        label_shapes = None if label_shapes is None else \
            [d if isinstance(d, DataDesc) else DataDesc(*d) for d in label_shapes]
        self.batch_size = None
        self.data_layouts = self.decide_slices(data_shapes)
        self.label_layouts = self.decide_slices(label_shapes) if label_shapes is not None else None
        previous = self.shards
        self.shards = []
        for i, ctx in enumerate(self.contexts):
            sl = self.slices[i]
            spec = self._shapes_for(data_shapes, self.data_layouts, sl)
            if label_shapes is not None:
                spec.update(self._shapes_for(label_shapes, self.label_layouts, sl))
            spec = {k: v for k, v in spec.items() if k in self.arg_names}
            g2c = self.group2ctxs
            if isinstance(g2c, (list, tuple)):
                g2c = g2c[i] if i < len(g2c) else None
            if isinstance(g2c, dict):
                # a group maps to one context for every device or to a per-device list
                g2c = {k: (v[i] if i < len(v) else v[-1]) if isinstance(v, (list, tuple)) else v
                       for k, v in g2c.items()}
            exe = self.symbol.simple_bind(ctx, grad_req=self.grad_req, type_dict={k: v[1] for k, v in spec.items()},
                                          group2ctx=g2c, **{k: v[0] for k, v in spec.items()})
            shared = self.shared_data_arrays[i]
            for j, name in enumerate(self.arg_names):
                if name in self.param_names:
                    continue
                have = shared.get(name)
                if have is not None and have.shape == exe.arg_arrays[j].shape and have.dtype == exe.arg_arrays[j].dtype:
                    exe.arg_arrays[j] = have
                else:
                    shared[name] = exe.arg_arrays[j]
            donor = shared_group.execs[i] if shared_group is not None else \
                (previous[i].exe if reshape and previous else None)
            if donor is not None:
                self._adopt_params(exe, donor)
            if reshape and previous and i < len(previous):
                # a monitor installed on the executor survives the rebind for new input shapes
                old = previous[i].exe
                exe._monitor_cb, exe._monitor_all = old._monitor_cb, old._monitor_all
            self.shards.append(_Shard(ctx, sl, exe))
        self.data_shapes, self.label_shapes = data_shapes, label_shapes
        self.data_names = [d.name for d in data_shapes]
        self.label_names = [d.name for d in label_shapes] if label_shapes is not None else []
        self._collect_arrays()

    def _adopt_params(self, exe, donor):
        """Share parameter / gradient / aux arrays of matching shape with ``donor`` (bucketing, reshape)."""
        for name in self.param_names:
            src = donor.arg_dict.get(name)
            j = self.arg_names.index(name)
            if src is None or src.shape != exe.arg_arrays[j].shape:
                continue
            exe.arg_arrays[j] = src
            g = donor.grad_dict.get(name)
            if exe.grad_arrays[j] is not None and g is not None:
                exe.grad_arrays[j] = g
        for j, name in enumerate(self.aux_names):
            src = donor.aux_dict.get(name)
            if src is not None and src.shape == exe.aux_arrays[j].shape:
                exe.aux_arrays[j] = src

    def reshape(self, data_shapes, label_shapes):
        if data_shapes != self.data_shapes or label_shapes != self.label_shapes:
            self.bind_exec(data_shapes, label_shapes, reshape=True)

    def _per_arg(self, names, pick):
        return [[pick(s.exe, self.arg_names.index(n)) for s in self.shards] for n in names if n in self.arg_names]

    def _collect_arrays(self):
        arg = lambda e, j: e.arg_arrays[j]       # noqa: E731
        grad = lambda e, j: e.grad_arrays[j]     # noqa: E731
        self.data_arrays = [[(s.slice, s.exe.arg_dict[n]) for s in self.shards]
                            for n in self.data_names if n in self.arg_names]
        self.label_arrays = [[(s.slice, s.exe.arg_dict[n]) for s in self.shards]
                             for n in self.label_names if n in self.arg_names]
        params = [n for n in self.arg_names if n in self.param_names]
        self.param_arrays = self._per_arg(params, arg)
        self.grad_arrays = self._per_arg(params, grad) if self.for_training else None
        self.input_grad_arrays = self._per_arg(self.data_names, grad) if self.inputs_need_grad else None
        self.aux_arrays = [[s.exe.aux_arrays[j] for s in self.shards] for j in range(len(self.aux_names))]

    # ---------------------------------------------------------------- parameters
    def set_params(self, arg_params, aux_params, allow_extra=False):
        for s in self.shards:
            s.exe.copy_params_from(arg_params, aux_params, allow_extra_params=allow_extra)

    def get_params(self, arg_params, aux_params):
        """Average each parameter over devices (host side) into the given dicts."""
        from ..context import cpu
        for names, arrays, dst in ((self.param_names, self.param_arrays, arg_params),
                                   (self.aux_names, self.aux_arrays, aux_params)):
            for name, per_dev in zip(names, arrays):
                mean = sum(a.copyto(cpu()) for a in per_dev) / len(per_dev)
                mean.astype(dst[name].dtype).copyto(dst[name])

    # ---------------------------------------------------------------- compute
    def forward(self, data_batch, is_train=None):
        _load_general(data_batch.data, self.data_arrays, self.data_layouts[0] if self.data_layouts else 0)
        if self.label_arrays and data_batch.label:
            _load_general(data_batch.label, self.label_arrays, self.label_layouts[0] if self.label_layouts else 0)
        train = self.for_training if is_train is None else is_train
        for s in self.shards:
            s.exe.forward(is_train=train)

    def backward(self, out_grads=None):
        if not self.for_training:
            raise AssertionError('bind with for_training=True to run backward')
        axes = self._output_axes() if len(self.shards) > 1 else [-1] * len(out_grads or [])
        for s in self.shards:
            heads = [(nd.slice_axis(g, axis=ax, begin=s.slice.start, end=s.slice.stop) if ax >= 0 else g)
                     .as_in_context(s.ctx) for g, ax in zip(out_grads or [], axes)]
            s.exe.backward(out_grads=heads or None)

    def get_output_shapes(self):
        """Whole-batch output shapes from shape inference (valid before any forward)."""
        known = {d.name: d.shape for d in (self.data_shapes + (self.label_shapes or [])) if d.name in self.arg_names}
        _, out_shapes, _ = self.symbol.infer_shape(**known)
        return list(zip(self.symbol.list_outputs(), [tuple(s) for s in out_shapes]))

    def _output_axes(self):
        """Batch axis of every output, from its ``__layout__`` attribute (default N first)."""
        axes = []
        for name in self.symbol.list_outputs():
            try:
                layout = self.symbol[name].attr('__layout__')
            except Exception:       # pylint: disable=broad-except
                layout = None
            axes.append(DataDesc.get_batch_axis(layout))
        return axes

    def get_outputs(self, merge_multi_context=True, begin=0, end=None):
        n_out = len(self.shards[0].exe.outputs)
        end = n_out if end is None else end
        picked = [[s.exe.outputs[i] for s in self.shards] for i in range(begin, end)]
        return _merge_multi_context(picked, self._output_axes()[begin:end]) if merge_multi_context else picked

    def get_input_grads(self, merge_multi_context=True):
        if not self.inputs_need_grad:
            raise AssertionError('bind with inputs_need_grad=True to get input gradients')
        g = self.input_grad_arrays
        return _merge_multi_context(g, list(self.data_layouts)) if merge_multi_context else g

    def get_states(self, merge_multi_context=True):
        if merge_multi_context:
            raise AssertionError('states are per device; call with merge_multi_context=False')
        return [[s.exe.arg_dict[n] for s in self.shards] for n in self.state_names]

    def set_states(self, states=None, value=None):
        targets = self.get_states(False)
        if states is not None:
            if value is not None:
                raise AssertionError('give either states or value')
            _load_general(states, targets, -1)
            return
        for per_dev in targets:
            for arr in per_dev:
                arr[:] = value

    def update_metric(self, eval_metric, labels, pre_sliced=False):
        outputs = self.symbol.list_outputs()
        for i, s in enumerate(self.shards):
            if pre_sliced:
                mine = labels[i]
            elif len(self.shards) > 1:
                mine = [nd.slice_axis(l, axis=0, begin=s.slice.start, end=s.slice.stop)
                        if l.shape[0] == self.batch_size else l for l in labels]
            else:
                mine = labels
            eval_metric.update_dict(dict(zip(self.label_names, mine)), dict(zip(outputs, s.exe.outputs)))

    def install_monitor(self, mon):
        for s in self.shards:
            mon.install(s.exe)
