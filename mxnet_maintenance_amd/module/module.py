"""Module: a Symbol bound to device(s), with parameters and an optimizer.

API parity: python/mxnet/module/module.py (bind / init_params / set_params /
init_optimizer / borrow_optimizer / forward / backward / update / get_outputs
/ get_input_grads / update_metric / reshape / save_checkpoint / Module.load /
optimizer-state save & load / states / monitor / prepare for row-sparse).

State is grouped by life cycle:

* construction: the input naming (``_data_names``, ``_label_names``,
  ``_state_names``, ``_fixed_param_names``) and the derived parameter names;
* bind: a :class:`DataParallelExecutorGroup` (``_exec_group``) plus host-side
  ``_arg_params`` / ``_aux_params`` dictionaries mirroring the device arrays
  (``_params_dirty`` marks when the device copies are newer);
* init_optimizer: optimizer, kvstore and (when updating locally) an updater.
"""
import logging
import warnings

from .. import context as ctx_mod
from .. import ndarray as nd
from .. import optimizer as opt
from ..initializer import Uniform, InitDesc
from ..model import (_create_kvstore, _initialize_kvstore, _update_params, _update_params_on_kvstore,
                     load_checkpoint, save_checkpoint_symbol)
from .base_module import BaseModule, _check_input_names, _parse_data_desc
from .executor_group import DataParallelExecutorGroup

__all__ = ['Module']


def _names(seq):
    return list(seq) if seq is not None else []


class Module(BaseModule):
    """Symbolic module over one or more contexts (one per process is the MI355X norm)."""

    # reference attribute names (user code and tests reach into these)
    _exec_group = property(lambda self: self._group)
    _params_dirty = property(lambda self: self._dirty, lambda self, v: setattr(self, '_dirty', v))
    _sync_params_from_devices = property(lambda self: self._pull_params)

    def __init__(self, symbol, data_names=('data',), label_names=('softmax_label',), logger=logging,
                 context=None, work_load_list=None, fixed_param_names=None, state_names=None, group2ctxs=None,
                 compression_params=None):
        super().__init__(logger=logger)
        ctxs = context if context is not None else ctx_mod.cpu()
        self._context = [ctxs] if isinstance(ctxs, ctx_mod.Context) else list(ctxs)
        self._work_load_list = work_load_list if work_load_list is not None else [1] * len(self._context)
        if len(self._work_load_list) != len(self._context):
            raise AssertionError('work_load_list needs one entry per context')
        self._group2ctxs = group2ctxs
        self._symbol = symbol
        self._compression_params = compression_params

        self._data_names = _names(data_names)
        self._label_names = _names(label_names)
        self._state_names = _names(state_names)
        self._fixed_param_names = _names(fixed_param_names)
        for names, kind, strict in ((self._data_names, 'data', True), (self._label_names, 'label', False),
                                    (self._state_names, 'state', True),
                                    (self._fixed_param_names, 'fixed_param', True)):
            _check_input_names(symbol, names, kind, strict)
        inputs = set(self._data_names + self._label_names + self._state_names)
        self._param_names = [a for a in symbol.list_arguments() if a not in inputs]
        self._aux_names = symbol.list_auxiliary_states()
        self._output_names = symbol.list_outputs()

        self._arg_params = self._aux_params = None
        self._dirty = False
        self._group = None
        self._data_shapes = self._label_shapes = None
        self._grad_req = None
        self._optimizer = self._kvstore = self._update_on_kvstore = self._updater = None
        self._pending_opt_states = None

    # ---------------------------------------------------------------- checkpoints
    @staticmethod
    def load(prefix, epoch, load_optimizer_states=False, **kwargs):
        """A Module whose parameters come from ``prefix-symbol.json`` / ``prefix-%04d.params``."""
        sym, args, auxs = load_checkpoint(prefix, epoch)
        mod = Module(symbol=sym, **kwargs)
        mod._arg_params, mod._aux_params = args, auxs
        mod.params_initialized = True
        if load_optimizer_states:
            mod._pending_opt_states = '%s-%04d.states' % (prefix, epoch)
        return mod

    def save_checkpoint(self, prefix, epoch, save_optimizer_states=False, remove_amp_cast=True):
        save_checkpoint_symbol(prefix, self._symbol)
        params_file = '%s-%04d.params' % (prefix, epoch)
        self.save_params(params_file)
        logging.info('Saved checkpoint to "%s"', params_file)
        if save_optimizer_states:
            states_file = '%s-%04d.states' % (prefix, epoch)
            self.save_optimizer_states(states_file)
            logging.info('Saved optimizer state to "%s"', states_file)

    # ---------------------------------------------------------------- names / shapes
    @property
    def data_names(self):
        return self._data_names

    @property
    def label_names(self):
        return self._label_names

    @property
    def output_names(self):
        return self._output_names

    @property
    def data_shapes(self):
        self._require('binded')
        return self._data_shapes

    @property
    def label_shapes(self):
        self._require('binded')
        return self._label_shapes

    @property
    def output_shapes(self):
        self._require('binded')
        return self._group.get_output_shapes()

    # ---------------------------------------------------------------- parameters
    def get_params(self):
        self._require('binded', 'params_initialized')
        if self._dirty:
            self._pull_params()
        return self._arg_params, self._aux_params

    def init_params(self, initializer=Uniform(0.01), arg_params=None, aux_params=None, allow_missing=False,
                    force_init=False, allow_extra=False):
        if self.params_initialized and not force_init:
            warnings.warn('Parameters already initialized and force_init=False. init_params call ignored.',
                          stacklevel=2)
            return
        if not self.binded:
            raise AssertionError('call bind before initializing the parameters')
        attrs = self._symbol.attr_dict()

        def fill(name, arr, given):
            desc = InitDesc(name, attrs.get(name, None))
            if given is None:
                initializer(desc, arr)
            elif name in given:
                if given[name] is not arr:
                    given[name].copyto(arr)
            elif not allow_missing:
                raise RuntimeError('%s is not presented' % name)
            elif initializer is not None:
                initializer(desc, arr)

        for mine, given in ((self._arg_params, arg_params), (self._aux_params, aux_params)):
            for name in sorted(mine):
                fill(name, mine[name], given)
        self.params_initialized = True
        self._dirty = False
        self._group.set_params(self._arg_params, self._aux_params, allow_extra=allow_extra)

    def set_params(self, arg_params, aux_params, allow_missing=False, force_init=True, allow_extra=False):
        if not allow_missing:
            self.init_params(initializer=None, arg_params=arg_params, aux_params=aux_params,
                             allow_missing=False, force_init=force_init, allow_extra=allow_extra)
            return
        if self.params_initialized and not force_init:
            warnings.warn('Parameters already initialized and force_init=False. set_params call ignored.',
                          stacklevel=2)
            return
        # partial update goes straight to the devices; host dicts are refreshed lazily
        self._group.set_params(arg_params, aux_params, allow_extra=allow_extra)
        self._dirty = True
        self.params_initialized = True

    def _pull_params(self):
        self._group.get_params(self._arg_params, self._aux_params)
        if self._kvstore and self._update_on_kvstore:
            for name, val in sorted(self._arg_params.items()):
                if val.stype == 'row_sparse':
                    self._kvstore.row_sparse_pull(name, val, row_ids=nd.arange(0, val.shape[0], dtype='int64'))
        self._dirty = False

    # ---------------------------------------------------------------- binding
    def _reset_bind(self):
        self.binded = False
        self._group = None
        self._data_shapes = self._label_shapes = None

    def bind(self, data_shapes, label_shapes=None, for_training=True, inputs_need_grad=False, force_rebind=False,
             shared_module=None, grad_req='write'):
        if force_rebind:
            self._reset_bind()
        if self.binded:
            self.logger.warning('Already bound, ignoring bind()')
            return
        if inputs_need_grad and not for_training:
            raise AssertionError('inputs_need_grad requires for_training')
        self.for_training, self.inputs_need_grad, self._grad_req = for_training, inputs_need_grad, grad_req
        self._data_shapes, self._label_shapes = _parse_data_desc(self._data_names, self._label_names,
                                                                 data_shapes, label_shapes)
        shared_group = None
        if shared_module is not None:
            if not (isinstance(shared_module, Module) and shared_module.binded and shared_module.params_initialized):
                raise AssertionError('shared_module must be a bound, initialised Module')
            shared_group = shared_module._group
            if len(shared_group.execs) < len(self._context):
                raise AssertionError('shared_module has fewer devices than this module')
        self._group = DataParallelExecutorGroup(
            self._symbol, self._context, self._work_load_list, self._data_shapes, self._label_shapes,
            self._param_names, for_training, inputs_need_grad, shared_group, logger=self.logger,
            fixed_param_names=self._fixed_param_names, grad_req=grad_req, state_names=self._state_names,
            group2ctxs=self._group2ctxs)
        self._total_exec_bytes = 0
        if shared_module is not None:
            self._arg_params, self._aux_params = shared_module._arg_params, shared_module._aux_params
            self.params_initialized = True
        elif self.params_initialized:
            self._group.set_params(self._arg_params, self._aux_params)    # loaded before bind
        else:
            g = self._group
            stypes = {n: v.attrs.get('__storage_type__') for n, v in self._symbol._var_nodes().items()}
            self._arg_params = {n: nd.zeros(a[0].shape, dtype=a[0].dtype, stype=_stype_name(stypes.get(n)))
                                for n, a in zip(self._param_names, g.param_arrays)}
            self._aux_params = {n: nd.zeros(a[0].shape, dtype=a[0].dtype)
                                for n, a in zip(self._aux_names, g.aux_arrays)}
        if shared_module is not None and shared_module.optimizer_initialized:
            self.borrow_optimizer(shared_module)
        self.binded = True

    def reshape(self, data_shapes, label_shapes=None):
        self._require('binded')
        self._data_shapes, self._label_shapes = _parse_data_desc(self._data_names, self._label_names,
                                                                 data_shapes, label_shapes)
        self._group.reshape(self._data_shapes, self._label_shapes)

    # ---------------------------------------------------------------- optimizer
    def _idx2name(self, update_on_kvstore):
        names = self._group.param_names
        if update_on_kvstore:
            return dict(enumerate(names))
        ndev = len(self._context)
        return {i * ndev + k: n for k in range(ndev) for i, n in enumerate(names)}

    def init_optimizer(self, kvstore='local', optimizer='sgd', optimizer_params=(('learning_rate', 0.01),),
                       force_init=False):
        self._require('binded', 'params_initialized')
        if self.optimizer_initialized and not force_init:
            self.logger.warning('optimizer already initialized, ignoring...')
            return
        if self._dirty:
            self._pull_params()
        kv, on_kv = _create_kvstore(kvstore, len(self._context), self._arg_params)
        batch = self._group.batch_size
        if kv and 'dist' in kv.type and '_sync' in kv.type:
            batch *= kv.num_workers
        rescale = 1.0 / batch
        idx2name = self._idx2name(on_kv)
        if isinstance(optimizer, str):
            kwargs = dict(optimizer_params)
            kwargs.setdefault('rescale_grad', rescale)
            optimizer = opt.create(optimizer, sym=self.symbol, param_idx2name=idx2name, **kwargs)
        else:
            if not isinstance(optimizer, opt.Optimizer):
                raise AssertionError('optimizer must be a name or an Optimizer')
            if optimizer.rescale_grad != rescale:
                warnings.warn('Optimizer created outside Module has rescale_grad %s, not 1/batch = %s. '
                              'Is this intended?' % (optimizer.rescale_grad, rescale), stacklevel=2)
            if not optimizer.idx2name:
                optimizer.idx2name = dict(idx2name)
        self._optimizer, self._kvstore, self._update_on_kvstore = optimizer, kv, on_kv
        self._updater = None
        if kv:
            if self._compression_params:
                kv.set_gradient_compression(self._compression_params)
            if on_kv:
                kv.set_optimizer(self._optimizer)
            _initialize_kvstore(kvstore=kv, param_arrays=self._group.param_arrays, arg_params=self._arg_params,
                                param_names=self._param_names, update_on_kvstore=on_kv)
        if not on_kv:
            self._updater = opt.get_updater(optimizer)
        self.optimizer_initialized = True
        if self._pending_opt_states is not None:
            self.load_optimizer_states(self._pending_opt_states)
            self._pending_opt_states = None

    def borrow_optimizer(self, shared_module):
        """Use ``shared_module``'s optimizer / kvstore / updater (bucketing)."""
        if not shared_module.optimizer_initialized:
            raise AssertionError('shared_module has no optimizer yet')
        self._optimizer = shared_module._optimizer
        self._kvstore = shared_module._kvstore
        self._update_on_kvstore = shared_module._update_on_kvstore
        self._updater = shared_module._updater
        self.optimizer_initialized = True

    def save_optimizer_states(self, fname):
        self._require('optimizer_initialized')
        if self._update_on_kvstore:
            self._kvstore.save_optimizer_states(fname)
            return
        with open(fname, 'wb') as f:
            f.write(self._updater.get_states())

    def load_optimizer_states(self, fname):
        self._require('optimizer_initialized')
        if self._update_on_kvstore:
            self._kvstore.load_optimizer_states(fname)
            return
        with open(fname, 'rb') as f:
            self._updater.set_states(f.read())

    # ---------------------------------------------------------------- computation
    def _batch_descs(self, batch):
        """Data / label descriptors of a batch whose shapes differ from the bound ones (else None)."""
        first = batch[0] if isinstance(batch, list) else batch
        shapes = tuple(a.shape for a in first.data)
        if shapes == tuple(d.shape for d in self._data_shapes):
            return None
        relabel = lambda d, shape: type(d)(d.name, shape, d.dtype, getattr(d, 'layout', 'NCHW'))   # noqa: E731
        data = getattr(batch, 'provide_data', None) or [relabel(d, s) for d, s in zip(self._data_shapes, shapes)]
        label = getattr(batch, 'provide_label', None)
        if not label and getattr(batch, 'label', None):
            label = [relabel(d, l.shape) for d, l in zip(self._label_shapes, batch.label)]
        return data, (label or None)

    def forward(self, data_batch, is_train=None):
        self._require('binded', 'params_initialized')
        new = self._batch_descs(data_batch)
        if new is not None:
            self.reshape(*new)
        self._group.forward(data_batch, is_train)

    def backward(self, out_grads=None):
        self._require('binded', 'params_initialized')
        self._group.backward(out_grads=out_grads)

    def update(self):
        self._require('binded', 'params_initialized', 'optimizer_initialized')
        self._dirty = True
        g = self._group
        if self._update_on_kvstore:
            _update_params_on_kvstore(g.param_arrays, g.grad_arrays, self._kvstore, g.param_names)
        else:
            _update_params(g.param_arrays, g.grad_arrays, updater=self._updater, num_device=len(self._context),
                           kvstore=self._kvstore, param_names=g.param_names)

    def get_outputs(self, merge_multi_context=True):
        self._require('binded', 'params_initialized')
        return self._group.get_outputs(merge_multi_context=merge_multi_context)

    def get_input_grads(self, merge_multi_context=True):
        self._require('binded', 'params_initialized', 'inputs_need_grad')
        return self._group.get_input_grads(merge_multi_context=merge_multi_context)

    def get_states(self, merge_multi_context=True):
        self._require('binded', 'params_initialized')
        return self._group.get_states(merge_multi_context=merge_multi_context)

    def set_states(self, states=None, value=None):
        self._require('binded', 'params_initialized')
        self._group.set_states(states, value)

    def update_metric(self, eval_metric, labels, pre_sliced=False):
        self._group.update_metric(eval_metric, labels, pre_sliced)

    def install_monitor(self, mon):
        self._require('binded')
        self._group.install_monitor(mon)

    def prepare(self, data_batch, sparse_row_id_fn=None):
        """Pull the rows a batch needs of row-sparse parameters kept on the kvstore."""
        self._require('binded')
        if sparse_row_id_fn is None:
            return
        if not (self._kvstore and self._update_on_kvstore):
            warnings.warn('Parameters are not updated in the KVStore; sparse_row_id_fn is not needed.',
                          stacklevel=2)
            return
        rows = sparse_row_id_fn(data_batch)
        if not isinstance(rows, dict):
            raise AssertionError('sparse_row_id_fn must return {param_name: row_ids}')
        g = self._group
        for name, row_id in rows.items():
            idx = g.param_names.index(name)
            per_dev = g.param_arrays[idx]
            if per_dev[0].stype != 'row_sparse':
                warnings.warn("%s is not 'row_sparse'; no row_sparse_pull needed." % name, stacklevel=2)
                continue
            self._kvstore.row_sparse_pull(name, per_dev, row_ids=row_id, priority=-idx)


def _stype_name(flag):
    """Storage type of a variable's ``__storage_type__`` attribute (stype flag or name)."""
    if flag is None:
        return 'default'
    names = {'0': 'default', '1': 'row_sparse', '2': 'csr', '-1': 'default'}
    return names.get(str(flag), str(flag) if str(flag) in ('default', 'row_sparse', 'csr') else 'default')
