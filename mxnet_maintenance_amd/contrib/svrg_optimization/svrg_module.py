"""SVRGModule: Module trained with SVRG (Johnson & Zhang, 2013).

Every ``update_freq`` epochs the current weights are frozen into a snapshot
``w~`` held by a twin module, and the full-data gradient ``mu = grad F(w~)`` is
computed.  Each mini-batch then updates with the variance-reduced gradient

    g = grad f_i(w) - grad f_i(w~) + mu

(the twin module runs forward/backward on the same batch at ``w~``).  The
optimizer, kvstore and checkpointing are the parent Module's, so any optimizer
works; the variance-reduced gradient simply replaces the raw one before
``update``.  API parity: contrib/svrg_optimization/svrg_module.py.
"""
import logging
import time

from ...module.module import Module
from ...module.base_module import BatchEndParam, _batch_labels, _fire
from ... import metric as _metric
from ...initializer import Uniform

__all__ = ['SVRGModule']


class SVRGModule(Module):
    def __init__(self, symbol, data_names=('data',), label_names=('softmax_label',), logger=logging, context=None,
                 work_load_list=None, fixed_param_names=None, state_names=None, group2ctxs=None,
                 compression_params=None, update_freq=None):
        super().__init__(symbol, data_names=data_names, label_names=label_names, logger=logger, context=context,
                         work_load_list=work_load_list, fixed_param_names=fixed_param_names,
                         state_names=state_names, group2ctxs=group2ctxs, compression_params=compression_params)
        if not isinstance(update_freq, int) or update_freq <= 0:
            raise ValueError('update_freq must be a positive integer (epochs between full-gradient passes)')
        self.update_freq = update_freq
        self._mod_aux = Module(symbol, data_names=data_names, label_names=label_names, logger=logger,
                               context=context, work_load_list=work_load_list, fixed_param_names=fixed_param_names,
                               state_names=state_names, group2ctxs=group2ctxs)
        self._full_grads = None     # per parameter, per device: mu

    def _reset_bind(self):
        super()._reset_bind()
        self._mod_aux._reset_bind()

    def bind(self, data_shapes, label_shapes=None, for_training=True, inputs_need_grad=False, force_rebind=False,
             shared_module=None, grad_req='write'):
        super().bind(data_shapes, label_shapes, for_training, inputs_need_grad, force_rebind, shared_module,
                     grad_req)
        if for_training:
            self._mod_aux.bind(data_shapes, label_shapes, for_training, inputs_need_grad, force_rebind, None,
                               grad_req)

    def reshape(self, data_shapes, label_shapes=None):
        super().reshape(data_shapes, label_shapes=label_shapes)
        self._mod_aux.reshape(data_shapes, label_shapes=label_shapes)

    def init_params(self, initializer=Uniform(0.01), arg_params=None, aux_params=None, allow_missing=False,
                    force_init=False, allow_extra=False):
        super().init_params(initializer=initializer, arg_params=arg_params, aux_params=aux_params,
                            allow_missing=allow_missing, force_init=force_init, allow_extra=allow_extra)
        if self._mod_aux.binded:
            args, auxs = self.get_params()
            self._mod_aux.init_params(initializer=None, arg_params=args, aux_params=auxs, force_init=True)

    def init_optimizer(self, kvstore='local', optimizer='sgd', optimizer_params=(('learning_rate', 0.01),),
                       force_init=False):
        """The parent Module's optimizer, wrapped in ``_SVRGOptimizer`` so KVStore keys of full-gradient
        slots (names containing ``full``) are stored rather than stepped."""
        from ... import optimizer as _opt
        from .svrg_optimizer import _SVRGOptimizer
        super().init_optimizer(kvstore=kvstore, optimizer=optimizer, optimizer_params=optimizer_params,
                               force_init=force_init)
        inner = self._optimizer
        if isinstance(inner, _SVRGOptimizer):
            return
        wrapped = _SVRGOptimizer(inner, param_idx2name=dict(inner.idx2name), rescale_grad=inner.rescale_grad)
        self._optimizer = wrapped
        if self._update_on_kvstore and self._kvstore is not None:
            self._kvstore.set_optimizer(wrapped)
        else:
            self._updater = _opt.get_updater(wrapped)

    # ---------------------------------------------------------------- per-batch
    def forward(self, data_batch, is_train=None):
        super().forward(data_batch, is_train)
        if (self.for_training if is_train is None else is_train) and self._mod_aux.binded:
            self._mod_aux.forward(data_batch, is_train=True)

    def backward(self, out_grads=None):
        super().backward(out_grads)
        if self._mod_aux.binded:
            self._mod_aux.backward(out_grads)

    def update(self):
        self._update_svrg_gradients()
        super().update()

    def _update_svrg_gradients(self):
        """grad(w) <- grad(w) - grad(w~) + mu, for every parameter on every device."""
        if self._full_grads is None:
            return
        mine, snap = self._exec_group.grad_arrays, self._mod_aux._exec_group.grad_arrays
        for i, (g_w, g_snap, mu) in enumerate(zip(mine, snap, self._full_grads)):
            for d in range(len(g_w)):
                if g_w[d] is None:
                    continue
                g_w[d][:] = self._svrg_grads_update_rule(g_w[d], g_snap[d], mu[d])

    @staticmethod
    def _svrg_grads_update_rule(g_curr_batch_curr_weight, g_curr_batch_special_weight, g_special_weight_all_batch):
        return g_curr_batch_curr_weight - g_curr_batch_special_weight + g_special_weight_all_batch

    # ---------------------------------------------------------------- full gradient
    def update_full_grads(self, train_data):
        """Snapshot the weights into the twin module and average its gradients over ``train_data``."""
        args, auxs = self.get_params()
        self._mod_aux.set_params(args, auxs)
        train_data.reset()
        sums, nbatch = None, 0
        for batch in train_data:
            self._mod_aux.forward(batch, is_train=True)
            self._mod_aux.backward()
            grads = self._mod_aux._exec_group.grad_arrays
            if sums is None:
                sums = [[None if g is None else g.copy() for g in per_dev] for per_dev in grads]
            else:
                for acc, per_dev in zip(sums, grads):
                    for d, g in enumerate(per_dev):
                        if g is not None:
                            acc[d] += g
            nbatch += 1
        train_data.reset()
        if sums is None:
            raise ValueError('update_full_grads: empty training iterator')
        self._full_grads = [[None if g is None else g / nbatch for g in per_dev] for per_dev in sums]

    # ---------------------------------------------------------------- training loop
    def fit(self, train_data, eval_data=None, eval_metric='acc', epoch_end_callback=None, batch_end_callback=None,
            kvstore='local', optimizer='sgd', optimizer_params=(('learning_rate', 0.01),), eval_end_callback=None,
            eval_batch_end_callback=None, initializer=Uniform(0.01), arg_params=None, aux_params=None,
            allow_missing=False, force_rebind=False, force_init=False, begin_epoch=0, num_epoch=None,
            validation_metric=None, monitor=None, sparse_row_id_fn=None):
        """Module.fit with a full-gradient pass at the start of every ``update_freq``-th epoch."""
        if num_epoch is None:
            raise AssertionError('fit() needs num_epoch')
        self.bind(data_shapes=train_data.provide_data, label_shapes=train_data.provide_label, for_training=True,
                  force_rebind=force_rebind)
        if monitor is not None:
            self.install_monitor(monitor)
        self.init_params(initializer=initializer, arg_params=arg_params, aux_params=aux_params,
                         allow_missing=allow_missing, force_init=force_init)
        self.init_optimizer(kvstore=kvstore, optimizer=optimizer, optimizer_params=optimizer_params)
        validation_metric = validation_metric or eval_metric
        train_metric = eval_metric if isinstance(eval_metric, _metric.EvalMetric) else _metric.create(eval_metric)
        for epoch in range(begin_epoch, num_epoch):
            t0 = time.time()
            if (epoch - begin_epoch) % self.update_freq == 0:
                self.update_full_grads(train_data)
            train_metric.reset()
            for nbatch, batch in enumerate(train_data):
                self.forward_backward(batch)
                self.update()
                labels, pre_sliced = _batch_labels(batch)
                self.update_metric(train_metric, labels, pre_sliced=pre_sliced)
                _fire(batch_end_callback, BatchEndParam(epoch, nbatch, train_metric, locals()))
            for name, val in train_metric.get_global_name_value():
                self.logger.info('Epoch[%d] Train-%s=%f', epoch, name, val)
            self.logger.info('Epoch[%d] Time cost=%.3f', epoch, time.time() - t0)
            args, auxs = self.get_params()
            self.set_params(args, auxs)
            _fire(epoch_end_callback, epoch, self.symbol, args, auxs)
            if eval_data is not None:
                for name, val in self.score(eval_data, validation_metric, score_end_callback=eval_end_callback,
                                            batch_end_callback=eval_batch_end_callback, epoch=epoch):
                    self.logger.info('Epoch[%d] Validation-%s=%f', epoch, name, val)
            train_data.reset()

    def prepare(self, data_batch, sparse_row_id_fn=None):
        super().prepare(data_batch, sparse_row_id_fn=sparse_row_id_fn)
        if self._mod_aux.binded:
            self._mod_aux.prepare(data_batch, sparse_row_id_fn=sparse_row_id_fn)
