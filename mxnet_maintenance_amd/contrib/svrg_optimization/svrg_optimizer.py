"""Optimizers that route SVRG's two kinds of KVStore keys.

Parity: reference python/mxnet/contrib/svrg_optimization/svrg_optimizer.py:51.
An SVRG run keeps, next to each weight ``w``, a full-gradient slot whose name
contains ``full`` (``w_full``).  Pushing to that slot must *store* the pushed
value (the accumulated full gradient), pushing to an ordinary key must apply
the user's optimizer.  ``_SVRGOptimizer`` dispatches per key name between the
two; ``_AssignmentOptimizer`` is the storing half.
"""
from ... import optimizer as _opt

__all__ = ['_AssignmentOptimizer', '_SVRGOptimizer']

# keyword arguments the Optimizer base understands (forwarded to the wrapper itself)
_BASE_KEYS = frozenset(('rescale_grad', 'param_idx2name', 'wd', 'clip_gradient', 'learning_rate', 'lr_scheduler',
                        'sym', 'begin_num_update', 'multi_precision', 'param_dict'))


@_opt.register
class _AssignmentOptimizer(_opt.Optimizer):
    """``weight <- grad``: a KVStore push becomes an assignment (full-gradient slots)."""

    def create_state(self, index, weight):
        return None

    def update(self, index, weight, grad, state):
        weight[:] = grad


@_opt.register
class _SVRGOptimizer(_opt.Optimizer):
    """Keys whose parameter name contains ``full`` are assigned, all others go to ``default_optimizer``
    (a name, created with every keyword given here, or an Optimizer instance)."""

    def __init__(self, default_optimizer, **kwargs):
        super().__init__(**{k: v for k, v in kwargs.items() if k in _BASE_KEYS})
        self.default_opt = (_opt.create(default_optimizer, **kwargs) if isinstance(default_optimizer, str)
                            else default_optimizer)
        self.aux_opt = _opt.create(_AssignmentOptimizer.__name__)

    def _name_of(self, index):
        return index if isinstance(index, str) else self.idx2name.get(index, '')

    def _pick(self, index):
        return self.aux_opt if 'full' in self._name_of(index) else self.default_opt

    def create_state(self, index, weight):
        return self._pick(index).create_state(index, weight)

    def update(self, index, weight, grad, state):
        self._pick(index).update(index, weight, grad, state)
