"""Legacy experimental autograd API (``mx.contrib.autograd``), kept for old scripts.

Parity: python/mxnet/contrib/autograd.py -- ``set_is_training`` / ``train_section`` /
``test_section`` switch recording and training mode together, ``mark_variables``,
``backward``, ``compute_gradient``, ``grad_and_loss`` and ``grad``.  Everything delegates to
the tape of ``mx.autograd``.
"""
import functools

from .. import autograd as _ag
from .. import ndarray as _nd
from ..ndarray.ndarray import NDArray

__all__ = ['set_is_training', 'TrainingStateScope', 'train_section', 'test_section', 'mark_variables',
           'backward', 'compute_gradient', 'grad_and_loss', 'grad']


def set_is_training(is_train):
    """Turn recording and training mode on/off together; returns the previous state."""
    prev = _ag.is_recording()
    _ag.set_recording(bool(is_train))
    _ag.set_training(bool(is_train))
    return prev


class TrainingStateScope:
    """``with`` scope that sets recording+training to ``enter_state`` and restores it on exit."""

    def __init__(self, enter_state):
        self._enter_state = enter_state
        self._prev = None

    def __enter__(self):
        self._prev = (_ag.is_recording(), _ag.is_training())
        _ag.set_recording(self._enter_state)
        _ag.set_training(self._enter_state)

    def __exit__(self, ptype, value, trace):
        _ag.set_recording(self._prev[0])
        _ag.set_training(self._prev[1])


def train_section():
    return TrainingStateScope(True)


def test_section():
    return TrainingStateScope(False)


def mark_variables(variables, gradients, grad_reqs='write'):
    _ag.mark_variables(variables, gradients, grad_reqs)


def backward(outputs, out_grads=None, retain_graph=False):
    if isinstance(outputs, NDArray):
        outputs = [outputs]
    if isinstance(out_grads, NDArray):
        out_grads = [out_grads]
    _ag.backward(outputs, out_grads, retain_graph=retain_graph)


def compute_gradient(outputs):
    """Deprecated alias of ``backward(outputs)``."""
    backward(outputs)


def grad_and_loss(func, argnum=None):
    """Wrap ``func`` to return ``(gradients w.r.t. the chosen NDArray arguments, loss)``."""
    @functools.wraps(func)
    def wrapped(*args):
        variables = args
        if argnum is not None:
            idx = argnum if isinstance(argnum, list) else [argnum]
            variables = [args[i] for i in idx]
        for x in variables:
            assert isinstance(x, NDArray), 'type of autograd input should be NDArray.'
        grads = [_nd.zeros_like(x) for x in variables]
        mark_variables(variables, grads)
        with train_section():
            outputs = func(*args)
        backward([outputs] if isinstance(outputs, NDArray) else outputs)
        return grads, outputs
    return wrapped


def grad(func, argnum=None):
    """Wrap ``func`` to return only the gradients of ``grad_and_loss``."""
    gl = grad_and_loss(func, argnum)

    @functools.wraps(gl)
    def wrapped(*args):
        return gl(*args)[0]
    return wrapped
