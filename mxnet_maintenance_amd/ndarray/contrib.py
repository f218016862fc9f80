"""Contrib operators (mx.nd.contrib), parity: python/mxnet/ndarray/contrib.py"""
from . import register as _register
from ..ops import registry as _registry
from ..ops import load_all as _load_all
_load_all()
for _n in _registry.list_ops():
    if _n.startswith('_contrib_'):
        globals()[_n[len('_contrib_'):]] = _register.make_op_function(_n)


# ---------------------------------------------------------------------------
# imperative control flow and helpers (parity: python/mxnet/ndarray/contrib.py)
# ---------------------------------------------------------------------------
import math as _math

import numpy as _np


def _as_list(x):
    return (list(x), True) if isinstance(x, (list, tuple)) else ([x], False)


def foreach(body, data, init_states):
    """``body(data_t, states) -> (outputs, new_states)`` over axis 0 of ``data``; outputs stacked."""
    from .ndarray import NDArray
    from . import stack
    data_l, data_is_list = _as_list(data)
    states = init_states
    outputs = []
    for t in range(data_l[0].shape[0]):
        d = [x[t] for x in data_l]
        out, states = body(d if data_is_list else d[0], states)
        outputs.append(out)
    if not outputs:
        return [], states
    if isinstance(outputs[0], (list, tuple)):
        res = [stack(*[o[i] for o in outputs], axis=0) for i in range(len(outputs[0]))]
    else:
        res = stack(*outputs, axis=0)
    return res, states


def while_loop(cond, func, loop_vars, max_iterations=None):
    """Imperative while loop; per-step outputs are stacked (and padded to ``max_iterations``)."""
    from .ndarray import NDArray
    from . import stack, zeros
    vars_l, vars_is_list = _as_list(loop_vars)
    outputs = []
    out_single = False
    steps = 0
    while max_iterations is None or steps < max_iterations:
        c = cond(*vars_l)
        if isinstance(c, NDArray):
            c = bool(c.asscalar())
        if not c:
            break
        out, new_vars = func(*vars_l)
        vars_l, _ = _as_list(new_vars)
        if out is not None:
            ol, is_list = _as_list(out)
            out_single = not is_list
            outputs.append(ol)
        steps += 1
    if outputs:
        stacked = []
        for i in range(len(outputs[0])):
            s = stack(*[o[i] for o in outputs], axis=0)
            if max_iterations is not None and s.shape[0] < max_iterations:
                from . import concat
                pad = zeros((max_iterations - s.shape[0],) + s.shape[1:], ctx=s.context, dtype=s.dtype)
                s = concat(s, pad, dim=0)
            stacked.append(s)
    else:
        stacked = []
    if out_single and len(stacked) == 1:
        stacked = stacked[0]
    return stacked, (vars_l if vars_is_list else vars_l[0])


def cond(pred, then_func, else_func):
    from .ndarray import NDArray
    p = bool(pred.asscalar()) if isinstance(pred, NDArray) else bool(pred)
    return then_func() if p else else_func()


def isinf(data):
    return abs(data) == _np.inf


def isfinite(data):
    is_data_not_nan = data == data
    is_data_not_infinite = abs(data) != _np.inf
    return is_data_not_infinite * is_data_not_nan


def isnan(data):
    return data != data


def rand_zipfian(true_classes, num_sampled, range_max, ctx=None):
    """Sample ``num_sampled`` candidates from an approximately log-uniform (Zipfian) distribution."""
    from . import array, log, random as _rnd
    log_range = _math.log(range_max + 1)
    rand = _rnd.uniform(0, log_range, shape=(num_sampled,), dtype='float64', ctx=ctx)
    sampled_classes = (rand.exp() - 1).astype('int64') % range_max
    true_cls = true_classes.as_in_context(sampled_classes.context).astype('float64')
    expected_count_true = ((true_cls + 2.0) / (true_cls + 1.0)).log() / log_range * num_sampled
    sampled_cls_fp64 = sampled_classes.astype('float64')
    expected_prob_sampled = ((sampled_cls_fp64 + 2.0) / (sampled_cls_fp64 + 1.0)).log() / log_range
    expected_count_sampled = expected_prob_sampled * num_sampled
    return sampled_classes, expected_count_true, expected_count_sampled


# graph operators on CSR adjacency (src/operator/contrib/dgl_graph.cc), on the compressed storage
from .dgl_graph import (dgl_csr_neighbor_uniform_sample, dgl_csr_neighbor_non_uniform_sample,  # noqa: E402,F401
                        dgl_subgraph, edge_id, dgl_adjacency, dgl_graph_compact)


# ---------------------------------------------------------------------------
# optimizer-update front ends taking Python lists (reference python/mxnet/ndarray/contrib.py:550-680):
# the registered operators take a flat, interleaved argument list (w0, g0, m0, v0, w1, ...) and a
# rescale_grad *array* (so the update can be skipped on the device for a non-finite scale)
# ---------------------------------------------------------------------------
def _rescale_array(rescale_grad, like):
    from .ndarray import NDArray
    from . import full
    if isinstance(rescale_grad, NDArray):
        return rescale_grad.as_in_context(like.context)
    return full((1,), rescale_grad, ctx=like.context)


def _interleave(*groups):
    return [a for row in zip(*groups) for a in row]


def _op(name):
    return _register.make_op_function(name)


def adamw_update(weight, grad, mean, var, rescale_grad, lr, eta, beta1=0.9, beta2=0.999, epsilon=1e-8, wd=0,
                 clip_gradient=-1, out=None, name=None, **kwargs):
    return _op('_adamw_update')(weight, grad, mean, var, _rescale_array(rescale_grad, weight), lr=lr, eta=eta,
                                beta1=beta1, beta2=beta2, epsilon=epsilon, wd=wd, clip_gradient=clip_gradient,
                                out=out, **kwargs)


def mp_adamw_update(weight, grad, mean, var, weight32, rescale_grad, lr, eta, beta1=0.9, beta2=0.999,
                    epsilon=1e-8, wd=0, clip_gradient=-1, out=None, name=None, **kwargs):
    return _op('_mp_adamw_update')(weight, grad, mean, var, weight32, _rescale_array(rescale_grad, weight), lr=lr,
                                   eta=eta, beta1=beta1, beta2=beta2, epsilon=epsilon, wd=wd,
                                   clip_gradient=clip_gradient, out=out, **kwargs)


def multi_adamw_update(weights, grads, mean, var, rescale_grad, lrs, wds, etas, out=None, name=None, size=0,
                       **kwargs):
    args = _interleave(weights, grads, mean, var) + [_rescale_array(rescale_grad, weights[0])]
    return _op('_multi_adamw_update')(*args, out=out, num_weights=size or len(weights), lrs=lrs, wds=wds,
                                      etas=etas, **kwargs)


def multi_mp_adamw_update(weights, grads, mean, var, weights32, rescale_grad, lrs, wds, etas, out=None, name=None,
                          size=0, **kwargs):
    args = _interleave(weights, grads, mean, var, weights32) + [_rescale_array(rescale_grad, weights[0])]
    return _op('_multi_mp_adamw_update')(*args, out=out, num_weights=size or len(weights), lrs=lrs, wds=wds,
                                         etas=etas, **kwargs)


def multi_lamb_update(weights, grads, mean, var, step_count, lrs, wds, out=None, num_tensors=0, **kwargs):
    return _op('_multi_lamb_update')(*_interleave(weights, grads, mean, var), out=out,
                                     num_tensors=num_tensors or len(weights), step_count=step_count,
                                     learning_rates=lrs, wds=wds, **kwargs)


def multi_mp_lamb_update(weights, grads, mean, var, weights32, step_count, lrs, wds, out=None, num_tensors=0,
                         **kwargs):
    return _op('_multi_mp_lamb_update')(*_interleave(weights, grads, mean, var, weights32), out=out,
                                        num_tensors=num_tensors or len(weights), step_count=step_count,
                                        learning_rates=lrs, wds=wds, **kwargs)
