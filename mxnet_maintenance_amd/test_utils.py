"""Testing utilities (parity: python/mxnet/test_utils.py).

Numerical comparison helpers, random array/shape generators, numeric
(finite-difference) gradient checking, symbolic forward/backward checks,
cross-context consistency checks, statistical generator checks and small
data helpers (offline: MNIST is synthesised when the files are absent).
"""
import contextlib
import functools
import os
import random as _pyrandom
import sys
from contextlib import contextmanager

import numpy as np
import numpy.random as rnd            # noqa: F401  (re-exported, as the reference module does)
import numpy.testing as npt           # noqa: F401
from collections import OrderedDict   # noqa: F401

import gzip                           # noqa: F401  (the reference module's imports are part of
import json                           # noqa: F401   its ``from mxnet.test_utils import *`` surface)
import logging                        # noqa: F401
import numbers                        # noqa: F401
import time                           # noqa: F401
import traceback                      # noqa: F401

from . import ndarray as nd
from . import symbol as sym_mod
mx = sys.modules[__package__]   # the framework package: tests reach ``mx`` through the star import
from .base import MXNetError
from .context import Context, cpu, gpu, current_context
from .ndarray import array            # noqa: F401  (tests use it via ``from mxnet.test_utils import *``)
from .ndarray.ndarray import NDArray, _STORAGE_TYPE_STR_TO_ID   # noqa: F401
from .symbol import Symbol            # noqa: F401
from .util import use_np, getenv, setenv   # noqa: F401
from .runtime import Features         # noqa: F401

_default_ctx = [None]


def default_context():
    """Context used by tests: this thread's default context (MXNET_TEST_DEVICE=gpu selects the first
    GPU while no context was set)."""
    from .context import Context
    if getattr(Context._default_ctx, 'value', None) is None and os.environ.get('MXNET_TEST_DEVICE', 'cpu') == 'gpu':
        return gpu(0)
    return current_context()


def set_default_context(ctx):
    """Set this thread's default context (``Context.default_ctx``)."""
    from .context import Context
    Context.default_ctx = ctx


def default_dtype():
    return np.float32


def default_rtols():
    return {np.dtype(np.float16): 1e-2, np.dtype(np.float32): 1e-4, np.dtype(np.float64): 1e-5,
            np.dtype(np.bool_): 0, np.dtype(np.int8): 0, np.dtype(np.uint8): 0, np.dtype(np.int32): 0,
            np.dtype(np.int64): 0}


def default_atols():
    return {np.dtype(np.float16): 1e-1, np.dtype(np.float32): 1e-3, np.dtype(np.float64): 1e-20,
            np.dtype(np.bool_): 0, np.dtype(np.int8): 0, np.dtype(np.uint8): 0, np.dtype(np.int32): 0,
            np.dtype(np.int64): 0}


def default_numeric_eps():
    return {np.dtype(np.float16): 1.0 / 2 ** 6, np.dtype(np.float32): 1.0 / 2 ** 9,
            np.dtype(np.float64): 1.0 / 2 ** 14}


def _np(a):
    if isinstance(a, NDArray):
        return a.asnumpy()
    return np.asarray(a)


def effective_dtype(dat):
    dt = _np(dat).dtype if not isinstance(dat, NDArray) else np.dtype(dat.dtype)
    return dt


def get_tolerance(dat, tol, default_tol):
    if isinstance(tol, (float, int)):
        return tol
    dt = effective_dtype(dat)
    if isinstance(tol, dict):
        return tol.get(dt, default_tol.get(dt, 0))
    return default_tol.get(dt, 1e-5)


def get_tols(x, y, rtol, atol):
    if isinstance(x, (int, float)):
        x = np.array(x)
    rtol = max(get_tolerance(x, rtol, default_rtols()), get_tolerance(y, rtol, default_rtols()))
    atol = max(get_tolerance(x, atol, default_atols()), get_tolerance(y, atol, default_atols()))
    return rtol, atol


def get_atol(atol=None, dtype=np.dtype(np.float64)):
    return default_atols().get(np.dtype(dtype), 1e-20) if atol is None else atol


def get_rtol(rtol=None, dtype=np.dtype(np.float64)):
    return default_rtols().get(np.dtype(dtype), 1e-5) if rtol is None else rtol


def get_etol(etol=None):
    return 0 if etol is None else etol


def random_arrays(*shapes):
    """Standard-normal float32 numpy arrays of the given shapes (scalars for ``()``)."""
    arrays = [np.array(np.random.randn(), dtype=default_dtype()) if len(s) == 0 else
              np.random.randn(*s).astype(default_dtype()) for s in shapes]
    if len(arrays) == 1:
        return arrays[0]
    return arrays


def random_uniform_arrays(*shapes, **kwargs):
    """Uniform [low, high) numpy arrays (keyword args ``low``, ``high``, ``dtype``)."""
    lo, hi = kwargs.pop('low', 0.0), kwargs.pop('high', 1.0)
    out_dtype = kwargs.pop('dtype', default_dtype())
    return [np.random.uniform(lo, hi, size=s).astype(out_dtype) for s in shapes]


def random_sample(population, k):
    """``k`` distinct elements of ``population`` in random order."""
    picked = list(population)
    np.random.shuffle(picked)
    return picked[:k]


def _rand_dims(limits, allow_zero_size):
    first = 0 if allow_zero_size else 1
    return tuple(int(np.random.randint(first, d + 1)) for d in limits)


def rand_shape_2d(dim0=10, dim1=10, allow_zero_size=False):
    return _rand_dims((dim0, dim1), allow_zero_size)


def rand_shape_3d(dim0=10, dim1=10, dim2=10, allow_zero_size=False):
    return _rand_dims((dim0, dim1, dim2), allow_zero_size)


def rand_shape_nd(num_dim, dim=10, allow_zero_size=False):
    return _rand_dims((dim,) * num_dim, allow_zero_size)


def rand_coord_2d(x_low, x_high, y_low, y_high):
    return _pyrandom.randint(x_low, x_high), _pyrandom.randint(y_low, y_high)


def _powerlaw_csr_parts(num_rows, num_cols, density, dtype):
    """Row r stores min(2**r, num_cols) leading columns until int(density * size) values are placed
    (the "powerlaw" layout of the reference generator: every row twice as dense as the previous one)."""
    total = int(num_rows * num_cols * density)
    counts = []
    left, k = total, 1
    for _ in range(num_rows):
        c = min(k, num_cols, left)
        counts.append(c)
        left -= c
        k *= 2
    indptr = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    indices = np.concatenate([np.arange(c, dtype=np.int64) for c in counts]) if total else np.zeros(0, np.int64)
    data = np.random.uniform(-1, 1, size=int(indptr[-1])).astype(dtype)
    return data, indices, indptr


def rand_sparse_ndarray(shape, stype, density=None, dtype=None, distribution=None, data_init=None,
                        rsp_indices=None, modifier_func=None, shuffle_csr_indices=False, ctx=None):
    """Random sparse array built directly in compressed form.

    Returns ``(array, (values, indices))`` for row_sparse and ``(array, (indptr, indices, data))`` for
    csr, like the reference helper.  ``distribution``: 'uniform' (default) or 'powerlaw' (csr only).
    """
    density = np.random.rand() if density is None else density
    dtype = default_dtype() if dtype is None else dtype
    if stype == 'row_sparse':
        if rsp_indices is not None:
            idx = np.unique(np.asarray(rsp_indices, dtype=np.int64))
        else:
            idx = np.argwhere(np.random.rand(shape[0]) < density).flatten().astype(np.int64)
        vshape = (len(idx),) + tuple(shape[1:])
        val = np.full(vshape, data_init, dtype=dtype) if data_init is not None else \
            np.random.rand(*vshape).astype(dtype)
        if modifier_func is not None and val.size:
            val = np.vectorize(modifier_func)(val).astype(dtype)
        arr = nd.sparse.row_sparse_array((val, idx), shape=shape, ctx=ctx, dtype=dtype)
        return arr, (val, idx)
    if stype == 'csr':
        assert len(shape) == 2, 'csr arrays are 2-D'
        if distribution == 'powerlaw':
            data, indices, indptr = _powerlaw_csr_parts(shape[0], shape[1], density, dtype)
        else:
            mask = np.random.rand(*shape) < density
            counts = mask.sum(1)
            indptr = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
            indices = np.nonzero(mask)[1].astype(np.int64)
            if shuffle_csr_indices:
                for r in range(shape[0]):
                    np.random.shuffle(indices[indptr[r]:indptr[r + 1]])
            data = np.full(len(indices), data_init, dtype=dtype) if data_init is not None else \
                np.random.rand(len(indices)).astype(dtype)
        if modifier_func is not None and data.size:
            data = np.vectorize(modifier_func)(data).astype(dtype)
        arr = nd.sparse.csr_matrix((data, indices, indptr), shape=shape, ctx=ctx, dtype=dtype)
        return arr, (indptr, indices, data)
    raise ValueError('unknown storage type %s' % stype)


def rand_ndarray(shape, stype='default', density=None, dtype=None, modifier_func=None,
                 shuffle_csr_indices=False, distribution=None, ctx=None):
    ctx = ctx or default_context()
    if stype == 'default':
        arr = np.random.uniform(-1, 1, size=shape).astype(dtype or default_dtype())
        return nd.array(arr if modifier_func is None else np.vectorize(modifier_func)(arr), ctx=ctx,
                        dtype=dtype or default_dtype())
    return rand_sparse_ndarray(shape, stype, density=density, dtype=dtype, modifier_func=modifier_func,
                               shuffle_csr_indices=shuffle_csr_indices, distribution=distribution, ctx=ctx)[0]


def create_sparse_array(shape, stype, data_init=None, rsp_indices=None, dtype=None, modifier_func=None,
                        density=.5, shuffle_csr_indices=False):
    return rand_sparse_ndarray(shape, stype, density=density, dtype=dtype, data_init=data_init,
                               rsp_indices=rsp_indices, modifier_func=modifier_func)[0]


def np_reduce(dat, axis, keepdims, numpy_reduce_func):
    """Apply a single-axis numpy reduction over several axes (highest axis first)."""
    if axis is None:
        axes = list(range(dat.ndim))
    else:
        axes = [a % max(dat.ndim, 1) for a in ([axis] if isinstance(axis, int) else axis)]
    out = dat
    for ax in sorted(axes, reverse=True):
        out = numpy_reduce_func(out, axis=ax)
    if not keepdims:
        return out
    kept = [1 if d in axes else n for d, n in enumerate(dat.shape)]
    return out.reshape(kept)


def _find_max_violation(a, b, rtol, atol):
    """(index, ratio) of the element whose |a-b| most exceeds atol + rtol*|b|."""
    ratio = np.abs(a - b) / (atol + rtol * np.abs(b) + 1e-20)
    flat = int(np.argmax(ratio))
    return np.unravel_index(flat, ratio.shape), ratio.reshape(-1)[flat]


def same(a, b):
    return np.array_equal(_np(a), _np(b))


def checkShapes(a, b):
    if a.shape != b.shape:
        msg = 'Shape mismatch: %s vs %s' % (str(a.shape), str(b.shape))
        raise AssertionError(msg)


def almost_equal(a, b, rtol=None, atol=None, equal_nan=False, use_broadcast=True):
    a, b = _np(a), _np(b)
    rtol, atol = get_tols(a, b, rtol, atol)
    if not use_broadcast:
        checkShapes(a, b)
    return np.allclose(a, b, rtol=rtol, atol=atol, equal_nan=equal_nan)


def locationError(a, b, index, names, maxError=False):
    return 'Error %f exceeds tolerance rtol=%f, atol=%f (mismatch at %s). Location of maximum error: %s, ' \
           '%s=%f, %s=%f' % (0, 0, 0, index, str(index), names[0], a[index], names[1], b[index])


def assert_almost_equal(a, b, rtol=None, atol=None, names=('a', 'b'), equal_nan=False, use_broadcast=True,
                        mismatches=(10, 10)):
    """Assert ``|a - b| <= atol + rtol*|b|`` elementwise, reporting the worst violation."""
    a, b = _np(a), _np(b)
    rtol, atol = get_tols(a, b, rtol, atol)
    if not use_broadcast:
        checkShapes(a, b)
    a64 = a.astype(np.float64) if a.dtype.kind in 'fiub' else a
    b64 = b.astype(np.float64) if b.dtype.kind in 'fiub' else b
    if np.allclose(a64, b64, rtol=rtol, atol=atol, equal_nan=equal_nan):
        return
    a64, b64 = np.broadcast_arrays(a64, b64)
    index, rel = _find_max_violation(a64, b64, rtol, atol)
    raise AssertionError('\nError %f exceeds tolerance rtol=%e, atol=%e.  Location of maximum error: %s, %s=%.8f, '
                         '%s=%.8f' % (rel, rtol, atol, str(index), names[0], a64[index], names[1], b64[index]))


def assert_allclose(a, b, rtol=1e-07, atol=0, equal_nan=True):
    assert_almost_equal(a, b, rtol=rtol, atol=atol, equal_nan=equal_nan)


def assert_almost_equal_with_err(a, b, rtol=None, atol=None, etol=None, names=('a', 'b'), equal_nan=False,
                                 mismatches=(10, 10)):
    etol = get_etol(etol)
    if etol > 0:
        a, b = _np(a), _np(b)
        rtol, atol = get_tols(a, b, rtol, atol)
        bad = ~np.isclose(a, b, rtol=rtol, atol=atol, equal_nan=equal_nan)
        if bad.mean() > etol:
            raise AssertionError('error rate %f exceeds etol %f' % (bad.mean(), etol))
    else:
        assert_almost_equal(a, b, rtol, atol, names, equal_nan)


def assert_almost_equal_ignore_nan(a, b, rtol=None, atol=None, names=('a', 'b')):
    a = np.copy(_np(a))
    b = np.copy(_np(b))
    nan_mask = np.logical_or(np.isnan(a), np.isnan(b))
    a[nan_mask] = 0
    b[nan_mask] = 0
    assert_almost_equal(a, b, rtol, atol, names)


def assert_exception(f, exception_type, *args, **kwargs):
    try:
        f(*args, **kwargs)
        assert False
    except exception_type:
        return


def retry(n):
    """Decorator: retry a (stochastic) test up to ``n`` times."""
    assert n > 0

    def decorate(f):
        @functools.wraps(f)
        def wrapper(*args, **kwargs):
            err = None
            for _ in range(n):
                try:
                    return f(*args, **kwargs)
                except AssertionError as e:
                    err = e
            raise err
        return wrapper
    return decorate


def simple_forward(sym, ctx=None, is_train=False, **inputs):
    ctx = ctx or default_context()
    inputs = {k: nd.array(v) if not isinstance(v, NDArray) else v for k, v in inputs.items()}
    exe = sym.bind(ctx, args=inputs)
    exe.forward(is_train=is_train)
    outputs = [x.asnumpy() for x in exe.outputs]
    if len(outputs) == 1:
        outputs = outputs[0]
    return outputs


def _arg_dtype(v, dtype):
    """dtype='asnumpy' (reference convention): every array keeps its own dtype."""
    if isinstance(dtype, str) and dtype == 'asnumpy':
        return v.dtype if hasattr(v, 'dtype') else default_dtype()
    return dtype


def _named_inputs(names, given, what):
    """Map ``given`` (dict, or a sequence in ``names`` order) to a dict keyed by ``names``."""
    if isinstance(given, dict):
        if set(given) != set(names):
            raise ValueError('%s names %s do not match the symbol\'s %s' % (what, sorted(given), sorted(names)))
        return dict(given)
    return dict(zip(names, given))


def _to_ctx(v, ctx, dtype):
    if isinstance(v, NDArray):
        return v.as_in_context(ctx)
    # reference _parse_location: numpy inputs take ``dtype`` (float32 by default) unless dtype='asnumpy'
    return nd.array(v, ctx=ctx, dtype=_arg_dtype(v, dtype))


def _parse_location(sym, location, ctx, dtype=default_dtype()):
    named = _named_inputs(sym.list_arguments(), location, 'location')
    return {k: _to_ctx(v, ctx, dtype) for k, v in named.items()}


def _parse_aux_states(sym, aux_states, ctx, dtype=default_dtype()):
    if aux_states is None:
        return None
    named = _named_inputs(sym.list_auxiliary_states(), aux_states, 'aux_states')
    return {k: _to_ctx(v, ctx, dtype) for k, v in named.items()}


def numeric_grad(executor, location, aux_states=None, eps=1e-4, use_forward_train=True, dtype=default_dtype()):
    """Central finite differences of sum(outputs) w.r.t. every input in ``location``."""
    def load_aux():
        for name, val in (aux_states or {}).items():
            executor.aux_dict[name][:] = val

    def total_output(point, name):
        executor.arg_dict[name][:] = nd.array(point.astype(dtype), dtype=dtype)
        load_aux()
        executor.forward(is_train=use_forward_train)
        return [o.asnumpy().astype(np.float64) for o in executor.outputs]

    for name, val in location.items():
        executor.arg_dict[name][:] = val
    load_aux()
    grads = {}
    for name, val in location.items():
        point = _np(val).astype(np.float64).copy()
        flat = point.reshape(-1)
        g = np.zeros(flat.size, dtype=dtype)
        for i in range(flat.size):
            x0 = flat[i]
            flat[i] = x0 + eps / 2.0
            up = total_output(point, name)
            flat[i] = x0 - eps / 2.0
            down = total_output(point, name)
            flat[i] = x0
            # elementwise differences first: unperturbed outputs cancel exactly, so the quotient
            # does not inherit the rounding of a large sum
            g[i] = sum(float((u - d).sum()) for u, d in zip(up, down)) / eps
        executor.arg_dict[name][:] = nd.array(point.astype(dtype), dtype=dtype)
        grads[name] = g.reshape(point.shape)
    return grads


def check_numeric_gradient(sym, location, aux_states=None, numeric_eps=None, rtol=None, atol=None,
                           grad_nodes=None, use_forward_train=True, ctx=None, grad_stype_dict=None,
                           dtype=default_dtype()):
    """Compare the symbol's backward against finite differences of sum(outputs * random projection)."""
    ctx = ctx or default_context()
    eps = numeric_eps if numeric_eps is not None else default_numeric_eps()[np.dtype(dtype)]
    rtol = 1e-2 if rtol is None else rtol
    atol = 1e-4 if atol is None else atol
    location = _parse_location(sym, location, ctx, dtype)
    location_npy = {k: v.asnumpy() for k, v in location.items()}
    aux_states = _parse_aux_states(sym, aux_states, ctx, dtype)
    aux_npy = {k: v.asnumpy() for k, v in aux_states.items()} if aux_states is not None else None
    if isinstance(grad_nodes, dict):
        grad_req = dict(grad_nodes)
    elif grad_nodes is None or isinstance(grad_nodes, (list, tuple)):
        grad_req = dict.fromkeys(sym.list_arguments() if grad_nodes is None else grad_nodes, 'write')
    else:
        raise ValueError('grad_nodes must be None, a list of names or a dict of grad_req')
    grad_nodes = list(grad_req)
    input_shape = {k: v.shape for k, v in location.items()}
    _, out_shape, _ = sym.infer_shape(**input_shape)
    proj = sym_mod.var('__random_proj')
    out = (sym * proj) if len(out_shape) == 1 else (sym_mod.Group(list(sym))[0] * proj)
    out = sym_mod.make_loss(out)
    location = dict(list(location.items()) + [('__random_proj', nd.array(np.random.normal(0, 0.01,
                                                                                          size=out_shape[0]),
                                                                         ctx=ctx, dtype=dtype))])
    args_grad_npy = {k: np.random.normal(0, 0.01, size=location[k].shape) for k in grad_nodes}
    args_grad_npy['__random_proj'] = np.random.normal(0, 0.01, size=out_shape[0])
    args_grad = {k: nd.array(v, ctx=ctx, dtype=dtype) for k, v in args_grad_npy.items()}
    grad_req['__random_proj'] = 'write'
    executor = out.bind(ctx, args=location, args_grad=args_grad, grad_req=grad_req, aux_states=aux_states)
    inps = executor.arg_arrays
    if len(inps) != len(location):
        raise ValueError('Executor arg_arrays and location len do not match.')
    executor.forward(is_train=True)
    executor.backward()
    symbolic_grads = {k: executor.grad_dict[k].asnumpy() for k in grad_nodes}
    numeric_gradients = numeric_grad(executor, {k: v for k, v in location_npy.items()} | {
        '__random_proj': location['__random_proj'].asnumpy()}, aux_npy, eps=eps,
        use_forward_train=use_forward_train, dtype=dtype)
    for name in grad_nodes:
        req, labels = grad_req[name], ('NUMERICAL_%s' % name, 'BACKWARD_%s' % name)
        if req not in ('write', 'add', 'null'):
            raise ValueError('Invalid grad_req %s for argument %s' % (req, name))
        got, before = symbolic_grads[name], args_grad_npy[name]
        # 'write' overwrites, 'add' accumulates onto the random initial buffer, 'null' leaves it untouched
        want = before if req == 'null' else numeric_gradients[name]
        assert_almost_equal(want, got - before if req == 'add' else got, rtol, atol, labels)


def check_symbolic_forward(sym, location, expected, rtol=None, atol=None, aux_states=None, ctx=None,
                           equal_nan=False, dtype=default_dtype()):
    ctx = ctx or default_context()
    location = _parse_location(sym, location, ctx, dtype)
    aux_states = _parse_aux_states(sym, aux_states, ctx, dtype)
    if isinstance(expected, dict):
        expected = [expected[k] for k in sym.list_outputs()]
    args_grad_data = {k: nd.empty(v.shape, ctx=ctx, dtype=_arg_dtype(v, dtype)) for k, v in location.items()}
    executor = sym.bind(ctx=ctx, args=location, args_grad=args_grad_data, aux_states=aux_states)
    for g in executor.grad_arrays:
        if g is not None:
            g[:] = 0
    executor.forward(is_train=False)
    outputs = [x.asnumpy() for x in executor.outputs]
    for output_name, expect, output in zip(sym.list_outputs(), expected, outputs):
        assert_almost_equal(expect, output, rtol, atol, ('EXPECTED_%s' % output_name, 'FORWARD_%s' % output_name),
                            equal_nan=equal_nan)
    return executor.outputs


def check_symbolic_backward(sym, location, out_grads, expected, rtol=None, atol=None, aux_states=None,
                            grad_req='write', ctx=None, grad_stypes=None, equal_nan=False, dtype=default_dtype()):
    ctx = ctx or default_context()
    location = _parse_location(sym, location, ctx, dtype)
    aux_states = _parse_aux_states(sym, aux_states, ctx, dtype)
    if isinstance(expected, (list, tuple)):
        expected = {k: v for k, v in zip(sym.list_arguments(), expected)}
    args_grad_npy = {k: np.random.normal(size=v.shape) for k, v in expected.items()}
    args_grad_data = {}
    for k, v in args_grad_npy.items():
        st = (grad_stypes or {}).get(k)
        if st is not None and st != 'default':
            # a sparse gradient buffer: the executor writes the gradient in that storage type
            args_grad_data[k] = nd.sparse.zeros(st, v.shape, ctx=ctx, dtype=_arg_dtype(location[k], dtype))
        else:
            args_grad_data[k] = nd.array(v, ctx=ctx, dtype=_arg_dtype(location[k], dtype))
    if isinstance(grad_req, str):
        grad_req = {k: grad_req for k in sym.list_arguments()}
    elif isinstance(grad_req, (list, tuple)):
        grad_req = {k: v for k, v in zip(sym.list_arguments(), grad_req)}
    executor = sym.bind(ctx=ctx, args=location, args_grad=args_grad_data, aux_states=aux_states,
                        grad_req=grad_req)
    executor.forward(is_train=True)
    if isinstance(out_grads, (tuple, list)):
        outg = [nd.array(v, ctx=ctx, dtype=_arg_dtype(v, dtype)) if not isinstance(v, NDArray) else v for v in out_grads]
    elif isinstance(out_grads, dict):
        outg = [nd.array(out_grads[k], ctx=ctx, dtype=_arg_dtype(out_grads[k], dtype)) for k in sym.list_outputs()]
    else:
        outg = out_grads
    executor.backward(outg)
    grad_arrays = {k: v for k, v in executor.grad_dict.items() if v is not None}
    grads = {k: v.asnumpy() for k, v in grad_arrays.items()}
    for name in expected:
        if grad_req[name] == 'write':
            assert_almost_equal(expected[name], grads[name], rtol, atol,
                                ('EXPECTED_%s' % name, 'BACKWARD_%s' % name), equal_nan=equal_nan)
        elif grad_req[name] == 'add':
            assert_almost_equal(expected[name], grads[name] - args_grad_npy[name], rtol, atol,
                                ('EXPECTED_%s' % name, 'BACKWARD_%s' % name), equal_nan=equal_nan)
        elif grad_req[name] == 'null':
            assert_almost_equal(args_grad_npy[name], grads[name], rtol, atol,
                                ('EXPECTED_%s' % name, 'BACKWARD_%s' % name), equal_nan=equal_nan)
    return grad_arrays


def check_speed(sym, location=None, ctx=None, N=20, grad_req=None, typ='whole', **kwargs):
    """Average seconds per forward ('forward') or forward+backward ('whole') iteration."""
    import time
    ctx = ctx or default_context()
    if grad_req is None:
        grad_req = 'write'
    if location is None:
        exe = sym.simple_bind(grad_req=grad_req, ctx=ctx, **kwargs)
        location = {k: np.random.normal(size=arr.shape, scale=1.0) for k, arr in exe.arg_dict.items()}
    else:
        exe = sym.simple_bind(grad_req=grad_req, ctx=ctx, **{k: v.shape for k, v in location.items()})
    for name, iarr in location.items():
        exe.arg_dict[name][:] = iarr.astype(exe.arg_dict[name].dtype)
    nd.waitall()
    if typ == 'whole':
        exe.forward(is_train=True)
        exe.backward(out_grads=exe.outputs)
        nd.waitall()
        tic = time.time()
        for _ in range(N):
            exe.forward(is_train=True)
            exe.backward(out_grads=exe.outputs)
        nd.waitall()
    elif typ == 'forward':
        exe.forward(is_train=False)
        nd.waitall()
        tic = time.time()
        for _ in range(N):
            exe.forward(is_train=False)
        nd.waitall()
    else:
        raise ValueError('typ can only be "whole" or "forward".')
    return (time.time() - tic) / N


def check_consistency(sym, ctx_list, scale=1.0, grad_req='write', arg_params=None, aux_params=None, tol=None,
                      raise_on_err=True, ground_truth=None, equal_nan=False, use_uniform=False, rand_type=np.float64):
    """Run ``sym`` on every (ctx, shapes, dtypes) entry of ``ctx_list`` and compare to the highest precision one."""
    if tol is None:
        tol = {np.dtype(np.float16): 1e-1, np.dtype(np.float32): 1e-3, np.dtype(np.float64): 1e-5,
               np.dtype(np.uint8): 0, np.dtype(np.int32): 0, np.dtype(np.int64): 0}
    elif isinstance(tol, (int, float)):
        tol = {np.dtype(t): tol for t in (np.float16, np.float32, np.float64, np.uint8, np.int32, np.int64)}
    assert len(ctx_list) > 1
    if isinstance(sym, sym_mod.Symbol):
        sym = [sym] * len(ctx_list)
    output_names = sym[0].list_outputs()
    arg_names = sym[0].list_arguments()
    exe_list = []
    for s, ctx in zip(sym, ctx_list):
        ctx = dict(ctx)
        c = ctx.pop('ctx')
        types = ctx.pop('type_dict', {})
        exe_list.append(s.simple_bind(c, grad_req=grad_req, type_dict=types, **ctx))
    arg_params = {} if arg_params is None else arg_params
    aux_params = {} if aux_params is None else aux_params
    for n, arr in exe_list[0].arg_dict.items():
        if n not in arg_params:
            arg_params[n] = (np.random.uniform(-scale, scale, size=arr.shape) if use_uniform else
                             np.random.normal(size=arr.shape, scale=scale)).astype(rand_type)
    for n, arr in exe_list[0].aux_dict.items():
        if n not in aux_params:
            aux_params[n] = 0
    for exe in exe_list:
        for name, arr in exe.arg_dict.items():
            arr[:] = nd.array(np.asarray(arg_params[name]), dtype=arr.dtype)
        for name, arr in exe.aux_dict.items():
            arr[:] = aux_params[name]
    dtypes = [np.dtype(exe.outputs[0].dtype) if exe.outputs else np.dtype(exe.arg_arrays[0].dtype)
              for exe in exe_list]
    for exe in exe_list:
        exe.forward(is_train=False)
    dtypes = [np.dtype(exe.outputs[0].dtype) for exe in exe_list]
    max_idx = int(np.argmax([d.itemsize for d in dtypes]))
    gt = ground_truth
    if gt is None:
        gt = exe_list[max_idx].output_dict.copy()
    for i, exe in enumerate(exe_list):
        if i == max_idx:
            continue
        for name, arr in zip(output_names, exe.outputs):
            gtarr = gt[name].astype(dtypes[i]).asnumpy() if isinstance(gt[name], NDArray) else gt[name]
            try:
                assert_almost_equal(arr.asnumpy(), gtarr, rtol=tol[dtypes[i]], atol=tol[dtypes[i]],
                                    equal_nan=equal_nan)
            except AssertionError as e:
                if raise_on_err:
                    raise e
    if grad_req != 'null':
        for exe in exe_list:
            exe.forward(is_train=True)
            exe.backward(exe.outputs)
        gt_g = {n: g for n, g in exe_list[max_idx].grad_dict.items() if g is not None}
        for i, exe in enumerate(exe_list):
            if i == max_idx:
                continue
            for name, g in exe.grad_dict.items():
                if g is None or name not in gt_g:
                    continue
                try:
                    assert_almost_equal(g.asnumpy(), gt_g[name].astype(g.dtype).asnumpy(), rtol=tol[dtypes[i]],
                                        atol=tol[dtypes[i]], equal_nan=equal_nan)
                except AssertionError as e:
                    if raise_on_err:
                        raise e
    return gt


def list_gpus():
    try:
        import torch
        return list(range(torch.cuda.device_count()))
    except Exception:
        return []


def download(url, fname=None, dirname=None, overwrite=False, retries=5):
    """No network on the target nodes: returns the local path if it exists, otherwise raises."""
    if fname is None:
        fname = url.split('/')[-1]
    if dirname is not None:
        fname = os.path.join(dirname, fname)
    if os.path.exists(fname) and not overwrite:
        return fname
    maker = _SYNTHETIC_DOWNLOADS.get(os.path.basename(fname)) if _synthetic_enabled() else None
    if maker is not None:
        cached = os.path.join(_synthetic_cache('downloads'), os.path.basename(fname))
        if not os.path.exists(cached):
            maker(cached + '.part')
            os.replace(cached + '.part', cached)
        if os.path.dirname(os.path.abspath(fname)):
            os.makedirs(os.path.dirname(os.path.abspath(fname)), exist_ok=True)
        import shutil
        shutil.copyfile(cached, fname)
        return fname
    raise MXNetError('download(%s): no network access; place the file at %s' % (url, fname))


def _make_synthetic_test_images(path, count=16, seed=5):
    """Stand-in for the reference's test_images.tar.gz: ``count`` JPEGs of varied sizes under
    ``test_images/`` (the ImageIter tests' batch arithmetic assumes 16 images)."""
    import io as _io
    import tarfile
    from PIL import Image
    rng = np.random.RandomState(seed)
    with tarfile.open(path, 'w:gz') as tar:
        for i in range(count):
            h, w = int(rng.randint(180, 400)), int(rng.randint(180, 400))
            yy, xx = np.mgrid[0:h, 0:w]
            img = np.stack([(xx * 255 // w), (yy * 255 // h), rng.randint(0, 256, size=(h, w))], 2).astype(np.uint8)
            buf = _io.BytesIO()
            Image.fromarray(img).save(buf, format='JPEG', quality=90)
            info = tarfile.TarInfo('test_images/img%02d.jpg' % i)
            info.size = len(buf.getvalue())
            buf.seek(0)
            tar.addfile(info, buf)


def get_mnist(num_train=60000, num_test=10000, seed=42):
    """MNIST arrays; synthesised deterministically (class-dependent blobs) when the dataset is absent."""
    root = os.path.join(os.environ.get('MXNET_HOME', os.path.expanduser('~/.mxnet')), 'datasets', 'mnist')
    try:
        from .gluon.data.vision import MNIST
        tr = MNIST(root, train=True)
        te = MNIST(root, train=False)
        return {'train_data': tr._data.asnumpy().transpose(0, 3, 1, 2).astype(np.float32) / 255,
                'train_label': tr._label.astype(np.float32),
                'test_data': te._data.asnumpy().transpose(0, 3, 1, 2).astype(np.float32) / 255,
                'test_label': te._label.astype(np.float32)}
    except Exception:
        rng = np.random.RandomState(seed)
        protos = rng.rand(10, 1, 28, 28).astype(np.float32)

        def make(n):
            y = rng.randint(0, 10, size=n)
            x = np.clip(protos[y] + 0.3 * rng.randn(n, 1, 28, 28).astype(np.float32), 0, 1)
            return x, y.astype(np.float32)
        trd, trl = make(num_train)
        ted, tel = make(num_test)
        return {'train_data': trd, 'train_label': trl, 'test_data': ted, 'test_label': tel}


def get_mnist_iterator(batch_size, input_shape, num_parts=1, part_index=0):
    from . import io
    mnist = get_mnist()
    flat = len(input_shape) == 1
    tr = mnist['train_data'].reshape((-1,) + tuple(input_shape)) if flat else mnist['train_data']
    te = mnist['test_data'].reshape((-1,) + tuple(input_shape)) if flat else mnist['test_data']
    n = tr.shape[0] // num_parts
    train = io.NDArrayIter(tr[part_index * n:(part_index + 1) * n], mnist['train_label'][part_index * n:
                                                                                        (part_index + 1) * n],
                           batch_size, shuffle=True)
    val = io.NDArrayIter(te, mnist['test_label'], batch_size)
    return train, val


def same_array(array1, array2):
    """True when two NDArrays share memory (writing one changes the other)."""
    probe = array2.asnumpy()
    array1[:] += 1
    moved = not same(probe, array2.asnumpy())
    array1[:] -= 1
    return moved and same(array1.asnumpy(), array2.asnumpy())


@contextmanager
def discard_stderr():
    """Silence file-descriptor-level stderr (native libraries included) inside the block."""
    fd = sys.stderr.fileno()
    saved = os.dup(fd)
    sink = os.open(os.devnull, os.O_WRONLY)
    try:
        os.dup2(sink, fd)
        yield
    finally:
        os.dup2(saved, fd)
        os.close(sink)
        os.close(saved)


class DummyIter:
    """Repeats the first batch of ``real_iter`` forever (for speed tests)."""

    def __init__(self, real_iter):
        self.batch_size = real_iter.batch_size
        self.provide_data = real_iter.provide_data
        self.provide_label = real_iter.provide_label
        self.the_batch = next(iter(real_iter))

    def __iter__(self):
        return self

    def reset(self):
        pass

    def __next__(self):
        return self.the_batch

    next = __next__


def gen_buckets_probs_with_ppf(ppf, nbuckets):
    """``nbuckets`` equal-probability intervals of a distribution given its inverse CDF."""
    assert nbuckets > 0
    edges = [ppf(q) for q in np.linspace(0.0, 1.0, nbuckets + 1)]
    return list(zip(edges[:-1], edges[1:])), [1.0 / nbuckets] * nbuckets


def _within(value, centre, half_width):
    return centre - half_width < value < centre + half_width


def mean_check(generator, mu, sigma, nsamples=1000000):
    """Sample mean within 3 standard errors of ``mu``."""
    draws = np.asarray(generator(nsamples), dtype=np.float64)
    return _within(draws.mean(), mu, 3.0 * sigma / np.sqrt(nsamples))


def var_check(generator, sigma, nsamples=1000000):
    """Unbiased sample variance within 3 standard errors of ``sigma**2`` (normal-theory SE)."""
    draws = np.asarray(generator(nsamples), dtype=np.float64)
    se = np.sqrt(2.0 * sigma ** 4 / (nsamples - 1))
    return _within(draws.var(ddof=1), sigma ** 2, 3.0 * se)


def chi_square_check(generator, buckets, probs, nsamples=1000000):
    """Pearson chi-square goodness of fit of ``generator`` samples against bucket probabilities."""
    import scipy.stats as ss
    if not isinstance(buckets, list):
        raise ValueError('buckets must be a list')
    samples = np.array(generator(nsamples)).reshape(-1)
    continuous_dist = isinstance(buckets[0], (tuple, list))
    if continuous_dist:
        buckets_npy = np.array([b for bucket in buckets for b in bucket])
        sample_bucket_ids = np.searchsorted(buckets_npy, samples, side='right')
        sample_bucket_ids = np.where(sample_bucket_ids % 2 == 1, sample_bucket_ids // 2, -1)
    else:
        lookup = {b: i for i, b in enumerate(buckets)}
        sample_bucket_ids = np.array([lookup.get(s, -1) for s in samples])
    obs_freq = np.bincount(sample_bucket_ids[sample_bucket_ids >= 0], minlength=len(buckets))
    expected_freq = np.array(probs) * nsamples
    _, p = ss.chisquare(f_obs=obs_freq, f_exp=expected_freq * obs_freq.sum() / expected_freq.sum())
    return p, obs_freq, expected_freq


def verify_generator(generator, buckets, probs, nsamples=1000000, nrepeat=5, success_rate=0.2, alpha=0.05):
    """Repeat the chi-square test; pass when at least ``success_rate`` of the p-values exceed ``alpha``."""
    runs = [chi_square_check(generator=generator, buckets=buckets, probs=probs, nsamples=nsamples)
            for _ in range(nrepeat)]
    pvals = [r[0] for r in runs]
    if sum(p > alpha for p in pvals) < nrepeat * success_rate:
        raise AssertionError('Generator test fails, Chi-square p=%s, obs_freq=%s, expected_freq=%s.'
                             % (pvals, [r[1] for r in runs], [r[2] for r in runs]))
    return pvals


def compare_ndarray_tuple(t1, t2, rtol=None, atol=None):
    """Compare (possibly nested tuples of) optimizer states; ``None`` on either side is skipped."""
    if t1 is None or t2 is None:
        return
    if not isinstance(t1, tuple):
        assert_almost_equal(t1, t2, rtol=rtol, atol=atol)
        return
    for pair in zip(t1, t2):
        compare_ndarray_tuple(*pair, rtol=rtol, atol=atol)


def compare_optimizer(opt1, opt2, shape, dtype, w_stype='default', g_stype='default', rtol=1e-4, atol=1e-5,
                      compare_states=True, ntensors=1):
    """Run one update of two optimizers on identical random weights/grads and compare."""
    if ntensors == 1:
        w1 = rand_ndarray(shape, w_stype, dtype=dtype)
        w2 = w1.copy()
        g1 = rand_ndarray(shape, g_stype, dtype=dtype)
        g2 = g1.copy()
        state1 = opt1.create_state_multi_precision(0, w1)
        state2 = opt2.create_state_multi_precision(0, w2)
        if compare_states:
            compare_ndarray_tuple(state1, state2)
        opt1.update_multi_precision(0, w1, g1, state1)
        opt2.update_multi_precision(0, w2, g2, state2)
        if compare_states:
            compare_ndarray_tuple(state1, state2, rtol=rtol, atol=atol)
        assert_almost_equal(w1, w2, rtol=rtol, atol=atol)
    else:
        # ``shape`` is a list of per-tensor shapes: opt1 updates tensor by tensor, opt2 takes the whole
        # list in one (aggregated / multi-tensor) update call
        shapes = list(shape)
        w1 = [rand_ndarray(s, w_stype, dtype=dtype) for s in shapes]
        g1 = [rand_ndarray(s, g_stype, dtype=dtype) for s in shapes]
        w2 = [w.copy() for w in w1]
        g2 = [g.copy() for g in g1]
        state2 = [opt2.create_state_multi_precision(i, w2[i]) for i in range(ntensors)]
        opt2.update_multi_precision(list(range(ntensors)), w2, g2, state2)
        for i in range(ntensors):
            state1 = opt1.create_state_multi_precision(i, w1[i])
            opt1.update_multi_precision(i, w1[i], g1[i], state1)
            if compare_states:
                compare_ndarray_tuple(state1, state2[i], rtol=rtol, atol=atol)
            assert_almost_equal(w1[i], w2[i], rtol=rtol, atol=atol)


def same_symbol_structure(sym1, sym2):
    conf = [sym1.tojson(), sym2.tojson()]
    import json
    a, b = json.loads(conf[0]), json.loads(conf[1])
    if len(a['nodes']) != len(b['nodes']):
        return False
    for n1, n2 in zip(a['nodes'], b['nodes']):
        if n1['op'] != n2['op'] or n1.get('inputs') != n2.get('inputs'):
            return False
    return True


@contextmanager
def environment(*args):
    """Temporarily set environment variables: ``environment('K', 'v')`` or ``environment({'K': 'v'})``."""
    if len(args) == 2:
        values = {args[0]: args[1]}
    elif len(args) == 1:
        values = args[0]
    else:
        raise ValueError('environment() takes (name, value) or a dict')
    old = {k: os.environ.get(k) for k in values}
    try:
        for k, v in values.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = str(v)
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def collapse_sum_like(a, shape):
    """Sum ``a`` down to a broadcast-compatible ``shape`` (the gradient of broadcasting)."""
    lead = a.ndim - len(shape)
    assert lead >= 0
    if a.size == 0 or int(np.prod(shape)) == 0:
        return np.zeros(shape, dtype=a.dtype)
    reduce_axes = list(range(lead))
    for i, n in enumerate(shape):
        if n != a.shape[lead + i]:
            assert n == 1, 'shape %s is not broadcast-compatible with %s' % (shape, a.shape)
            reduce_axes.append(lead + i)
    return a.sum(axis=tuple(reduce_axes)).reshape(shape)


def is_op_runnable():
    return True


def assert_raises_cudnn_not_satisfied(min_version):
    def test_helper(orig_test):
        return orig_test
    return test_helper


# ---------------------------------------------------------------------------------------------
# small array builders / elementwise helpers used across the reference unit tests
# ---------------------------------------------------------------------------------------------

def assign_each(the_input, function):
    """``function`` applied to every element of a numpy array (identity copy when None)."""
    arr = np.asarray(the_input)
    if function is None:
        return np.array(arr)
    return np.vectorize(function, otypes=[np.float64])(arr) if arr.size else np.zeros(arr.shape)


def assign_each2(input1, input2, function):
    """``function(a, b)`` over matching elements of two same-shape numpy arrays."""
    a, b = np.asarray(input1), np.asarray(input2)
    if function is None:
        return np.array(a)
    if a.shape != b.shape:
        raise AssertionError('assign_each2: shapes differ: %s vs %s' % (a.shape, b.shape))
    return np.vectorize(function, otypes=[np.float64])(a, b) if a.size else np.zeros(a.shape)


def create_vector(size, dtype=np.int64):
    """0 .. size-1 as an NDArray (large-tensor tests)."""
    return nd.arange(0, size, dtype=dtype)


def create_2d_tensor(rows, columns, dtype=np.int64):
    """rows x columns NDArray whose row i is filled with i."""
    return nd.broadcast_to(nd.arange(0, rows, dtype=dtype).reshape((rows, 1)), shape=(rows, columns))


def get_identity_mat(size):
    return nd.array(np.eye(size, dtype=np.float32))


def get_identity_mat_batch(size):
    eye = np.eye(size, dtype=np.float32)
    return nd.array(np.stack([eye, eye]))


def shuffle_csr_column_indices(csr):
    """Shuffle the column indices inside every row of a CSR matrix (unordered-index validation)."""
    indptr = np.asarray(csr.indptr.asnumpy() if hasattr(csr.indptr, 'asnumpy') else csr.indptr)
    for row in range(len(indptr) - 1):
        lo, hi = int(indptr[row]), int(indptr[row + 1])
        seg = np.array(csr.indices[lo:hi].asnumpy() if hasattr(csr.indices, 'asnumpy') else csr.indices[lo:hi])
        np.random.shuffle(seg)
        csr.indices[lo:hi] = seg


def create_sparse_array_zd(shape, stype, density, data_init=None, rsp_indices=None, dtype=None,
                           modifier_func=None, shuffle_csr_indices=False):
    """Sparse array that may have zero density (row_sparse: only ``rsp_indices`` rows)."""
    if stype == 'row_sparse':
        density = 0.0
        if rsp_indices is not None and len(rsp_indices) > shape[0]:
            raise AssertionError('more row indices than rows')
    return create_sparse_array(shape, stype, data_init=data_init, rsp_indices=rsp_indices, dtype=dtype,
                               modifier_func=modifier_func, density=density,
                               shuffle_csr_indices=shuffle_csr_indices)


# ---- matrices with controlled spectra (linalg operator tests) --------------------------------

def new_orthonormal_matrix_2d(n):
    """A random n x n orthonormal matrix (Q of a QR factorisation)."""
    g = np.random.randn(n, n)
    return np.linalg.qr(g.T @ g)[0]


def new_sym_matrix_with_real_eigvals_2d(n):
    """Q^T D Q: symmetric, eigenvalues uniform in [-10, 10]."""
    q = new_orthonormal_matrix_2d(n)
    return q.T @ np.diag(np.random.uniform(-10.0, 10.0, n)) @ q


def new_sym_matrix_with_real_eigvals_nd(shape):
    batch = int(np.prod(shape[:-2])) if len(shape) > 2 else 1
    return np.stack([new_sym_matrix_with_real_eigvals_2d(shape[-1]) for _ in range(batch)]).reshape(shape)


def new_matrix_with_real_eigvals_2d(n):
    """A non-symmetric matrix with real eigenvalues: P D P^-1 with a well-conditioned P."""
    while True:
        house = np.eye(n) - 2 * np.outer(*(lambda v: (v, v))(
            (lambda v: v / np.linalg.norm(v))(np.random.uniform(-1.0, 1.0, n))))
        p = house @ np.diag(np.random.uniform(-1.0, 1.0, n))
        if np.linalg.cond(p, 2) < 3:
            break
    return p @ np.diag(np.random.uniform(-10.0, 10.0, n)) @ np.linalg.inv(p)


def new_matrix_with_real_eigvals_nd(shape):
    batch = int(np.prod(shape[:-2])) if len(shape) > 2 else 1
    return np.stack([new_matrix_with_real_eigvals_2d(shape[-1]) for _ in range(batch)]).reshape(shape)


# ---- gluon hybridization consistency ---------------------------------------------------------

def check_gluon_hybridize_consistency(net_builder, data_l, numpy_func=None, test_grad=True, rtol=1E-4,
                                      atol=1E-4):
    """Outputs (and input gradients) of a block built by ``net_builder()`` agree between eager
    execution and ``hybridize()`` (and with ``numpy_func`` when given).  The block must be
    deterministic; both copies share one parameter file."""
    import tempfile
    from . import autograd
    saved = None
    results = []
    for hybrid in (False, True):
        net = net_builder()
        net.initialize()
        if saved is None:
            net(*data_l)
            saved = os.path.join(tempfile.mkdtemp(), 'params')
            net.save_parameters(saved)
        else:
            net(*data_l)
            net.load_parameters(saved)
        if hybrid:
            net.hybridize()
        inputs = [d.copy() for d in data_l]
        for d in inputs:
            d.attach_grad()
        with autograd.record():
            out = net(*inputs)
        outs = out if isinstance(out, (list, tuple)) else [out]
        if test_grad:
            autograd.backward(outs)
        results.append(([o.asnumpy() for o in outs], [d.grad.asnumpy() for d in inputs] if test_grad else []))
    (o0, g0), (o1, g1) = results
    for a, b in zip(o0, o1):
        assert_almost_equal(a, b, rtol=rtol, atol=atol)
    for a, b in zip(g0, g1):
        assert_almost_equal(a, b, rtol=rtol, atol=atol)
    if numpy_func is not None:
        ref = numpy_func(*[d.asnumpy() for d in data_l])
        for a, b in zip(o0, ref if isinstance(ref, (list, tuple)) else [ref]):
            assert_almost_equal(a, b, rtol=rtol, atol=atol)


# ---- environment probes / offline data ---------------------------------------------------------

def is_cd_run():
    return os.environ.get('CD_JOB', '0') == '1'


def is_aarch64_run():
    import platform
    return platform.machine() == 'aarch64'


def has_tvm_ops():
    """No TVM-generated operators in this build (gfx950 kernels are hand-written HIP)."""
    return False


def get_im2rec_path(home_env='MXNET_HOME'):
    """Path of the im2rec tool of this repository (tools/im2rec.py)."""
    root = os.environ.get(home_env) or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return os.path.join(root, 'tools', 'im2rec.py')


def _offline(what):
    raise IOError('%s: there is no network access; place the files locally and pass their path' % what)


def download_model(model_name, dst_dir='./', meta_info=None):
    _offline('download_model(%s)' % model_name)


def get_zip_data(data_dir, url, data_origin_name):
    if not os.path.exists(os.path.join(data_dir, data_origin_name)):
        _offline('get_zip_data(%s)' % url)


# Synthetic stand-ins for the reference's downloadable test datasets (there is no network).  Only
# when MXNET_TEST_SYNTHETIC_DATA=1 (set by tools/refconf): same file formats, shapes and class
# balance as the real data, random pixels.  Generated once into a cache directory and linked.
def _synthetic_enabled():
    return os.environ.get('MXNET_TEST_SYNTHETIC_DATA', '0') == '1'


def _synthetic_cache(name):
    import tempfile
    root = os.environ.get('MXNET_TEST_DATA_CACHE', os.path.join(tempfile.gettempdir(), 'mxamd_synthetic_data'))
    d = os.path.join(root, name)
    os.makedirs(d, exist_ok=True)
    return d


def _link(src, dst):
    if os.path.lexists(dst):
        return
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    os.symlink(src, dst)


def _make_synthetic_cifar10(d):
    import io as _io
    from PIL import Image
    from . import recordio
    for name, n in (('train', 50000), ('test', 10000)):
        rec = os.path.join(d, name + '.rec')
        if os.path.exists(rec):
            continue
        rng = np.random.RandomState(7 if name == 'train' else 8)
        tmp = rec + '.part'
        w = recordio.MXRecordIO(tmp, 'w')
        for i in range(n):
            img = rng.randint(0, 256, size=(32, 32, 3), dtype=np.uint8)
            buf = _io.BytesIO()
            Image.fromarray(img).save(buf, format='PNG')
            w.write(recordio.pack(recordio.IRHeader(0, float(i % 10), i, 0), buf.getvalue()))
        w.close()
        os.replace(tmp, rec)


def _make_synthetic_mnist(d):
    import struct as _struct
    for prefix, n, seed in (('train', 60000, 1), ('t10k', 10000, 2)):
        img, lab = os.path.join(d, prefix + '-images-idx3-ubyte'), os.path.join(d, prefix + '-labels-idx1-ubyte')
        if os.path.exists(img) and os.path.exists(lab):
            continue
        rng = np.random.RandomState(seed)
        with open(img + '.part', 'wb') as f:
            f.write(_struct.pack('>IIII', 2051, n, 28, 28))
            f.write(rng.randint(0, 256, size=(n, 28, 28), dtype=np.uint8).tobytes())
        with open(lab + '.part', 'wb') as f:
            f.write(_struct.pack('>II', 2049, n))
            f.write((np.arange(n) % 10).astype(np.uint8).tobytes())
        os.replace(img + '.part', img)
        os.replace(lab + '.part', lab)


def _make_synthetic_libsvm(path, n, dim, nclass, seed=3):
    if os.path.exists(path):
        return
    rng = np.random.RandomState(seed)
    with open(path + '.part', 'w') as f:
        for i in range(n):
            idx = np.sort(rng.choice(dim, size=rng.randint(1, 40), replace=False))
            f.write('%d %s\n' % (1 + i % nclass, ' '.join('%d:%.4f' % (j, rng.rand()) for j in idx)))
    os.replace(path + '.part', path)


_SYNTHETIC_LIBSVM = {'news20.t': (3993, 62061, 20)}
_SYNTHETIC_DOWNLOADS = {'test_images.tar.gz': _make_synthetic_test_images}


def get_bz2_data(data_dir, data_name, url, data_origin_name):
    path = os.path.join(data_dir, data_name)
    if os.path.exists(path):
        return
    if _synthetic_enabled() and data_name in _SYNTHETIC_LIBSVM:
        cached = os.path.join(_synthetic_cache('libsvm'), data_name)
        _make_synthetic_libsvm(cached, *_SYNTHETIC_LIBSVM[data_name])
        _link(cached, path)
        return
    _offline('get_bz2_data(%s)' % url)


def get_cifar10(path='data'):
    if os.path.isdir(os.path.join(path, 'cifar')):
        return
    if _synthetic_enabled():
        d = _synthetic_cache('cifar')
        _make_synthetic_cifar10(d)
        _link(d, os.path.join(path, 'cifar'))
        return
    _offline('get_cifar10')


def get_mnist_pkl(path='data'):
    if not os.path.exists(os.path.join(path, 'mnist.pkl.gz')):
        _offline('get_mnist_pkl')


def get_mnist_ubyte(path='data'):
    files = ['train-images-idx3-ubyte', 'train-labels-idx1-ubyte', 't10k-images-idx3-ubyte',
             't10k-labels-idx1-ubyte']
    if all(os.path.exists(os.path.join(path, f)) for f in files):
        return
    if _synthetic_enabled():
        d = _synthetic_cache('mnist')
        _make_synthetic_mnist(d)
        for f in files:
            _link(os.path.join(d, f), os.path.join(path, f))
        return
    _offline('get_mnist_ubyte')
