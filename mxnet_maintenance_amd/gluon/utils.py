"""Gluon utilities.

Parity: python/mxnet/gluon/utils.py (split_data, split_and_load,
clip_global_norm, check_sha1, download, HookHandle, shape_is_known).
``clip_global_norm`` computes all squared norms in one multi-tensor pass
(torch._foreach_norm) and scales in place without a host sync unless asked.
"""
import hashlib
import math
import os
import uuid
import warnings
import weakref
from collections import OrderedDict

import numpy as np
import torch

from .. import ndarray
from ..ndarray.ndarray import NDArray

__all__ = ['split_data', 'split_and_load', 'clip_global_norm', 'check_sha1', 'download', 'shape_is_known',
           'HookHandle']


def split_data(data, num_slice, batch_axis=0, even_split=True):
    size = data.shape[batch_axis]
    if even_split and size % num_slice != 0:
        raise ValueError(
            "data with shape %s cannot be evenly split into %d slices along axis %d. Use a batch size that's "
            "multiple of %d or set even_split=False to allow uneven partitioning of data." % (
                str(data.shape), num_slice, batch_axis, num_slice))
    n_each_section, extras = divmod(size, num_slice)
    section_sizes = [0] + (extras * [n_each_section + 1] + (num_slice - extras) * [n_each_section])
    div_points = np.array(section_sizes).cumsum()
    if not even_split and size < num_slice:
        num_slice = size
        div_points = list(range(size + 1))
    slices = []
    if getattr(data, 'stype', 'default') == 'csr':
        # compressed row slices keep the CSR storage
        if batch_axis != 0:
            raise ValueError('CSRNDArray can only be split along axis 0, got %d' % batch_axis)
        return [data[int(div_points[i]):int(div_points[i + 1])] for i in range(num_slice)]
    for i in range(num_slice):
        st, end = int(div_points[i]), int(div_points[i + 1])
        idx = [slice(None)] * data.ndim
        idx[batch_axis] = slice(st, end)
        slices.append(NDArray(data._data[tuple(idx)]))
    return slices


def _upload(slices, ctx_list):
    """Host -> GPU copies of the batch slices as engine device ops on each GPU's copy stream
    (engine.host_to_device): they overlap the compute still queued on the consumer streams, which
    wait for their slice with a HIP event -- no host sync.
    Parity: the reference's CopyFromTo pushed to the ThreadedEnginePerDevice copy workers
    (src/engine/threaded_engine_perdevice.cc, src/ndarray/ndarray.cc CopyFromTo)."""
    from .. import engine
    from .. import autograd
    outs = []
    for s, ctx in zip(slices, ctx_list):
        t = s._data
        if (ctx.device_type != 'gpu' or t.device.type != 'cpu' or not torch.cuda.is_available()
                or (autograd.is_recording() and t.requires_grad)):
            outs.append(s.as_in_context(ctx))
            continue
        dst, var = engine.host_to_device(t, torch.device('cuda', ctx.device_id), name='split_and_load_h2d')
        out = NDArray(dst)
        out._engine_var = var
        outs.append(out)
    return outs


def wait_host_reads(ptr, nbytes):
    """Block until every pending H2D copy reading ``[ptr, ptr + nbytes)`` has finished (see
    engine.wait_host_reads)."""
    from .. import engine
    engine.wait_host_reads(ptr, nbytes)


def split_and_load(data, ctx_list, batch_axis=0, even_split=True):
    if not isinstance(data, NDArray):
        data = ndarray.array(data)      # host first: the per-device slices then go up as async copies
    if len(ctx_list) == 1:
        return _upload([data], ctx_list)
    slices = split_data(data, len(ctx_list), batch_axis, even_split)
    return _upload(slices, ctx_list)


def clip_global_norm(arrays, max_norm, check_isfinite=True):
    """Rescale arrays so that the sum of their 2-norms is at most ``max_norm``."""
    assert len(arrays) > 0
    tensors = [a._data for a in arrays]
    with torch.no_grad():
        norms = torch._foreach_norm(tensors)
        total = torch.linalg.vector_norm(torch.stack([n.float().to(tensors[0].device) for n in norms]))
        scale = torch.clamp(max_norm / (total + 1e-8), max=1.0)
        if check_isfinite:
            tn = float(total)
            if not math.isfinite(tn):
                warnings.warn(UserWarning('nan or inf is detected. Clipping results will be undefined.'),
                              stacklevel=2)
        torch._foreach_mul_(tensors, scale.to(tensors[0].dtype))
    if check_isfinite:
        return float(total)
    return NDArray(total.reshape(1))


def _indent(s_, numSpaces):
    s = s_.split('\n')
    if len(s) == 1:
        return s_
    first = s.pop(0)
    s = [first] + [(numSpaces * ' ') + line for line in s]
    return '\n'.join(s)


def check_sha1(filename, sha1_hash):
    sha1 = hashlib.sha1()
    with open(filename, 'rb') as f:
        while True:
            data = f.read(1048576)
            if not data:
                break
            sha1.update(data)
    return sha1.hexdigest() == sha1_hash


def download(url, path=None, overwrite=False, sha1_hash=None, retries=5, verify_ssl=True):
    """Download is unavailable in this offline build unless the file already exists."""
    if path is None:
        fname = url.split('/')[-1]
    else:
        path = os.path.expanduser(path)
        fname = os.path.join(path, url.split('/')[-1]) if os.path.isdir(path) else path
    if os.path.exists(fname) and not overwrite and (not sha1_hash or check_sha1(fname, sha1_hash)):
        return fname
    raise RuntimeError('download(%s): no network access on this host; place the file at %s' % (url, fname))


def _get_repo_url():
    return os.environ.get('MXNET_GLUON_REPO', 'https://apache-mxnet.s3-accelerate.dualstack.amazonaws.com/')


def _get_repo_file_url(namespace, filename):
    return '{base_url}{namespace}/{filename}'.format(base_url=_get_repo_url(), namespace=namespace,
                                                     filename=filename)


def _brief_print_list(lst, limit=7):
    lst = list(lst)
    if len(lst) > limit:
        return _brief_print_list(lst[:limit // 2], limit) + ', ..., ' + _brief_print_list(lst[-limit // 2:], limit)
    return ', '.join(["'%s'" % str(i) for i in lst])


class HookHandle:
    """A handle that can detach a registered hook."""

    def __init__(self):
        self._hooks_dict_ref = None
        self._id = None

    def attach(self, hooks_dict, hook):
        assert not self._hooks_dict_ref, 'The same handle cannot be attached twice.'
        self._id = id(hook)
        hooks_dict[self._id] = hook
        self._hooks_dict_ref = weakref.ref(hooks_dict)

    def detach(self):
        hooks_dict = self._hooks_dict_ref()
        if hooks_dict is not None and self._id in hooks_dict:
            del hooks_dict[self._id]

    def __getstate__(self):
        return (self._hooks_dict_ref(), self._id)

    def __setstate__(self, state):
        if state[0] is None:
            self._hooks_dict_ref = weakref.ref(OrderedDict())
        else:
            self._hooks_dict_ref = weakref.ref(state[0])
        self._id = state[1]

    def __enter__(self):
        return self

    def __exit__(self, ptype, value, trace):
        self.detach()


def shape_is_known(shape):
    if shape is None:
        return False
    unknown_dim_size = 0
    if len(shape) == 0:
        return unknown_dim_size == -1
    for dim_size in shape:
        if dim_size == unknown_dim_size:
            return False
        assert dim_size > unknown_dim_size, 'shape dimension size cannot be less than {}, while ' \
                                            'received {}'.format(unknown_dim_size, dim_size)
    return True
