"""NDArray serialisation (``mx.nd.save`` / ``mx.nd.load``) in MXNet's binary format.

Parity: src/ndarray/ndarray.cc:1737-2040 (NDArray::Save/Load, LegacyLoad,
kMXAPINDArrayListMagic) + include/mxnet/tuple.h (TShape::Save: int32 ndim,
int64 dims) + include/mxnet/base.h (Context::Save: int32 dev_type, dev_id) +
dmlc::Stream vector/string encoding (uint64 length prefix).

File layout::

    uint64 0x112, uint64 reserved
    uint64 n_arrays, n_arrays x NDArray
    uint64 n_names,  n_names x (uint64 len, bytes)

NDArray (V2, default storage)::

    uint32 0xF993fac9, int32 stype(0), int32 ndim, int64[ndim] shape,
    int32 dev_type, int32 dev_id, int32 type_flag, raw little-endian data

V1 (0xF993fac8) has no stype; legacy (magic = ndim) uses uint32 dims.
Sparse arrays (row_sparse = 1, csr = 2) carry storage shape + aux arrays.
"""
import io
import struct

import numpy as np
import torch

from ..base import MXNetError, dtype_to_flag, flag_to_dtype, string_types
from .ndarray import NDArray, array, empty, zeros  # noqa: F401

LIST_MAGIC = 0x112
V1_MAGIC = 0xF993FAC8
V2_MAGIC = 0xF993FAC9
V3_MAGIC = 0xF993FACA

_STYPE_ID = {'default': 0, 'row_sparse': 1, 'csr': 2}
_ID_STYPE = {v: k for k, v in _STYPE_ID.items()}


def _np_of(t):
    t = t.detach()
    if t.dtype == torch.bfloat16:
        return t.cpu().view(torch.int16).numpy()
    return t.cpu().contiguous().numpy()


def _write_shape(f, shape):
    f.write(struct.pack('<i', len(shape)))
    if shape:
        f.write(struct.pack('<%dq' % len(shape), *shape))


def _write_array(f, arr, np_shape=False):
    stype = getattr(arr, 'stype', 'default')
    f.write(struct.pack('<I', V3_MAGIC if np_shape else V2_MAGIC))
    f.write(struct.pack('<i', _STYPE_ID[stype]))
    if stype != 'default':
        aux = arr._aux_arrays()
        data = arr._values()
        _write_shape(f, data.shape)
    _write_shape(f, arr.shape)
    if len(arr.shape) == 0 and not np_shape:
        return
    ctx = arr.context
    f.write(struct.pack('<ii', 1, 0))  # always saved as a cpu array (MXNet copies to cpu)
    if stype == 'default':
        flag = dtype_to_flag(arr._data.dtype)
        f.write(struct.pack('<i', flag))
        f.write(_np_of(arr._data).tobytes())
        return
    flag = dtype_to_flag(data.dtype)
    f.write(struct.pack('<i', flag))
    for a in aux:
        f.write(struct.pack('<i', dtype_to_flag(a.dtype)))
        _write_shape(f, tuple(a.shape))
    f.write(_np_of(data).tobytes())
    for a in aux:
        f.write(_np_of(a).tobytes())


def _write_str(f, s):
    b = s.encode('utf-8')
    f.write(struct.pack('<Q', len(b)))
    f.write(b)


def save_to_stream(f, data, np_shape=None):
    if np_shape is None:
        # NumPy-shape semantics (0-d arrays are scalars, 0-size dims are real): the V3 record
        from ..util import is_np_shape
        np_shape = is_np_shape()
    if isinstance(data, NDArray):
        data = [data]
    names = []
    if isinstance(data, dict):
        names = list(data.keys())
        arrays = [data[k] for k in names]
    elif isinstance(data, (list, tuple)):
        arrays = list(data)
    else:
        raise ValueError('data needs to either be a NDArray, dict of str, NDArray pairs or a list of NDarrays.')
    for a in arrays:
        if not isinstance(a, NDArray):
            raise TypeError('save only accepts NDArray values')
    f.write(struct.pack('<QQ', LIST_MAGIC, 0))
    f.write(struct.pack('<Q', len(arrays)))
    for a in arrays:
        _write_array(f, a, np_shape)
    f.write(struct.pack('<Q', len(names)))
    for n in names:
        if not isinstance(n, string_types):
            raise TypeError('keys must be str')
        _write_str(f, n)


def save(fname, data, np_shape=None):
    """Save a list or a str->NDArray dict to ``fname`` (MXNet .params format; V3 records under
    NumPy-shape semantics)."""
    if isinstance(fname, str):
        buf = io.BytesIO()
        save_to_stream(buf, data, np_shape)
        with open(fname, 'wb') as f:
            f.write(buf.getvalue())
    else:
        save_to_stream(fname, data, np_shape)


class _Reader:
    def __init__(self, buf):
        self.buf = memoryview(buf)
        self.pos = 0

    def read(self, n):
        if self.pos + n > len(self.buf):
            raise MXNetError('Invalid NDArray file format (truncated)')
        b = self.buf[self.pos:self.pos + n]
        self.pos += n
        return b

    def unpack(self, fmt):
        n = struct.calcsize(fmt)
        return struct.unpack(fmt, self.read(n))


def _read_shape(r):
    ndim, = r.unpack('<i')
    return tuple(r.unpack('<%dq' % ndim)) if ndim > 0 else ()


def _read_data(r, flag, shape):
    dt = flag_to_dtype(flag)
    count = int(np.prod(shape)) if shape else 1
    if dt == torch.bfloat16:
        raw = np.frombuffer(r.read(2 * count), dtype=np.int16).copy()
        return torch.from_numpy(raw).view(torch.bfloat16).reshape(shape)
    npd = np.dtype(torch.empty(0, dtype=dt).numpy().dtype)
    raw = np.frombuffer(r.read(npd.itemsize * count), dtype=npd.newbyteorder('<')).copy()
    return torch.from_numpy(raw.reshape(shape))


def _check_shape_semantics(magic):
    """An array saved under numpy shape semantics (V3) loads only under them, and a legacy-semantics
    array only outside them (reference: src/ndarray/ndarray.cc:1884 NDArray::Load) -- the two
    disagree on what a 0 in a shape means."""
    from .. import _state
    np_shape = bool(_state.STATE.np_shape)
    if magic == V3_MAGIC and not np_shape:
        raise MXNetError('ndarray was saved in np shape semantics, must be loaded in the same semantics: '
                         'use `with np_shape(True)` around the load')
    if magic != V3_MAGIC and np_shape and not getattr(_state.STATE, 'np_shape_global', False):
        raise MXNetError('ndarray was not saved in np shape semantics, but is being loaded in np shape '
                         'semantics: use `with np_shape(False)` around the load')


def _read_array(r):
    magic, = r.unpack('<I')
    _check_shape_semantics(magic)
    if magic in (V2_MAGIC, V3_MAGIC):
        stype_id, = r.unpack('<i')
        stype = _ID_STYPE.get(stype_id, 'default')
        nad = {'default': 0, 'row_sparse': 1, 'csr': 2}[stype]
        sshape = _read_shape(r) if nad else None
        shape = _read_shape(r)
        if len(shape) == 0 and magic == V2_MAGIC:
            return NDArray(torch.empty(0))
        r.unpack('<ii')  # context (arrays load on cpu; caller moves them)
        flag, = r.unpack('<i')
        if nad == 0:
            return NDArray(_read_data(r, flag, shape))
        aux = []
        for _ in range(nad):
            af, = r.unpack('<i')
            aux.append((af, _read_shape(r)))
        values = _read_data(r, flag, sshape)
        aux_t = [_read_data(r, af, ash) for af, ash in aux]
        from . import sparse
        if stype == 'row_sparse':
            return sparse.row_sparse_array((values, aux_t[0]), shape=shape)
        return sparse.csr_matrix((values, aux_t[1], aux_t[0]), shape=shape)
    # V1 / legacy
    if magic == V1_MAGIC:
        shape = _read_shape(r)
    else:
        ndim = magic
        shape = tuple(r.unpack('<%dI' % ndim)) if ndim else ()
    if len(shape) == 0:
        return NDArray(torch.empty(0))
    r.unpack('<ii')
    flag, = r.unpack('<i')
    return NDArray(_read_data(r, flag, shape))


def _read_str(r):
    n, = r.unpack('<Q')
    return bytes(r.read(n)).decode('utf-8')


def load_frombuffer(buf):
    """Load arrays saved with ``save`` from a bytes-like object."""
    r = _Reader(buf)
    header, _reserved = r.unpack('<QQ')
    if header != LIST_MAGIC:
        raise MXNetError('Invalid NDArray file format')
    n, = r.unpack('<Q')
    arrays = [_read_array(r) for _ in range(n)]
    m, = r.unpack('<Q')
    names = [_read_str(r) for _ in range(m)]
    if m and m != n:
        raise MXNetError('Invalid NDArray file format')
    if names:
        return dict(zip(names, arrays))
    return arrays


def load(fname):
    """Load a list or dict of NDArrays from an MXNet .params/.nd file."""
    if not isinstance(fname, str):
        raise TypeError('fname required to be a string')
    with open(fname, 'rb') as f:
        return load_frombuffer(f.read())
