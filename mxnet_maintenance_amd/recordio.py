"""RecordIO files (mx.recordio).

Parity: python/mxnet/recordio.py (MXRecordIO, MXIndexedRecordIO, IRHeader,
pack, unpack, pack_img, unpack_img).  Reading/writing goes through the native
C++ RecordIO implementation (src/native/recordio.cc); a pure-python codec is
kept for hosts without the native library.
"""
import numbers
import os
import struct
from collections import namedtuple

import numpy as np

from .base import MXNetError

__all__ = ['MXRecordIO', 'MXIndexedRecordIO', 'IRHeader', 'pack', 'unpack', 'pack_img', 'unpack_img']

_MAGIC = 0xced7230a


def _native():
    try:
        from ._lib import _native
        return _native
    except Exception:  # pragma: no cover
        return None


class _PyWriter:
    def __init__(self, path, append=False):
        self.f = open(path, 'ab' if append else 'wb')

    def write(self, buf):
        start = self.f.tell()
        n = len(buf)
        lower = (n >> 2) << 2
        upper = ((n + 3) >> 2) << 2
        dptr = 0
        for i in range(0, lower, 4):
            if struct.unpack_from('<I', buf, i)[0] == _MAGIC:
                self.f.write(struct.pack('<II', _MAGIC, ((1 if dptr == 0 else 2) << 29) | (i - dptr)))
                self.f.write(buf[dptr:i])
                dptr = i + 4
        self.f.write(struct.pack('<II', _MAGIC, ((3 if dptr else 0) << 29) | (n - dptr)))
        self.f.write(buf[dptr:])
        self.f.write(b'\x00' * (upper - n))
        return start

    def tell(self):
        return self.f.tell()

    def close(self):
        self.f.close()


class _PyReader:
    def __init__(self, path):
        self.f = open(path, 'rb')

    def read(self):
        out = b''
        while True:
            h = self.f.read(8)
            if not h:
                return None if not out else out
            magic, lrec = struct.unpack('<II', h)
            if magic != _MAGIC:
                raise MXNetError('Invalid RecordIO file')
            cflag, ln = lrec >> 29, lrec & ((1 << 29) - 1)
            data = self.f.read(((ln + 3) >> 2) << 2)[:ln]
            out += data
            if cflag in (0, 3):
                return out
            out += struct.pack('<I', _MAGIC)

    def seek(self, pos):
        self.f.seek(pos)

    def tell(self):
        return self.f.tell()

    def close(self):
        self.f.close()


class MXRecordIO:
    """Sequential RecordIO reader/writer (flag 'r' or 'w')."""

    def __init__(self, uri, flag):
        self.uri = uri
        self.flag = flag
        self.handle = None
        self.is_open = False
        self.open()

    def open(self):
        nat = _native()
        if self.flag == 'w':
            self.handle = nat.RecordWriter(self.uri, False) if nat else _PyWriter(self.uri)
            self.writable = True
        elif self.flag == 'r':
            if not os.path.exists(self.uri):
                raise MXNetError('cannot open %s' % self.uri)
            self.handle = nat.RecordReader(self.uri) if nat else _PyReader(self.uri)
            self.writable = False
        else:
            raise ValueError('Invalid flag %s' % self.flag)
        self.pid = os.getpid()
        self.is_open = True

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __getstate__(self):
        is_open = self.is_open
        self.close()
        d = dict(self.__dict__)
        d['is_open'] = is_open
        d['handle'] = None
        if is_open:
            self.open()
        return d

    def __setstate__(self, d):
        self.__dict__ = d
        is_open = d['is_open']
        self.is_open = False
        self.handle = None
        if is_open:
            self.open()

    def _check_pid(self, allow_reset=False):
        if self.pid != os.getpid():
            if allow_reset:
                self.reset()
            else:
                raise RuntimeError('Forbidden operation in multiple processes')

    def close(self):
        if not self.is_open:
            return
        self.handle.close()
        self.is_open = False
        self.pid = None

    def reset(self):
        self.close()
        self.open()

    def write(self, buf):
        assert self.writable
        self._check_pid(allow_reset=False)
        if isinstance(buf, str):
            buf = buf.encode()
        return self.handle.write(bytes(buf))

    def read(self):
        assert not self.writable
        self._check_pid(allow_reset=True)
        return self.handle.read()

    def tell(self):
        return self.handle.tell()


class MXIndexedRecordIO(MXRecordIO):
    """RecordIO with a ``key\\toffset`` index file for random access."""

    def __init__(self, idx_path, uri, flag, key_type=int):
        self.idx_path = idx_path
        self.idx = {}
        self.keys = []
        self.key_type = key_type
        self.fidx = None
        super().__init__(uri, flag)

    def open(self):
        super().open()
        self.idx = {}
        self.keys = []
        self.fidx = open(self.idx_path, self.flag)
        if not self.writable:
            for line in iter(self.fidx.readline, ''):
                line = line.strip().split('\t')
                key = self.key_type(line[0])
                self.idx[key] = int(line[1])
                self.keys.append(key)

    def close(self):
        if not self.is_open:
            return
        super().close()
        if self.fidx is not None:
            self.fidx.close()
            self.fidx = None

    def __getstate__(self):
        d = super().__getstate__()
        d['fidx'] = None
        return d

    def seek(self, idx):
        assert not self.writable
        self._check_pid(allow_reset=True)
        self.handle.seek(self.idx[idx])

    def tell(self):
        assert self.writable
        return self.handle.tell()

    def read_idx(self, idx):
        self.seek(idx)
        return self.read()

    def write_idx(self, idx, buf):
        key = self.key_type(idx)
        pos = self.write(buf)
        self.fidx.write('%s\t%d\n' % (str(key), pos))
        self.idx[key] = pos
        self.keys.append(key)


IRHeader = namedtuple('HEADER', ['flag', 'label', 'id', 'id2'])
_IR_FORMAT = 'IfQQ'
_IR_SIZE = struct.calcsize(_IR_FORMAT)


def pack(header, s):
    """Pack an IRHeader + payload bytes into one record."""
    header = IRHeader(*header)
    if isinstance(header.label, numbers.Number):
        header = header._replace(flag=0)
    else:
        label = np.asarray(header.label, dtype=np.float32)
        header = header._replace(flag=label.size, label=0)
        s = label.tobytes() + s
    return struct.pack(_IR_FORMAT, *header) + s


def unpack(s):
    header = IRHeader(*struct.unpack(_IR_FORMAT, s[:_IR_SIZE]))
    s = s[_IR_SIZE:]
    if header.flag > 0:
        header = header._replace(label=np.frombuffer(s, np.float32, header.flag))
        s = s[header.flag * 4:]
    return header, s


def unpack_img(s, iscolor=-1):
    """Unpack a record into (header, HxWxC uint8 numpy image) using PIL."""
    header, s = unpack(s)
    from .image import imdecode_np
    img = imdecode_np(s, iscolor)
    return header, img


def pack_img(header, img, quality=95, img_fmt='.jpg'):
    """Pack an image (numpy HxWxC uint8, RGB) into a record (JPEG/PNG via PIL)."""
    import io
    from PIL import Image
    buf = io.BytesIO()
    arr = np.asarray(img)
    if arr.ndim == 3 and arr.shape[2] == 1:
        arr = arr[:, :, 0]
    im = Image.fromarray(arr.astype(np.uint8))
    fmt = 'JPEG' if img_fmt.lower() in ('.jpg', '.jpeg') else 'PNG'
    if fmt == 'JPEG':
        im.save(buf, format=fmt, quality=quality)
    else:
        im.save(buf, format=fmt)
    return pack(header, buf.getvalue())
