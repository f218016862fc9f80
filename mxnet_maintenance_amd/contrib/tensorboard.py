"""TensorBoard metric logging.

Parity: python/mxnet/contrib/tensorboard.py:24-72 (``LogMetricsCallback``).  The
reference delegates to the external ``mxboard`` package; none of mxboard,
tensorboard or tensorboardX exists in this image, so this module writes the
TensorBoard event-file format itself: TFRecord framing (length, masked CRC-32C
of the length, payload, masked CRC-32C of the payload) around hand-encoded
``Event`` protocol buffers carrying scalar ``Summary`` values.  The files load
in any TensorBoard.
"""
import os
import socket
import struct
import time

__all__ = ['LogMetricsCallback', 'SummaryWriter']


def _crc32c_table():
    poly = 0x82F63B78
    table = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ poly if c & 1 else c >> 1
        table.append(c)
    return table


_CRC_TABLE = _crc32c_table()


def crc32c(data):
    c = 0xFFFFFFFF
    for b in data:
        c = _CRC_TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _masked_crc(data):
    c = crc32c(data)
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


# ---- minimal protobuf encoding (wire types 0, 1, 2, 5)
def _varint(n):
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field, wire):
    return _varint((field << 3) | wire)


def _bytes_field(field, payload):
    return _key(field, 2) + _varint(len(payload)) + payload


def _event(wall_time, step, summary=None, file_version=None):
    """Serialized tensorflow.Event: wall_time=1 (double), step=2 (int64), file_version=3 (string),
    summary=5 (Summary)."""
    msg = _key(1, 1) + struct.pack('<d', wall_time) + _key(2, 0) + _varint(int(step))
    if file_version is not None:
        msg += _bytes_field(3, file_version.encode())
    if summary is not None:
        msg += _bytes_field(5, summary)
    return msg


def _scalar_summary(tag, value):
    """Serialized tensorflow.Summary with one Value{tag=1, simple_value=2 (float)}."""
    val = _bytes_field(1, tag.encode()) + _key(2, 5) + struct.pack('<f', float(value))
    return _bytes_field(1, val)


class SummaryWriter:
    """Append-only writer of one ``events.out.tfevents.*`` file with scalar summaries."""

    def __init__(self, logdir):
        os.makedirs(logdir, exist_ok=True)
        name = 'events.out.tfevents.%d.%s' % (int(time.time()), socket.gethostname())
        self.path = os.path.join(logdir, name)
        self._f = open(self.path, 'ab')
        self._write(_event(time.time(), 0, file_version='brain.Event:2'))

    def _write(self, payload):
        head = struct.pack('<Q', len(payload))
        self._f.write(head + struct.pack('<I', _masked_crc(head)) + payload + struct.pack('<I', _masked_crc(payload)))

    def add_scalar(self, tag, value, global_step=0):
        self._write(_event(time.time(), global_step, summary=_scalar_summary(tag, value)))
        self._f.flush()

    def close(self):
        self._f.close()


def read_scalars(path):
    """[(step, tag, value)] of an event file written by ``SummaryWriter`` (CRC-checked)."""
    out = []
    with open(path, 'rb') as f:
        data = f.read()
    pos = 0
    while pos < len(data):
        (n,) = struct.unpack_from('<Q', data, pos)
        if struct.unpack_from('<I', data, pos + 8)[0] != _masked_crc(data[pos:pos + 8]):
            raise ValueError('corrupt record length at %d' % pos)
        payload = data[pos + 12:pos + 12 + n]
        if struct.unpack_from('<I', data, pos + 12 + n)[0] != _masked_crc(payload):
            raise ValueError('corrupt record at %d' % pos)
        pos += 16 + n
        rec = _parse(payload)
        if 5 in rec:
            val = _parse(_parse(rec[5])[1])
            out.append((rec.get(2, 0), val[1].decode(), struct.unpack('<f', val[2])[0]))
    return out


def _parse(buf):
    """Top-level fields of a protobuf message: {field: value} (last occurrence wins)."""
    out, i = {}, 0
    while i < len(buf):
        k, i = _read_varint(buf, i)
        field, wire = k >> 3, k & 7
        if wire == 0:
            out[field], i = _read_varint(buf, i)
        elif wire == 1:
            out[field], i = buf[i:i + 8], i + 8
        elif wire == 5:
            out[field], i = buf[i:i + 4], i + 4
        elif wire == 2:
            n, i = _read_varint(buf, i)
            out[field], i = buf[i:i + n], i + n
        else:
            raise ValueError('unsupported wire type %d' % wire)
    return out


def _read_varint(buf, i):
    shift = n = 0
    while True:
        b = buf[i]
        i += 1
        n |= (b & 0x7F) << shift
        if not b & 0x80:
            return n, i
        shift += 7


class LogMetricsCallback:
    """``Module.fit`` batch/eval callback writing every metric of ``param.eval_metric`` as a
    TensorBoard scalar (step = epoch), optionally prefixed ``<prefix>-``."""

    def __init__(self, logging_dir, prefix=None):
        self.prefix = prefix
        self.summary_writer = SummaryWriter(logging_dir)

    def __call__(self, param):
        if param.eval_metric is None:
            return
        for name, value in param.eval_metric.get_name_value():
            if self.prefix is not None:
                name = '%s-%s' % (self.prefix, name)
            self.summary_writer.add_scalar(name, value, global_step=param.epoch)
