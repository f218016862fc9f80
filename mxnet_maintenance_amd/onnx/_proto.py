"""ONNX protobuf messages without the ``onnx`` package.

The ``onnx`` wheel is not part of this environment, so the subset of ``onnx.proto`` (IR version 8)
the exporter / importer use is declared here as a protobuf descriptor and turned into message
classes by ``google.protobuf`` itself.  Field numbers and enum values follow onnx.proto, so the bytes
written are ordinary ``.onnx`` files (and real ONNX files parse with these classes).  Parity with the
reference's onnx-based converters is unpinned here: neither onnx nor onnxruntime is importable, so
the tests check round trips through this framework's own exporter and importer.
"""
import numpy as np

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_F = descriptor_pb2.FieldDescriptorProto
_OPT, _REP = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED
_T = {'int64': _F.TYPE_INT64, 'int32': _F.TYPE_INT32, 'string': _F.TYPE_STRING, 'bytes': _F.TYPE_BYTES,
      'float': _F.TYPE_FLOAT, 'double': _F.TYPE_DOUBLE, 'uint64': _F.TYPE_UINT64, 'enum': _F.TYPE_ENUM,
      'msg': _F.TYPE_MESSAGE}

# message -> [(field, number, label, type, type_name or None, packed)]
_SCHEMA = {
    'StringStringEntryProto': [('key', 1, _OPT, 'string'), ('value', 2, _OPT, 'string')],
    'OperatorSetIdProto': [('domain', 1, _OPT, 'string'), ('version', 2, _OPT, 'int64')],
    'TensorShapeProto.Dimension': [('dim_value', 1, _OPT, 'int64'), ('dim_param', 2, _OPT, 'string'),
                                   ('denotation', 3, _OPT, 'string')],
    'TensorShapeProto': [('dim', 1, _REP, 'msg', '.onnx.TensorShapeProto.Dimension')],
    'TypeProto.Tensor': [('elem_type', 1, _OPT, 'int32'), ('shape', 2, _OPT, 'msg', '.onnx.TensorShapeProto')],
    'TypeProto': [('tensor_type', 1, _OPT, 'msg', '.onnx.TypeProto.Tensor'), ('denotation', 6, _OPT, 'string')],
    'ValueInfoProto': [('name', 1, _OPT, 'string'), ('type', 2, _OPT, 'msg', '.onnx.TypeProto'),
                       ('doc_string', 3, _OPT, 'string')],
    'TensorProto': [('dims', 1, _REP, 'int64'), ('data_type', 2, _OPT, 'int32'),
                    ('float_data', 4, _REP, 'float', None, True), ('int32_data', 5, _REP, 'int32', None, True),
                    ('string_data', 6, _REP, 'bytes'), ('int64_data', 7, _REP, 'int64', None, True),
                    ('name', 8, _OPT, 'string'), ('raw_data', 9, _OPT, 'bytes'),
                    ('double_data', 10, _REP, 'double', None, True), ('uint64_data', 11, _REP, 'uint64', None, True),
                    ('doc_string', 12, _OPT, 'string')],
    'AttributeProto': [('name', 1, _OPT, 'string'), ('f', 2, _OPT, 'float'), ('i', 3, _OPT, 'int64'),
                       ('s', 4, _OPT, 'bytes'), ('t', 5, _OPT, 'msg', '.onnx.TensorProto'),
                       ('g', 6, _OPT, 'msg', '.onnx.GraphProto'), ('floats', 7, _REP, 'float'),
                       ('ints', 8, _REP, 'int64'), ('strings', 9, _REP, 'bytes'),
                       ('tensors', 10, _REP, 'msg', '.onnx.TensorProto'), ('graphs', 11, _REP, 'msg', '.onnx.GraphProto'),
                       ('doc_string', 13, _OPT, 'string'), ('type', 20, _OPT, 'int32'),
                       ('ref_attr_name', 21, _OPT, 'string')],
    'NodeProto': [('input', 1, _REP, 'string'), ('output', 2, _REP, 'string'), ('name', 3, _OPT, 'string'),
                  ('op_type', 4, _OPT, 'string'), ('attribute', 5, _REP, 'msg', '.onnx.AttributeProto'),
                  ('doc_string', 6, _OPT, 'string'), ('domain', 7, _OPT, 'string')],
    'GraphProto': [('node', 1, _REP, 'msg', '.onnx.NodeProto'), ('name', 2, _OPT, 'string'),
                   ('initializer', 5, _REP, 'msg', '.onnx.TensorProto'), ('doc_string', 10, _OPT, 'string'),
                   ('input', 11, _REP, 'msg', '.onnx.ValueInfoProto'), ('output', 12, _REP, 'msg', '.onnx.ValueInfoProto'),
                   ('value_info', 13, _REP, 'msg', '.onnx.ValueInfoProto')],
    'ModelProto': [('ir_version', 1, _OPT, 'int64'), ('producer_name', 2, _OPT, 'string'),
                   ('producer_version', 3, _OPT, 'string'), ('domain', 4, _OPT, 'string'),
                   ('model_version', 5, _OPT, 'int64'), ('doc_string', 6, _OPT, 'string'),
                   ('graph', 7, _OPT, 'msg', '.onnx.GraphProto'),
                   ('opset_import', 8, _REP, 'msg', '.onnx.OperatorSetIdProto'),
                   ('metadata_props', 14, _REP, 'msg', '.onnx.StringStringEntryProto')],
}

# AttributeProto.AttributeType
A_FLOAT, A_INT, A_STRING, A_TENSOR, A_GRAPH, A_FLOATS, A_INTS, A_STRINGS = 1, 2, 3, 4, 5, 6, 7, 8

# TensorProto.DataType <-> numpy
_DT2NP = {1: np.float32, 2: np.uint8, 3: np.int8, 4: np.uint16, 5: np.int16, 6: np.int32, 7: np.int64,
          9: np.bool_, 10: np.float16, 11: np.float64, 12: np.uint32, 13: np.uint64}
_NP2DT = {np.dtype(v): k for k, v in _DT2NP.items()}
BFLOAT16 = 16

IR_VERSION = 8
OPSET = 13


def _build():
    fd = descriptor_pb2.FileDescriptorProto(name='mxamd_onnx_subset.proto', package='onnx', syntax='proto2')
    msgs = {}
    for full in _SCHEMA:
        parts = full.split('.')
        if len(parts) == 1:
            msgs[full] = fd.message_type.add(name=full)
    for full in _SCHEMA:
        parts = full.split('.')
        if len(parts) == 2:
            msgs[full] = msgs[parts[0]].nested_type.add(name=parts[1])
    for full, fields in _SCHEMA.items():
        m = msgs[full]
        for spec in fields:
            name, num, label, typ = spec[:4]
            f = m.field.add(name=name, number=num, label=label, type=_T[typ])
            if typ == 'msg':
                f.type_name = spec[4]
            if len(spec) > 5 and spec[5]:
                f.options.packed = True
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    classes = message_factory.GetMessageClassesForFiles([fd.name], pool)
    return {k.split('.', 1)[1]: v for k, v in classes.items()}


_CLASSES = _build()
ModelProto = _CLASSES['ModelProto']
GraphProto = _CLASSES['GraphProto']
NodeProto = _CLASSES['NodeProto']
TensorProto = _CLASSES['TensorProto']
AttributeProto = _CLASSES['AttributeProto']
ValueInfoProto = _CLASSES['ValueInfoProto']


def dtype_to_onnx(dt):
    dt = np.dtype(dt)
    if dt not in _NP2DT:
        raise TypeError('ONNX: unsupported element type %s' % dt)
    return _NP2DT[dt]


def onnx_to_dtype(code):
    if code not in _DT2NP:
        raise TypeError('ONNX: unsupported TensorProto data type %d' % code)
    return np.dtype(_DT2NP[code])


def make_tensor(name, arr):
    """TensorProto holding ``arr`` (little-endian raw_data)."""
    arr = np.ascontiguousarray(arr)
    t = TensorProto(name=name, data_type=dtype_to_onnx(arr.dtype))
    t.dims.extend(int(d) for d in arr.shape)
    t.raw_data = arr.astype(arr.dtype.newbyteorder('<'), copy=False).tobytes()
    return t


def tensor_to_array(t):
    dt = onnx_to_dtype(t.data_type)
    shape = tuple(int(d) for d in t.dims)
    if t.raw_data:
        a = np.frombuffer(t.raw_data, dtype=dt.newbyteorder('<')).astype(dt)
    elif t.data_type in (1,):
        a = np.asarray(t.float_data, dtype=dt)
    elif t.data_type == 11:
        a = np.asarray(t.double_data, dtype=dt)
    elif t.data_type in (7,):
        a = np.asarray(t.int64_data, dtype=dt)
    elif t.data_type in (12, 13):
        a = np.asarray(t.uint64_data, dtype=dt)
    elif t.data_type == 10:
        a = np.asarray(t.int32_data, dtype=np.uint16).view(np.float16)
    else:
        a = np.asarray(t.int32_data, dtype=dt)
    return a.reshape(shape)


def make_attribute(name, value):
    a = AttributeProto(name=name)
    if isinstance(value, bool):
        a.type, a.i = A_INT, int(value)
    elif isinstance(value, (int, np.integer)):
        a.type, a.i = A_INT, int(value)
    elif isinstance(value, (float, np.floating)):
        a.type, a.f = A_FLOAT, float(value)
    elif isinstance(value, (str, bytes)):
        a.type, a.s = A_STRING, value.encode() if isinstance(value, str) else value
    elif isinstance(value, np.ndarray):
        a.type = A_TENSOR
        a.t.CopyFrom(make_tensor(name, value))
    elif isinstance(value, (list, tuple)):
        if all(isinstance(v, (int, np.integer)) and not isinstance(v, bool) for v in value):
            a.type = A_INTS
            a.ints.extend(int(v) for v in value)
        elif all(isinstance(v, (int, float, np.number)) for v in value):
            a.type = A_FLOATS
            a.floats.extend(float(v) for v in value)
        else:
            a.type = A_STRINGS
            a.strings.extend(v.encode() if isinstance(v, str) else v for v in value)
    else:
        raise TypeError('ONNX attribute %s: unsupported value %r' % (name, value))
    return a


def attribute_value(a):
    if a.type == A_FLOAT:
        return a.f
    if a.type == A_INT:
        return a.i
    if a.type == A_STRING:
        return a.s.decode()
    if a.type == A_TENSOR:
        return tensor_to_array(a.t)
    if a.type == A_FLOATS:
        return list(a.floats)
    if a.type == A_INTS:
        return list(a.ints)
    if a.type == A_STRINGS:
        return [s.decode() for s in a.strings]
    raise TypeError('ONNX attribute %s: unsupported type %d' % (a.name, a.type))


def make_node(op_type, inputs, outputs, name=None, **attrs):
    n = NodeProto(op_type=op_type, name=name or outputs[0])
    n.input.extend(inputs)
    n.output.extend(outputs)
    for k, v in sorted(attrs.items()):
        if v is not None:
            n.attribute.append(make_attribute(k, v))
    return n


def make_value_info(name, dtype_code, shape):
    v = ValueInfoProto(name=name)
    tt = v.type.tensor_type
    tt.elem_type = dtype_code
    for d in shape:
        dim = tt.shape.dim.add()
        if d is None or (isinstance(d, int) and d < 0):
            dim.dim_param = 'N'
        else:
            dim.dim_value = int(d)
    return v


def load_model(path_or_bytes):
    """ModelProto from a file path, bytes or file object."""
    if isinstance(path_or_bytes, (bytes, bytearray)):
        data = bytes(path_or_bytes)
    elif hasattr(path_or_bytes, 'read'):
        data = path_or_bytes.read()
    else:
        with open(path_or_bytes, 'rb') as f:
            data = f.read()
    m = ModelProto()
    m.ParseFromString(data)
    return m
