"""Python side of the C predict API (``libmxamd_predict.so``, src/capi/c_predict_api.cc).

Parity: include/mxnet/c_predict_api.h + src/c_api/c_predict_api.cc of the reference -- a minimal
inference interface for applications that link a C library: create a predictor from a symbol JSON
string and the raw bytes of a ``.params`` file, set inputs from float buffers, run forward, read
outputs back; plus ``MXNDList*`` to read any saved NDArray file (e.g. a mean image).

The C library embeds (or joins) the Python interpreter and calls the functions below; the graph
executes through the same executor as ``Symbol.simple_bind`` (HIP kernels on a GPU context).
"""
import numpy as np

from . import ndarray as nd
from . import symbol as sym_mod
from .context import cpu, gpu

# reference dtype codes (mshadow): 0 float32, 1 float64, 2 float16, 3 uint8, 4 int32, 5 int8, 6 int64
_DTYPES = {0: 'float32', 1: 'float64', 2: 'float16', 3: 'uint8', 4: 'int32', 5: 'int8', 6: 'int64'}
_CODES = {np.dtype(v): k for k, v in _DTYPES.items()}


def _split_params(raw):
    """``arg:`` / ``aux:`` prefixed arrays of a params file -> (args, auxs); unprefixed go to args."""
    args, auxs = {}, {}
    for key, arr in raw.items():
        if key.startswith('aux:'):
            auxs[key[4:]] = arr
        else:
            args[key[4:] if key.startswith('arg:') else key] = arr
    return args, auxs


class Predictor:
    """One bound inference executor with host-visible inputs / outputs."""

    def __init__(self, symbol_json, param_bytes, dev_type, dev_id, input_shapes, dtypes=None, output_keys=None):
        self._symbol_json = symbol_json
        self._ctx = cpu(dev_id) if dev_type == 1 else gpu(dev_id)
        net = sym_mod.load_json(symbol_json)
        if output_keys:
            internals = net.get_internals()
            names = internals.list_outputs()
            picked = []
            for key in output_keys:
                name = key if key in names else key + '_output'
                if name not in names:
                    raise ValueError('MXPredCreatePartialOut: no output named %s' % key)
                picked.append(internals[names.index(name)])
            net = sym_mod.Group(picked)
        self._net = net
        raw = nd.load_frombuffer(param_bytes) if param_bytes else {}
        self._args, self._auxs = _split_params(raw if isinstance(raw, dict) else {})
        self._dtypes = dict(dtypes or {})
        self._bind(dict(input_shapes))

    def _bind(self, input_shapes):
        self._input_shapes = {k: tuple(int(d) for d in v) for k, v in input_shapes.items()}
        type_dict = {k: _DTYPES[v] for k, v in self._dtypes.items()}
        for name, arr in self._args.items():
            type_dict.setdefault(name, np.dtype(arr.dtype).name)
        self._exe = self._net.simple_bind(self._ctx, grad_req='null', type_dict=type_dict, **self._input_shapes)
        for name, arr in self._exe.arg_dict.items():
            if name in self._args and name not in self._input_shapes:
                arr[:] = self._args[name].as_in_context(arr.context).astype(arr.dtype)
        for name, arr in self._exe.aux_dict.items():
            if name in self._auxs:
                arr[:] = self._auxs[name].as_in_context(arr.context).astype(arr.dtype)
        self._outputs = None

    # ------------------------------------------------------------------ C entry points
    def reshape(self, input_shapes):
        """A new predictor sharing the weights, bound for other input shapes (MXPredReshape)."""
        twin = Predictor.__new__(Predictor)
        twin.__dict__.update({k: v for k, v in self.__dict__.items() if k not in ('_exe', '_outputs')})
        twin._bind(dict(input_shapes))
        return twin

    def set_input(self, key, buf):
        arr = self._exe.arg_dict.get(key)
        if arr is None or key not in self._input_shapes:
            raise ValueError('MXPredSetInput: %s is not an input of the predictor' % key)
        host = np.frombuffer(buf, dtype=np.float32)
        if host.size != int(np.prod(arr.shape)):
            raise ValueError('MXPredSetInput: %s expects %d values, got %d' % (key, int(np.prod(arr.shape)),
                                                                              host.size))
        arr[:] = nd.array(host.reshape(arr.shape), ctx=arr.context).astype(arr.dtype)

    def forward(self):
        self._exe.forward(is_train=False)
        self._outputs = [o.asnumpy() for o in self._exe.outputs]

    def num_outputs(self):
        return len(self._net.list_outputs())

    def _out(self, index):
        if self._outputs is None:
            raise ValueError('MXPredGetOutput: call MXPredForward first')
        if not 0 <= index < len(self._outputs):
            raise ValueError('MXPredGetOutput: output index %d out of range' % index)
        return self._outputs[index]

    def output_shape(self, index):
        if self._outputs is not None:
            return list(self._out(index).shape)
        return list(self._exe.outputs[index].shape)

    def output_dtype(self, index):
        return _CODES.get(np.dtype(self._exe.outputs[index].dtype), 0)

    def output_bytes(self, index):
        """Output ``index`` as float32 bytes (the C API's ``mx_float`` buffer)."""
        return np.ascontiguousarray(self._out(index), dtype=np.float32).tobytes()


def create(symbol_json, param_bytes, dev_type, dev_id, keys, shapes, dtype_names=(), dtype_codes=(),
           output_keys=()):
    """MXPredCreate / MXPredCreateEx / MXPredCreatePartialOut."""
    return Predictor(symbol_json, param_bytes, dev_type, dev_id, dict(zip(keys, shapes)),
                     dict(zip(dtype_names, dtype_codes)), list(output_keys))


def nd_list(file_bytes):
    """MXNDListCreate: [(key, float32 bytes, shape)] of a saved NDArray file."""
    raw = nd.load_frombuffer(file_bytes)
    items = raw.items() if isinstance(raw, dict) else [('', a) for a in raw]
    return [(key, np.ascontiguousarray(arr.asnumpy(), dtype=np.float32).tobytes(), list(arr.shape))
            for key, arr in items]
