"""Operator registry.

Parity: nnvm op registry (3rdparty/tvm/nnvm, NNVM_REGISTER_OP in
src/operator/**). Every operator is registered once here with

* ``fn``           -- a function over torch tensors (HIP kernels on gfx950 for
                      the hot ops, torch for the long tail),
* ``arg_names``    -- names of tensor inputs (list or ``f(attrs) -> list``);
                      used to auto-create Symbol variables (``fc1_weight``),
* ``aux_names``    -- auxiliary states mutated in place (BatchNorm moving stats),
* ``params``       -- attribute spec ``name -> (kind, default)``; string values
                      coming from JSON are parsed according to ``kind``,
* ``num_outputs``  -- int or ``f(attrs) -> int``,
* ``infer_params`` -- optional ``f(in_shapes, attrs) -> {arg_index: shape}``
                      for deferred parameter shape inference.

The same OpDef serves the imperative ``mx.nd.*`` path, the symbolic ``mx.sym.*``
path and the hybridized cached-graph executor.
"""
import ast

from ..base import MXNetError

_OPS = {}


_ACCEPTS = {}


def _fn_accepts(fn, key):
    """Whether ``fn`` takes keyword ``key`` (True for functions with ``**kwargs``)."""
    acc = _ACCEPTS.get(fn)
    if acc is None:
        import inspect
        try:
            ps = inspect.signature(fn).parameters.values()
            acc = True if any(p.kind == p.VAR_KEYWORD for p in ps) else frozenset(p.name for p in ps)
        except (TypeError, ValueError):
            acc = True
        _ACCEPTS[fn] = acc
    return acc is True or key in acc


class OpDef:
    __slots__ = ('name', 'fn', 'arg_names', 'aux_names', 'params', 'num_outputs',
                 'infer_params', 'key_var_num_args', 'doc', 'num_visible_outputs',
                 'output_names', 'extra_params')

    def __init__(self, name, fn, arg_names=('data',), aux_names=(), params=None,
                 num_outputs=1, infer_params=None, key_var_num_args=None, doc=None,
                 num_visible_outputs=None, output_names=None, extra_params=False):
        self.name = name
        self.fn = fn
        self.arg_names = arg_names
        self.aux_names = aux_names
        self.params = params or {}
        self.num_outputs = num_outputs
        self.infer_params = infer_params
        self.key_var_num_args = key_var_num_args
        self.doc = doc
        self.num_visible_outputs = num_visible_outputs
        self.output_names = output_names
        self.extra_params = extra_params   # keep undeclared attributes (Custom op kwargs)

    def get_arg_names(self, attrs):
        a = self.arg_names
        return list(a(attrs)) if callable(a) else list(a)

    def get_aux_names(self, attrs):
        a = self.aux_names
        return list(a(attrs)) if callable(a) else list(a)

    def get_num_outputs(self, attrs):
        n = self.num_outputs
        return n(attrs) if callable(n) else n

    def get_num_visible_outputs(self, attrs):
        n = self.num_visible_outputs
        if n is None:
            return self.get_num_outputs(attrs)
        return n(attrs) if callable(n) else n

    def parse_attrs(self, attrs):
        """Parse/normalise user or JSON attributes into python values."""
        out = {}
        spec = self.params
        for k, v in attrs.items():
            if v is None:
                s = spec.get(k)
                if s is not None and isinstance(s[0], str) and s[0].endswith('?'):
                    out[k] = None       # an optional parameter explicitly set to None
                continue
            if k.startswith('__') and k.endswith('__') and k not in spec:
                continue
            s = spec.get(k)
            if s is None:
                if not self.extra_params and not _fn_accepts(self.fn, k):
                    continue        # an attribute the operator does not take is ignored (as by nnvm)
                out[k] = _auto_parse(v) if isinstance(v, str) else v
            else:
                out[k] = parse_value(s[0], v)
        for k, s in spec.items():
            if k not in out:
                out[k] = s[1]
        return out

    def __repr__(self):
        return 'OpDef(%s)' % self.name


def register(name, fn=None, aliases=(), **kwargs):
    """Register an operator; usable as a decorator."""
    def _do(f):
        op = OpDef(name, f, **kwargs)
        _OPS[name] = op
        for a in aliases:
            _OPS[a] = op
        return f
    if fn is not None:
        return _do(fn)
    return _do


def alias(name, *aliases):
    for a in aliases:
        _OPS[a] = _OPS[name]


def get(name):
    try:
        return _OPS[name]
    except KeyError:
        raise MXNetError('Operator %s is not registered' % name)


def has(name):
    return name in _OPS


def list_ops():
    return sorted(_OPS.keys())


# ---------------------------------------------------------------------------
# attribute parsing / formatting (MXNet stores every attribute as a string)
# ---------------------------------------------------------------------------

def _auto_parse(v):
    s = v.strip()
    if s in ('True', 'true'):
        return True
    if s in ('False', 'false'):
        return False
    if s == 'None':
        return None
    try:
        return ast.literal_eval(s)
    except Exception:
        return v


def _to_tuple(v):
    if v is None:
        return None
    if isinstance(v, str):
        v = v.strip()
        if v in ('None', ''):
            return None
        v = ast.literal_eval(v.replace('L', '')) if v not in ('()', '[]') else ()
    if isinstance(v, (int, float)):
        return (int(v),)
    return tuple(None if x is None else int(x) for x in v)


def _to_float_tuple(v):
    if isinstance(v, str):
        v = ast.literal_eval(v)
    if isinstance(v, (int, float)):
        return (float(v),)
    return tuple(float(x) for x in v)


def _to_bool(v):
    if isinstance(v, str):
        return v.strip() in ('True', 'true', '1')
    return bool(v)


def _to_opt(conv):
    def f(v):
        if v is None or (isinstance(v, str) and v.strip() in ('None', '')):
            return None
        return conv(v)
    return f


def _to_int(v):
    if isinstance(v, str):
        v = v.strip()
        return int(float(v)) if '.' in v or 'e' in v else int(v)
    return int(v)


def _to_float(v):
    if isinstance(v, str):
        v = v.strip()
        if v in ('inf', 'Infinity'):
            return float('inf')
        if v in ('-inf', '-Infinity'):
            return float('-inf')
    return float(v)


def _to_str(v):
    if isinstance(v, str):
        return v
    if isinstance(v, type) or type(v).__name__ in ('dtype', '_BF16Marker'):
        from ..base import dtype_name
        try:
            return dtype_name(v)
        except Exception:
            return getattr(v, '__name__', str(v))
    return str(v)


def _to_axis(v):
    """axis attribute: int, tuple of ints or None."""
    if v is None:
        return None
    if isinstance(v, str):
        v = v.strip()
        if v in ('None', '', '()'):
            return None if v != '()' else ()
        v = ast.literal_eval(v)
    if isinstance(v, (list, tuple)):
        return tuple(int(x) for x in v)
    return int(v)


def _to_dtype(v):
    if v is None:
        return None
    if isinstance(v, str) and v.strip() == 'None':
        return None
    return v


_PARSERS = {
    'int': _to_int, 'float': _to_float, 'bool': _to_bool, 'str': _to_str,
    'shape': _to_tuple, 'floats': _to_float_tuple, 'axis': _to_axis,
    'int?': _to_opt(_to_int), 'float?': _to_opt(_to_float), 'shape?': _to_opt(_to_tuple),
    'str?': _to_opt(_to_str), 'bool?': _to_opt(_to_bool), 'dtype': _to_dtype,
    'any': lambda v: _auto_parse(v) if isinstance(v, str) else v,
}


def parse_value(kind, v):
    return _PARSERS[kind](v)


def format_value(v):
    """Format a python attribute value the way MXNet writes it into JSON."""
    if isinstance(v, bool):
        return 'True' if v else 'False'
    if v is None:
        return 'None'
    if isinstance(v, (tuple, list)):
        return '(' + ', '.join(format_value(x) for x in v) + (',)' if len(v) == 1 else ')')
    if isinstance(v, float):
        r = repr(v)
        return r
    if hasattr(v, '__name__') and not isinstance(v, str):
        return v.__name__
    return str(v)
