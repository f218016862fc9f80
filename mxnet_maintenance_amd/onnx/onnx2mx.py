"""ONNX model -> Symbol + parameters.

Behaviour of the reference importer (python/mxnet/contrib/onnx/onnx2mx/import_onnx.py
``GraphProto.from_onnx`` / ``get_graph_metadata`` / ``graph_to_gluon``, import_model.py:24,
_op_translations.py): initializers become parameters (BatchNorm running statistics as auxiliary
states), graph inputs that are not initializers become data variables, and each ONNX node is mapped
onto the equivalent registered operator.  Operands ONNX passes as constant tensors (Reshape's shape,
Unsqueeze's axes, Clip's bounds, Pad's pads, ...) are read from the initializers / Constant nodes.
"""
import numpy as np

from . import _proto as P


def _scalar(arr):
    return float(np.asarray(arr).reshape(-1)[0])


def _attrs(node):
    return {a.name: P.attribute_value(a) for a in node.attribute}


def _sym_pads(pads, nd, what):
    if not pads:
        return (0,) * nd
    b, e = tuple(pads[:nd]), tuple(pads[nd:])
    if b != e:
        raise NotImplementedError('ONNX import: asymmetric %s pads %s' % (what, pads))
    return b


class _Importer:
    def __init__(self, graph):
        from .. import symbol as S
        self.S = S
        self.graph = graph
        self.consts = {t.name: P.tensor_to_array(t) for t in graph.initializer}
        self.used_params = {}
        self.env = {}

    # operands --------------------------------------------------------------
    def const(self, name):
        if name not in self.consts:
            raise NotImplementedError('ONNX import: operand %s must be a constant' % name)
        return self.consts[name]

    def sym(self, name):
        s = self.env.get(name)
        if s is None:
            if name in self.consts:
                arr = self.consts[name]
                self.used_params[name] = arr
                s = self.env[name] = self.S.Variable(name, shape=arr.shape)
            else:
                raise KeyError('ONNX import: unknown tensor %s' % name)
        return s

    def param(self, name, arr):
        """A new parameter variable holding ``arr`` (e.g. a transposed or reshaped initializer)."""
        self.used_params[name] = arr
        return self.S.Variable(name, shape=arr.shape)

    # conversion ----------------------------------------------------------
    def run(self):
        S = self.S
        for vi in self.graph.input:
            if vi.name not in self.consts:
                self.env[vi.name] = S.Variable(vi.name)
        for node in self.graph.node:
            fn = getattr(self, '_op_' + node.op_type, None)
            if fn is None:
                raise NotImplementedError('ONNX import: operator %s is not supported' % node.op_type)
            res = fn(node, _attrs(node), list(node.input))
            if res is None:
                continue
            res = res if isinstance(res, (list, tuple)) else [res]
            for o, r in zip(node.output, res):
                if o:
                    self.env[o] = r
        outs = [self.env[o.name] for o in self.graph.output]
        return outs[0] if len(outs) == 1 else S.Group(outs)

    def _n(self, node):
        return node.name or node.output[0]

    def _op_Constant(self, node, a, ins):
        self.consts[node.output[0]] = np.asarray(a['value'])
        return None

    def _op_Identity(self, node, a, ins):
        return self.S.identity(self.sym(ins[0]), name=self._n(node))

    _op_Dropout = _op_Identity

    def _op_Conv(self, node, a, ins):
        w = self.const(ins[1]) if ins[1] in self.consts else None
        k = tuple(a.get('kernel_shape') or (w.shape[2:] if w is not None else ()))
        nd = len(k)
        return self.S.Convolution(self.sym(ins[0]), self.sym(ins[1]), *([self.sym(ins[2])] if len(ins) > 2 else []),
                                  kernel=k, stride=tuple(a.get('strides', (1,) * nd)),
                                  dilate=tuple(a.get('dilations', (1,) * nd)),
                                  pad=_sym_pads(a.get('pads'), nd, 'Conv'), num_group=a.get('group', 1),
                                  num_filter=int(w.shape[0]) if w is not None else int(a['num_filter']),
                                  no_bias=len(ins) < 3, name=self._n(node))

    def _op_ConvTranspose(self, node, a, ins):
        w = self.const(ins[1])
        k = tuple(a.get('kernel_shape') or w.shape[2:])
        nd = len(k)
        g = a.get('group', 1)
        return self.S.Deconvolution(self.sym(ins[0]), self.sym(ins[1]), *([self.sym(ins[2])] if len(ins) > 2 else []),
                                    kernel=k, stride=tuple(a.get('strides', (1,) * nd)),
                                    dilate=tuple(a.get('dilations', (1,) * nd)),
                                    pad=_sym_pads(a.get('pads'), nd, 'ConvTranspose'),
                                    adj=tuple(a.get('output_padding', (0,) * nd)), num_group=g,
                                    num_filter=int(w.shape[1]) * g, no_bias=len(ins) < 3, name=self._n(node))

    def _op_Gemm(self, node, a, ins):
        S = self.S
        alpha, beta = a.get('alpha', 1.0), a.get('beta', 1.0)
        ta, tb = a.get('transA', 0), a.get('transB', 0)
        if ins[1] in self.consts and alpha == 1.0 and beta == 1.0 and not ta:
            w = self.const(ins[1])
            if not tb:
                wsym = self.param(ins[1] + '_T', np.ascontiguousarray(w.T))
                nh = w.shape[1]
            else:
                wsym, nh = self.sym(ins[1]), w.shape[0]
            return S.FullyConnected(self.sym(ins[0]), wsym, *([self.sym(ins[2])] if len(ins) > 2 else []),
                                    num_hidden=int(nh), no_bias=len(ins) < 3, flatten=True, name=self._n(node))
        y = S.dot(self.sym(ins[0]), self.sym(ins[1]), transpose_a=bool(ta), transpose_b=bool(tb))
        if alpha != 1.0:
            y = y * alpha
        if len(ins) > 2:
            c = self.sym(ins[2])
            y = S.broadcast_add(y, c * beta if beta != 1.0 else c)
        return y

    def _op_MatMul(self, node, a, ins):
        S = self.S
        if ins[1] in self.consts and self.consts[ins[1]].ndim == 2:
            w = self.const(ins[1])
            return S.FullyConnected(self.sym(ins[0]), self.param(ins[1] + '_T', np.ascontiguousarray(w.T)),
                                    num_hidden=int(w.shape[1]), no_bias=True, flatten=False, name=self._n(node))
        return S.linalg.gemm2(self.sym(ins[0]), self.sym(ins[1]), name=self._n(node))

    def _op_BatchNormalization(self, node, a, ins):
        return self.S.BatchNorm(*[self.sym(i) for i in ins[:5]], eps=a.get('epsilon', 1e-5),
                                momentum=a.get('momentum', 0.9), fix_gamma=False, name=self._n(node))

    def _op_InstanceNormalization(self, node, a, ins):
        return self.S.InstanceNorm(*[self.sym(i) for i in ins[:3]], eps=a.get('epsilon', 1e-5), name=self._n(node))

    def _op_LayerNormalization(self, node, a, ins):
        return self.S.LayerNorm(*[self.sym(i) for i in ins[:3]], axis=a.get('axis', -1), eps=a.get('epsilon', 1e-5),
                                name=self._n(node))

    def _act(self, node, ins, t):
        return self.S.Activation(self.sym(ins[0]), act_type=t, name=self._n(node))

    def _op_Relu(self, node, a, ins):
        return self._act(node, ins, 'relu')

    def _op_Sigmoid(self, node, a, ins):
        return self._act(node, ins, 'sigmoid')

    def _op_Tanh(self, node, a, ins):
        return self._act(node, ins, 'tanh')

    def _op_Softplus(self, node, a, ins):
        return self._act(node, ins, 'softrelu')

    def _op_Softsign(self, node, a, ins):
        return self._act(node, ins, 'softsign')

    def _op_LeakyRelu(self, node, a, ins):
        return self.S.LeakyReLU(self.sym(ins[0]), act_type='leaky', slope=a.get('alpha', 0.01), name=self._n(node))

    def _op_Elu(self, node, a, ins):
        return self.S.LeakyReLU(self.sym(ins[0]), act_type='elu', slope=a.get('alpha', 1.0), name=self._n(node))

    def _op_Selu(self, node, a, ins):
        return self.S.LeakyReLU(self.sym(ins[0]), act_type='selu', name=self._n(node))

    def _op_PRelu(self, node, a, ins):
        g = self.const(ins[1]).reshape(-1)
        return self.S.LeakyReLU(self.sym(ins[0]), self.param(ins[1] + '_flat', g), act_type='prelu',
                                name=self._n(node))

    def _pool(self, node, a, ins, ptype):
        k = tuple(a['kernel_shape'])
        nd = len(k)
        kw = dict(kernel=k, pool_type=ptype, stride=tuple(a.get('strides', (1,) * nd)),
                  pad=_sym_pads(a.get('pads'), nd, 'pool'),
                  pooling_convention='full' if a.get('ceil_mode', 0) else 'valid')
        if ptype == 'avg':
            kw['count_include_pad'] = bool(a.get('count_include_pad', 0))
        return self.S.Pooling(self.sym(ins[0]), name=self._n(node), **kw)

    def _op_MaxPool(self, node, a, ins):
        return self._pool(node, a, ins, 'max')

    def _op_AveragePool(self, node, a, ins):
        return self._pool(node, a, ins, 'avg')

    def _op_GlobalAveragePool(self, node, a, ins):
        return self.S.Pooling(self.sym(ins[0]), kernel=(1, 1), global_pool=True, pool_type='avg', name=self._n(node))

    def _op_GlobalMaxPool(self, node, a, ins):
        return self.S.Pooling(self.sym(ins[0]), kernel=(1, 1), global_pool=True, pool_type='max', name=self._n(node))

    def _bin(self, node, ins, op):
        return getattr(self.S, op)(self.sym(ins[0]), self.sym(ins[1]), name=self._n(node))

    def _op_Add(self, node, a, ins):
        return self._bin(node, ins, 'broadcast_add')

    def _op_Sub(self, node, a, ins):
        return self._bin(node, ins, 'broadcast_sub')

    def _op_Mul(self, node, a, ins):
        return self._bin(node, ins, 'broadcast_mul')

    def _op_Div(self, node, a, ins):
        return self._bin(node, ins, 'broadcast_div')

    def _op_Pow(self, node, a, ins):
        return self._bin(node, ins, 'broadcast_power')

    def _op_Max(self, node, a, ins):
        return self._bin(node, ins, 'broadcast_maximum')

    def _op_Min(self, node, a, ins):
        return self._bin(node, ins, 'broadcast_minimum')

    def _op_Equal(self, node, a, ins):
        return self._bin(node, ins, 'broadcast_equal')

    def _op_Greater(self, node, a, ins):
        return self._bin(node, ins, 'broadcast_greater')

    def _op_Less(self, node, a, ins):
        return self._bin(node, ins, 'broadcast_lesser')

    def _op_Sum(self, node, a, ins):
        return self.S.add_n(*[self.sym(i) for i in ins], name=self._n(node))

    def _unary(self, node, ins, op):
        return getattr(self.S, op)(self.sym(ins[0]), name=self._n(node))

    def _op_Exp(self, node, a, ins):
        return self._unary(node, ins, 'exp')

    def _op_Log(self, node, a, ins):
        return self._unary(node, ins, 'log')

    def _op_Sqrt(self, node, a, ins):
        return self._unary(node, ins, 'sqrt')

    def _op_Abs(self, node, a, ins):
        return self._unary(node, ins, 'abs')

    def _op_Neg(self, node, a, ins):
        return self._unary(node, ins, 'negative')

    def _op_Reciprocal(self, node, a, ins):
        return self._unary(node, ins, 'reciprocal')

    def _op_Floor(self, node, a, ins):
        return self._unary(node, ins, 'floor')

    def _op_Ceil(self, node, a, ins):
        return self._unary(node, ins, 'ceil')

    def _op_Erf(self, node, a, ins):
        return self._unary(node, ins, 'erf')

    def _op_Sin(self, node, a, ins):
        return self._unary(node, ins, 'sin')

    def _op_Cos(self, node, a, ins):
        return self._unary(node, ins, 'cos')

    def _op_Sign(self, node, a, ins):
        return self._unary(node, ins, 'sign')

    def _op_Softmax(self, node, a, ins):
        return self.S.softmax(self.sym(ins[0]), axis=a.get('axis', -1), name=self._n(node))

    def _op_LogSoftmax(self, node, a, ins):
        return self.S.log_softmax(self.sym(ins[0]), axis=a.get('axis', -1), name=self._n(node))

    def _op_Flatten(self, node, a, ins):
        axis = a.get('axis', 1)
        if axis == 1:
            return self.S.Flatten(self.sym(ins[0]), name=self._n(node))
        return self.S.reshape(self.sym(ins[0]), shape=(0,) * axis + (-1,), name=self._n(node))

    def _op_Reshape(self, node, a, ins):
        shape = tuple(int(s) for s in self.const(ins[1]))
        return self.S.reshape(self.sym(ins[0]), shape=shape, name=self._n(node))

    def _op_Concat(self, node, a, ins):
        return self.S.concat(*[self.sym(i) for i in ins], dim=a.get('axis', 1), name=self._n(node))

    def _op_Transpose(self, node, a, ins):
        perm = a.get('perm')
        return self.S.transpose(self.sym(ins[0]), axes=tuple(perm) if perm else (), name=self._n(node))

    def _op_Unsqueeze(self, node, a, ins):
        axes = sorted(int(x) for x in (a['axes'] if 'axes' in a else self.const(ins[1])))
        s = self.sym(ins[0])
        for ax in axes:
            s = self.S.expand_dims(s, axis=ax)
        return s

    def _op_Squeeze(self, node, a, ins):
        axes = a.get('axes') if 'axes' in a else (list(self.const(ins[1])) if len(ins) > 1 and ins[1] else None)
        return self.S.squeeze(self.sym(ins[0]), axis=tuple(int(x) for x in axes) if axes else None, name=self._n(node))

    def _op_Clip(self, node, a, ins):
        lo = _scalar(self.const(ins[1])) if len(ins) > 1 and ins[1] else a.get('min', -np.inf)
        hi = _scalar(self.const(ins[2])) if len(ins) > 2 and ins[2] else a.get('max', np.inf)
        return self.S.clip(self.sym(ins[0]), a_min=lo, a_max=hi, name=self._n(node))

    def _reduce(self, node, a, ins, op):
        axes = a.get('axes')
        if axes is None and len(ins) > 1 and ins[1]:
            axes = [int(x) for x in self.const(ins[1])]
        kw = dict(keepdims=bool(a.get('keepdims', 1)), name=self._n(node))
        if axes:
            kw['axis'] = tuple(int(x) for x in axes)
        return getattr(self.S, op)(self.sym(ins[0]), **kw)

    def _op_ReduceMean(self, node, a, ins):
        return self._reduce(node, a, ins, 'mean')

    def _op_ReduceSum(self, node, a, ins):
        return self._reduce(node, a, ins, 'sum')

    def _op_ReduceMax(self, node, a, ins):
        return self._reduce(node, a, ins, 'max')

    def _op_ReduceMin(self, node, a, ins):
        return self._reduce(node, a, ins, 'min')

    def _op_ReduceProd(self, node, a, ins):
        return self._reduce(node, a, ins, 'prod')

    def _op_Gather(self, node, a, ins):
        return self.S.take(self.sym(ins[0]), self.sym(ins[1]), axis=a.get('axis', 0), name=self._n(node))

    def _op_Cast(self, node, a, ins):
        return self.S.Cast(self.sym(ins[0]), dtype=P.onnx_to_dtype(a['to']).name, name=self._n(node))

    def _op_Slice(self, node, a, ins):
        starts = [int(x) for x in self.const(ins[1])]
        ends = [int(x) for x in self.const(ins[2])]
        axes = [int(x) for x in self.const(ins[3])] if len(ins) > 3 and ins[3] else list(range(len(starts)))
        steps = [int(x) for x in self.const(ins[4])] if len(ins) > 4 and ins[4] else [1] * len(starts)
        s = self.sym(ins[0])
        big = np.iinfo(np.int64).max // 2
        for b, e, ax, st in zip(starts, ends, axes, steps):
            if st != 1:
                raise NotImplementedError('ONNX import: Slice with step %d' % st)
            s = self.S.slice_axis(s, axis=ax, begin=b, end=None if e >= big else e)
        return s

    def _op_Pad(self, node, a, ins):
        pads = [int(x) for x in (self.const(ins[1]) if len(ins) > 1 else a['pads'])]
        nd = len(pads) // 2
        pw = []
        for i in range(nd):
            pw += [pads[i], pads[i + nd]]
        val = _scalar(self.const(ins[2])) if len(ins) > 2 and ins[2] else a.get('value', 0.0)
        mode = a.get('mode', 'constant')
        return self.S.Pad(self.sym(ins[0]), mode=mode, pad_width=tuple(pw), constant_value=val, name=self._n(node))

    def _op_Resize(self, node, a, ins):
        if a.get('mode', 'nearest') != 'nearest':
            raise NotImplementedError('ONNX import: Resize mode %s' % a.get('mode'))
        scales = self.const(ins[2]) if len(ins) > 2 and ins[2] else None
        if scales is None or len(scales) != 4 or scales[2] != scales[3] or scales[0] != 1 or scales[1] != 1:
            raise NotImplementedError('ONNX import: Resize needs constant scales [1, 1, s, s]')
        return self.S.UpSampling(self.sym(ins[0]), scale=int(scales[2]), sample_type='nearest', name=self._n(node))

    _op_Upsample = _op_Resize

    def _op_Split(self, node, a, ins):
        split = a.get('split') or (list(self.const(ins[1])) if len(ins) > 1 and ins[1] else None)
        n = len(node.output)
        if split and len(set(int(x) for x in split)) != 1:
            raise NotImplementedError('ONNX import: uneven Split %s' % split)
        outs = self.S.split(self.sym(ins[0]), num_outputs=n, axis=a.get('axis', 0), name=self._n(node))
        return [outs[i] for i in range(n)]

    def _op_Expand(self, node, a, ins):
        return self.S.broadcast_to(self.sym(ins[0]), shape=tuple(int(x) for x in self.const(ins[1])),
                                   name=self._n(node))

    def _op_Tile(self, node, a, ins):
        return self.S.tile(self.sym(ins[0]), reps=tuple(int(x) for x in self.const(ins[1])), name=self._n(node))

    def _op_Where(self, node, a, ins):
        return self.S.where(self.sym(ins[0]), self.sym(ins[1]), self.sym(ins[2]), name=self._n(node))

    def _op_ArgMax(self, node, a, ins):
        return self.S.argmax(self.sym(ins[0]), axis=a.get('axis', 0), keepdims=bool(a.get('keepdims', 1)),
                             name=self._n(node))

    def _op_ArgMin(self, node, a, ins):
        return self.S.argmin(self.sym(ins[0]), axis=a.get('axis', 0), keepdims=bool(a.get('keepdims', 1)),
                             name=self._n(node))


def from_onnx(model):
    """(sym, arg_params, aux_params) of a ModelProto."""
    from .. import ndarray as nd
    imp = _Importer(model.graph)
    sym = imp.run()
    aux = set(sym.list_auxiliary_states())
    args = set(sym.list_arguments())
    arg_params, aux_params = {}, {}
    for k, v in imp.used_params.items():
        if k in aux:
            aux_params[k] = nd.array(v, dtype=v.dtype)
        elif k in args:
            arg_params[k] = nd.array(v, dtype=v.dtype)
    return sym, arg_params, aux_params


def graph_metadata(graph):
    params = {t.name for t in graph.initializer}
    inputs = []
    for vi in graph.input:
        if vi.name not in params:
            tt = vi.type.tensor_type
            inputs.append((vi.name, tuple(d.dim_value for d in tt.shape.dim), tt.elem_type))
    outputs = [(vi.name, tuple(d.dim_value for d in vi.type.tensor_type.shape.dim)) for vi in graph.output]
    return {'input_tensor_data': inputs, 'output_tensor_data': outputs}


def import_model(model_file):
    """Import an ONNX file: (sym, arg_params, aux_params) (reference contrib/onnx/onnx2mx/import_model.py:24)."""
    return from_onnx(P.load_model(model_file))


def get_model_metadata(model_file):
    """Names and shapes of the model's data inputs and outputs (import_model.py:63)."""
    return graph_metadata(P.load_model(model_file).graph)


def import_to_gluon(model_file, ctx):
    """A SymbolBlock with the model's parameters loaded on ``ctx`` (import_to_gluon.py:24)."""
    from .. import symbol as S
    from ..gluon import SymbolBlock
    model = P.load_model(model_file)
    sym, arg_params, aux_params = from_onnx(model)
    meta = graph_metadata(model.graph)
    inputs = [S.Variable(n) for n, _s, _t in meta['input_tensor_data']]
    net = SymbolBlock(sym, inputs)
    params = net.collect_params()
    for k, v in list(arg_params.items()) + list(aux_params.items()):
        if k in params:
            params[k]._load_init(v, ctx) if hasattr(params[k], '_load_init') else params[k].set_data(v)
    for k, p in params.items():
        if p._data is None:
            p.initialize(ctx=ctx)
    return net
