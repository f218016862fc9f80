"""``_FusedOp``: a chain of elementwise operators run as ONE generated gfx950 kernel.

The symbolic pointwise-fusion pass (symbol/passes.py ``fuse_pointwise``; reference
src/executor/pointwise_fusion_pass.cc + src/operator/fusion/fused_op.cu, which generates CUDA and
compiles it with NVRTC) replaces single-consumer elementwise chains by a ``_FusedOp`` node carrying
the chain as a JSON subgraph.  Here that subgraph becomes HIP C++ -- one expression per node, all
intermediates in registers -- compiled for gfx950 by the runtime compiler (rtc.py: hipcc --genco,
content-hash cached) and launched on the current stream: the intermediates never touch HBM and the
chain costs one launch.

Training graphs (reference: FusePointwise runs over forward AND backward on GPU) get a second
generated kernel: the backward of the whole chain, derived symbolically here (reverse-mode over the
expression DAG, per-op rules in ``_D_*``).  It recomputes the forward values in registers from the
saved inputs and writes every input's gradient in one pass, so a fused chain costs one kernel
forward and one backward, with no intermediate saved.  Both kernels serve same-shape contiguous
fp32/fp16/bf16 GPU inputs; anything else (broadcasting inputs, CPU) runs the subgraph op by op, with
gradients through the ordinary per-op autograd.
"""
import json

import torch

from .registry import register

# canonical operator name -> C expression over x (unary) or a, b (binary); s = the scalar attribute
_UNARY = {
    'relu': 'fmaxf(x, 0.f)', 'sigmoid': '1.f / (1.f + expf(-x))', 'tanh': 'tanhf(x)', 'exp': 'expf(x)',
    'log': 'logf(x)', 'sqrt': 'sqrtf(x)', 'rsqrt': 'rsqrtf(x)', 'square': 'x * x', 'abs': 'fabsf(x)',
    'negative': '-x', 'reciprocal': '1.f / x', 'sin': 'sinf(x)', 'cos': 'cosf(x)', 'erf': 'erff(x)',
    'softsign': 'x / (1.f + fabsf(x))', 'log1p': 'log1pf(x)', 'expm1': 'expm1f(x)', 'floor': 'floorf(x)',
    'ceil': 'ceilf(x)', 'round': 'roundf(x)', 'trunc': 'truncf(x)', 'sign': '(float)((x > 0.f) - (x < 0.f))',
    'cbrt': 'cbrtf(x)', 'rcbrt': '1.f / cbrtf(x)', 'log2': 'log2f(x)', 'log10': 'log10f(x)',
}
_ACT = {'relu': 'relu', 'sigmoid': 'sigmoid', 'tanh': 'tanh', 'softsign': 'softsign', 'softrelu': None}
_SCALAR = {
    '_plus_scalar': 'x + s', '_minus_scalar': 'x - s', '_rminus_scalar': 's - x', '_mul_scalar': 'x * s',
    '_div_scalar': 'x / s', '_rdiv_scalar': 's / x', '_power_scalar': 'powf(x, s)', '_rpower_scalar': 'powf(s, x)',
    '_maximum_scalar': 'fmaxf(x, s)', '_minimum_scalar': 'fminf(x, s)',
}
_BINARY = {'elemwise_add': 'a + b', 'elemwise_sub': 'a - b', 'elemwise_mul': 'a * b', 'elemwise_div': 'a / b',
           '_maximum': 'fmaxf(a, b)', '_minimum': 'fminf(a, b)'}

# derivative rules: adjoint contribution to each input, in terms of the input value(s) x / a / b,
# the node's own value y, the scalar attribute s and the node's adjoint g
_D_UNARY = {
    'relu': 'g * (x > 0.f ? 1.f : 0.f)', 'sigmoid': 'g * y * (1.f - y)', 'tanh': 'g * (1.f - y * y)',
    'exp': 'g * y', 'log': 'g / x', 'sqrt': '0.5f * g / y', 'rsqrt': '-0.5f * g * y / x', 'square': '2.f * g * x',
    'abs': 'g * (float)((x > 0.f) - (x < 0.f))', 'negative': '-g', 'reciprocal': '-g * y * y',
    'sin': 'g * cosf(x)', 'cos': '-g * sinf(x)', 'erf': '1.1283791670955126f * g * expf(-x * x)',
    'softsign': 'g / ((1.f + fabsf(x)) * (1.f + fabsf(x)))', 'log1p': 'g / (1.f + x)', 'expm1': 'g * (y + 1.f)',
    'floor': '0.f', 'ceil': '0.f', 'round': '0.f', 'trunc': '0.f', 'sign': '0.f',
    'cbrt': 'g * y / (3.f * x)', 'rcbrt': '-g * y / (3.f * x)', 'log2': 'g / (x * 0.6931471805599453f)',
    'log10': 'g / (x * 2.302585092994046f)',
}
_D_SCALAR = {
    '_plus_scalar': 'g', '_minus_scalar': 'g', '_rminus_scalar': '-g', '_mul_scalar': 'g * s',
    '_div_scalar': 'g / s', '_rdiv_scalar': '-g * s / (x * x)', '_power_scalar': 'g * s * powf(x, s - 1.f)',
    '_rpower_scalar': 'g * y * logf(s)', '_maximum_scalar': 'g * (x >= s ? 1.f : 0.f)',
    '_minimum_scalar': 'g * (x <= s ? 1.f : 0.f)',
}
_D_BINARY = {
    'elemwise_add': ('g', 'g'), 'elemwise_sub': ('g', '-g'), 'elemwise_mul': ('g * b', 'g * a'),
    'elemwise_div': ('g / b', '-g * a / (b * b)'), '_maximum': ('g * (a >= b ? 1.f : 0.f)', 'g * (a < b ? 1.f : 0.f)'),
    '_minimum': ('g * (a <= b ? 1.f : 0.f)', 'g * (a > b ? 1.f : 0.f)'),
}

_LOAD = {torch.float32: 'float(p[i])', torch.float16: '__half2float(p[i])',
         torch.bfloat16: '__uint_as_float(((unsigned)p[i]) << 16)'}
_CTYPE = {torch.float32: 'float', torch.float16: '__half', torch.bfloat16: 'unsigned short'}

_PROGRAMS = {}
_KERNELS = {}


def _program(subgraph):
    prog = _PROGRAMS.get(subgraph)
    if prog is None:
        from ..symbol.symbol import load_json
        sym = load_json(subgraph)
        from ..executor import GraphProgram
        prog = _PROGRAMS[subgraph] = (sym, GraphProgram(sym), json.loads(subgraph))
    return prog


def _subst(template, **vals):
    out = []
    i = 0
    while i < len(template):
        c = template[i]
        if c in vals and (i == 0 or not template[i - 1].isalnum()) and \
                (i + 1 == len(template) or not template[i + 1].isalnum()):
            out.append(vals[c])
        else:
            out.append(c)
        i += 1
    return ''.join(out)


def _expr_safe(node, args):
    """As _expr, with whole-identifier substitution of x / a / b / s (so 'expf' keeps its x-free name)."""
    from . import registry as _reg
    op = _reg.get(node['op'])
    name = op.name
    attrs = op.parse_attrs(node.get('attrs', {}))
    if name == 'Activation':
        name = _ACT.get(attrs.get('act_type'))
        if name is None:
            return None
    if name in _UNARY and len(args) == 1:
        return '(%s)' % _subst(_UNARY[name], x='(%s)' % args[0])
    if name in _SCALAR and len(args) == 1:
        return '(%s)' % _subst(_SCALAR[name], x='(%s)' % args[0], s='%.9ef' % float(attrs.get('scalar', 0.0)))
    if name in _BINARY and len(args) == 2:
        return '(%s)' % _subst(_BINARY[name], a='(%s)' % args[0], b='(%s)' % args[1])
    return None


def _node_rule(node):
    """(canonical name, parsed attrs) of a subgraph node, Activation resolved to its act_type."""
    from . import registry as _reg
    op = _reg.get(node['op'])
    attrs = op.parse_attrs(node.get('attrs', {}))
    name = op.name
    if name == 'Activation':
        name = _ACT.get(attrs.get('act_type'))
    return name, attrs


def _store(dtype, dst, val):
    if dtype == torch.float32:
        return '%s = %s;' % (dst, val)
    if dtype == torch.float16:
        return '%s = __float2half(%s);' % (dst, val)
    return ('{ unsigned u = __float_as_uint(%s); u += 0x7fffu + ((u >> 16) & 1u); '
            '%s = (unsigned short)(u >> 16); }' % (val, dst))


def backward_source(graph, dtype):
    """HIP source of the chain's backward kernel: recompute the forward values from the saved inputs,
    then propagate the output adjoint to every input (reverse topological order, all in registers).
    None when some node has no derivative rule."""
    nodes = graph['nodes']
    n_in = sum(1 for d in nodes if d['op'] == 'null')
    fwd = kernel_source(graph, dtype, body_only=True)
    if fwd is None:
        return None
    head = graph['heads'][0][0]
    lines = [fwd, '    float d%d = %s;' % (head, _LOAD[dtype].replace('p[', 'gout['))]
    for i, d in enumerate(nodes):
        if i != head:
            lines.append('    float d%d = 0.f;' % i)
    for i in range(len(nodes) - 1, -1, -1):
        d = nodes[i]
        if d['op'] == 'null':
            continue
        name, attrs = _node_rule(d)
        ins = [a[0] for a in d['inputs']]
        vals = {'g': 'd%d' % i, 'y': 'v%d' % i, 's': '%.9ef' % float(attrs.get('scalar', 0.0))}
        if name in _D_UNARY and len(ins) == 1:
            rules = [_D_UNARY[name]]
            vals['x'] = 'v%d' % ins[0]
        elif name in _D_SCALAR and len(ins) == 1:
            rules = [_D_SCALAR[name]]
            vals['x'] = 'v%d' % ins[0]
        elif name in _D_BINARY and len(ins) == 2:
            rules = list(_D_BINARY[name])
            vals['a'], vals['b'] = 'v%d' % ins[0], 'v%d' % ins[1]
        else:
            return None
        for src, rule in zip(ins, rules):
            lines.append('    d%d += %s;' % (src, _subst(rule, **vals)))
    for i, d in enumerate(nodes):
        if d['op'] == 'null':
            lines.append('    ' + _store(dtype, 'gin%d[i]' % int(d['name'][4:]), 'd%d' % i))
    ct = _CTYPE[dtype]
    params = ', '.join(['const %s* __restrict__ in%d' % (ct, k) for k in range(n_in)] +
                       ['const %s* __restrict__ gout' % ct] +
                       ['%s* __restrict__ gin%d' % (ct, k) for k in range(n_in)] + ['long n'])
    return ('extern "C" __global__ void __launch_bounds__(256) fused_pointwise_bwd(%s) {\n'
            '  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {\n'
            '%s\n  }\n}\n') % (params, '\n'.join(lines))


def kernel_source(graph, dtype, body_only=False):
    """HIP source of the fused kernel for a subgraph (JSON dict) and storage dtype; None if some node
    has no generated form."""
    nodes = graph['nodes']
    n_in = sum(1 for d in nodes if d['op'] == 'null')
    expr = {}
    lines = []
    for i, d in enumerate(nodes):
        if d['op'] == 'null':
            k = int(d['name'][4:])
            lines.append('    const float v%d = %s;' % (i, _LOAD[dtype].replace('p[', 'in%d[' % k)))
            expr[i] = 'v%d' % i
            continue
        e = _expr_safe(d, [expr[a[0]] for a in d['inputs']])
        if e is None:
            return None
        lines.append('    const float v%d = %s;' % (i, e))
        expr[i] = 'v%d' % i
    if body_only:
        return '\n'.join(lines)
    head = graph['heads'][0][0]
    ct = _CTYPE[dtype]
    if dtype == torch.float32:
        store = 'out[i] = v%d;' % head
    elif dtype == torch.float16:
        store = 'out[i] = __float2half(v%d);' % head
    else:
        store = ('{ unsigned u = __float_as_uint(v%d); u += 0x7fffu + ((u >> 16) & 1u); '
                 'out[i] = (unsigned short)(u >> 16); }' % head)
    params = ', '.join(['const %s* __restrict__ in%d' % (ct, k) for k in range(n_in)] +
                       ['%s* __restrict__ out' % ct, 'long n'])
    return ('extern "C" __global__ void __launch_bounds__(256) fused_pointwise(%s) {\n'
            '  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {\n'
            '%s\n    %s\n  }\n}\n') % (params, '\n'.join(lines), store)


def _compile(key, src, name, n_ptr):
    k = _KERNELS.get(key, 0)
    if k == 0:
        k = None
        if src is not None:
            from .. import rtc
            sig = ', '.join(['const float* p%d' % i for i in range(n_ptr)] + ['int64_t n'])
            k = rtc.CudaModule(src, exports=[name]).get_kernel(name, sig)
        _KERNELS[key] = k
    return k


def _hip_kernel(subgraph, graph, dtype, n_in):
    return _compile((subgraph, dtype), kernel_source(graph, dtype), 'fused_pointwise', n_in + 1)


def _hip_bwd_kernel(subgraph, graph, dtype, n_in):
    return _compile((subgraph, dtype, 'bwd'), backward_source(graph, dtype), 'fused_pointwise_bwd', 2 * n_in + 1)


def _launch(kernel, tensors, n):
    from ..context import Context
    grid = max(1, min((n + 255) // 256, 8192))
    kernel.launch(list(tensors) + [n], Context('gpu', tensors[0].device.index or 0), (grid, 1, 1), (256, 1, 1))


def _hip_ok(inputs):
    if not inputs or not all(isinstance(t, torch.Tensor) and t.is_cuda for t in inputs):
        return False
    t0 = inputs[0]
    return t0.dtype in _CTYPE and all(t.dtype == t0.dtype and t.shape == t0.shape and t.is_contiguous()
                                      for t in inputs)


class _FusedChain(torch.autograd.Function):
    """Generated forward kernel; backward = the generated adjoint kernel over the saved inputs."""

    @staticmethod
    def forward(ctx, fwd, bwd, *inputs):
        out = torch.empty_like(inputs[0])
        _launch(fwd, list(inputs) + [out], out.numel())
        ctx.bwd = bwd
        ctx.save_for_backward(*inputs)
        return out

    @staticmethod
    def backward(ctx, gout):
        inputs = ctx.saved_tensors
        grads = [torch.empty_like(t) for t in inputs]
        _launch(ctx.bwd, list(inputs) + [gout.contiguous()] + grads, gout.numel())
        return (None, None) + tuple(g if need else None for g, need in zip(grads, ctx.needs_input_grad[2:]))


def _fused_args(a):
    return ['data%d' % i for i in range(int(a.get('num_inputs', 1)))]


@register('_FusedOp', arg_names=_fused_args, params={'num_inputs': ('int', 1), 'subgraph': ('str', '')})
def fused_op(*inputs, num_inputs=1, subgraph=''):
    """Run a fused elementwise chain: one generated HIP kernel when possible, else op by op."""
    sym, prog, graph = _program(subgraph)
    if _hip_ok(inputs):
        dtype, n_in = inputs[0].dtype, len(inputs)
        fwd = _hip_kernel(subgraph, graph, dtype, n_in)
        if fwd is not None:
            if torch.is_grad_enabled() and any(t.requires_grad for t in inputs):
                bwd = _hip_bwd_kernel(subgraph, graph, dtype, n_in)
                if bwd is not None:
                    return _FusedChain.apply(fwd, bwd, *inputs)
            else:
                out = torch.empty_like(inputs[0])
                _launch(fwd, list(inputs) + [out], out.numel())
                return out
    feed = {'data%d' % i: t for i, t in enumerate(inputs)}
    return prog.run(feed)[0]
