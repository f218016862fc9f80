"""``_FusedOp``: a chain of elementwise operators run as ONE generated gfx950 kernel.

The symbolic pointwise-fusion pass (symbol/passes.py ``fuse_pointwise``; reference
src/executor/pointwise_fusion_pass.cc + src/operator/fusion/fused_op.cu, which generates CUDA and
compiles it with NVRTC) replaces single-consumer elementwise chains by a ``_FusedOp`` node carrying
the chain as a JSON subgraph.  Here that subgraph becomes HIP C++ -- one expression per node, all
intermediates in registers -- compiled for gfx950 by the runtime compiler (rtc.py: hipcc --genco,
content-hash cached) and launched on the current stream: the intermediates never touch HBM and the
chain costs one launch.

The generated kernel serves inference (no autograd recording) on same-shape contiguous
fp32/fp16/bf16 inputs; anything else -- recording for a backward pass, broadcasting inputs, CPU --
runs the subgraph op by op (so gradients flow through the ordinary per-op autograd).
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


def kernel_source(graph, dtype):
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


def _hip_kernel(subgraph, graph, dtype, n_in):
    key = (subgraph, dtype)
    k = _KERNELS.get(key, 0)
    if k == 0:
        k = None
        src = kernel_source(graph, dtype)
        if src is not None:
            from .. import rtc
            sig = ', '.join(['const %s* in%d' % ('half' if dtype != torch.float32 else 'float', i)
                             for i in range(n_in)] + ['%s* out' % ('half' if dtype != torch.float32 else 'float'),
                                                      'int64_t n'])
            k = rtc.CudaModule(src, exports=['fused_pointwise']).get_kernel('fused_pointwise', sig)
        _KERNELS[key] = k
    return k


def _hip_ok(inputs):
    if not inputs or not all(isinstance(t, torch.Tensor) and t.is_cuda for t in inputs):
        return False
    t0 = inputs[0]
    return (t0.dtype in _CTYPE and all(t.dtype == t0.dtype and t.shape == t0.shape and t.is_contiguous()
                                       for t in inputs)
            and not (torch.is_grad_enabled() and any(t.requires_grad for t in inputs)))


def _fused_args(a):
    return ['data%d' % i for i in range(int(a.get('num_inputs', 1)))]


@register('_FusedOp', arg_names=_fused_args, params={'num_inputs': ('int', 1), 'subgraph': ('str', '')})
def fused_op(*inputs, num_inputs=1, subgraph=''):
    """Run a fused elementwise chain: one generated HIP kernel when possible, else op by op."""
    sym, prog, graph = _program(subgraph)
    if _hip_ok(inputs):
        k = _hip_kernel(subgraph, graph, inputs[0].dtype, len(inputs))
        if k is not None:
            from ..context import Context
            out = torch.empty_like(inputs[0])
            n = out.numel()
            grid = max(1, min((n + 255) // 256, 8192))
            k.launch(list(inputs) + [out, n], Context('gpu', inputs[0].device.index or 0), (grid, 1, 1),
                     (256, 1, 1))
            return out
    feed = {'data%d' % i: t for i, t in enumerate(inputs)}
    return prog.run(feed)[0]
