"""Control-flow operators with subgraphs: ``_foreach``, ``_while_loop``, ``_cond``.

Parity: src/operator/control_flow.cc and python/mxnet/{ndarray,symbol}/contrib.py
(foreach / while_loop / cond).  The body graphs are stored in the node's
attributes as symbol JSON (so the op survives ``tojson``/``load_json``) and run
with a ``GraphProgram`` per iteration; the iterations are ordinary torch ops,
so autograd differentiates through the loop.
"""
import json

import torch

from .registry import register

_PROGRAMS = {}


def _program(js):
    p = _PROGRAMS.get(js)
    if p is None:
        from ..symbol import symbol as sym_mod
        from ..executor import GraphProgram
        p = GraphProgram(sym_mod.load_json(js))
        _PROGRAMS[js] = p
    return p


def _names(s):
    return json.loads(s) if isinstance(s, str) else list(s)


def _foreach_nout(a):
    return int(a.get('num_out_data', 1)) + len(_names(a.get('state_names', '[]')))


def _foreach_args(a):
    return (['data%d' % i for i in range(len(_names(a.get('data_names', '[]'))))] +
            ['state%d' % i for i in range(len(_names(a.get('state_names', '[]'))))] +
            ['remain%d' % i for i in range(len(_names(a.get('remain_names', '[]'))))])


def _foreach_infer(in_shapes, a):
    """Shapes of unknown loop states / free inputs from the body graph's (partial) shape inference,
    given the per-step slice shapes of the data (reference control_flow.cc ForeachShape)."""
    from ..symbol import symbol as sym_mod
    dn, sn, rn = _names(a.get('data_names', '[]')), _names(a.get('state_names', '[]')), \
        _names(a.get('remain_names', '[]'))
    names = dn + sn + rn
    known = {}
    for i, (name, shp) in enumerate(zip(names, in_shapes)):
        if shp is None:
            continue
        known[name] = tuple(shp[1:]) if i < len(dn) else tuple(shp)
    body = sym_mod.load_json(a['subgraph'])
    args = body.list_arguments()
    arg_shapes, _, _ = body.infer_shape_partial(**{k: v for k, v in known.items() if k in args})
    inferred = dict(zip(args, arg_shapes or []))
    fill = {}
    for i, name in enumerate(names):
        if in_shapes[i] is None and i >= len(dn) and inferred.get(name):
            fill[i] = tuple(inferred[name])
    return fill


@register('_foreach', arg_names=_foreach_args, num_outputs=_foreach_nout, infer_params=_foreach_infer,
          params={'subgraph': ('str', ''), 'data_names': ('str', '[]'), 'state_names': ('str', '[]'),
                  'remain_names': ('str', '[]'), 'num_out_data': ('int', 1)})
def foreach_op(*inputs, subgraph='', data_names='[]', state_names='[]', remain_names='[]', num_out_data=1):
    dn, sn, rn = _names(data_names), _names(state_names), _names(remain_names)
    prog = _program(subgraph)
    data = inputs[:len(dn)]
    states = list(inputs[len(dn):len(dn) + len(sn)])
    remain = inputs[len(dn) + len(sn):]
    T = data[0].shape[0]
    outs = [[] for _ in range(num_out_data)]
    for t in range(T):
        feed = dict(zip(dn, [d[t] for d in data]))
        feed.update(zip(sn, states))
        feed.update(zip(rn, remain))
        res = prog.run(feed)
        for i in range(num_out_data):
            outs[i].append(res[i])
        states = list(res[num_out_data:])
    stacked = [torch.stack(o) for o in outs]
    return tuple(stacked + states)


def _while_nout(a):
    return int(a.get('num_out_data', 0)) + len(_names(a.get('var_names', '[]')))


def _while_args(a):
    return (['var%d' % i for i in range(len(_names(a.get('var_names', '[]'))))] +
            ['remain%d' % i for i in range(len(_names(a.get('remain_names', '[]'))))])


@register('_while_loop', arg_names=_while_args, num_outputs=_while_nout,
          params={'cond_graph': ('str', ''), 'func_graph': ('str', ''), 'var_names': ('str', '[]'),
                  'remain_names': ('str', '[]'), 'num_out_data': ('int', 0), 'max_iterations': ('int', 1)})
def while_loop_op(*inputs, cond_graph='', func_graph='', var_names='[]', remain_names='[]', num_out_data=0,
                  max_iterations=1):
    vn, rn = _names(var_names), _names(remain_names)
    cprog, fprog = _program(cond_graph), _program(func_graph)
    loop_vars = list(inputs[:len(vn)])
    remain = inputs[len(vn):]
    outs = [[] for _ in range(num_out_data)]
    steps = 0
    meta = loop_vars[0].device.type == 'meta'
    while steps < max_iterations:
        feed = dict(zip(vn, loop_vars))
        feed.update(zip(rn, remain))
        if not meta:
            c = cprog.run(feed)[0]
            if not bool(c.reshape(-1)[0]):
                break
        res = fprog.run(feed)
        for i in range(num_out_data):
            outs[i].append(res[i])
        loop_vars = list(res[num_out_data:])
        steps += 1
        if meta:
            break
    stacked = []
    for i in range(num_out_data):
        if outs[i]:
            o = torch.stack(outs[i])
            if o.shape[0] < max_iterations:
                pad = torch.zeros((max_iterations - o.shape[0],) + tuple(o.shape[1:]), dtype=o.dtype, device=o.device)
                o = torch.cat([o, pad])
            stacked.append(o)
        else:
            stacked.append(torch.zeros((max_iterations,), device=loop_vars[0].device))
    return tuple(stacked + loop_vars)


def _cond_nout(a):
    return int(a.get('num_outputs', 1))


def _cond_args(a):
    return ['pred'] + ['input%d' % i for i in range(len(_names(a.get('input_names', '[]'))))]


@register('_cond', arg_names=_cond_args, num_outputs=_cond_nout,
          params={'then_graph': ('str', ''), 'else_graph': ('str', ''), 'input_names': ('str', '[]'),
                  'num_outputs': ('int', 1)})
def cond_op(pred, *inputs, then_graph='', else_graph='', input_names='[]', num_outputs=1):
    names = _names(input_names)
    feed = dict(zip(names, inputs))
    if pred.device.type == 'meta':
        res = _program(then_graph).run(feed)
    else:
        res = _program(then_graph if bool(pred.reshape(-1)[0]) else else_graph).run(feed)
    return tuple(res) if num_outputs > 1 else res[0]
