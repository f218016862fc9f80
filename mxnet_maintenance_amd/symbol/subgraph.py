"""Graph partitioning into subgraph nodes (reference src/operator/subgraph/build_subgraph.cc,
default_subgraph_property.cc / default_subgraph_property_v2.cc, the MXBuildSubgraphByOpNames /
MXSetSubgraphPropertyOpNames C API and ``Symbol.optimize_for``).

A *backend* is a named property holding the operator names it claims.  Partitioning walks the graph
in topological order and grows groups of selected nodes; a node joins the group of a selected
producer only if none of its other inputs depends on that group -- so every group is convex and the
partitioned graph stays acyclic.  Each group becomes one ``_CachedOp`` node whose ``subgraph``
attribute is the group as a JSON graph (external entries become ``data<i>`` variables, in the order
the original graph visits them, so the argument / auxiliary-state lists of the partitioned symbol are
those of the original).  A ``_CachedOp`` runs its subgraph through the same GraphProgram as an
executor, infers shapes by inferring its subgraph, and keeps auxiliary states (BatchNorm moving
statistics) as auxiliary inputs.
"""
import json
import os

import torch

from ..ops import registry
from ..ops.registry import register

__all__ = ['set_backend_op_names', 'remove_backend', 'backend_op_names', 'partition', 'partition_for_backend']

_BACKENDS = {}


def set_backend_op_names(backend, op_names):
    _BACKENDS[backend] = list(op_names)


def remove_backend(backend):
    _BACKENDS.pop(backend, None)


def backend_op_names(backend):
    return _BACKENDS.get(backend)


def _depends_on(node, members, memo):
    """True when ``node`` (outside ``members``) has a member among its ancestors."""
    key = id(node)
    if key in memo:
        return memo[key]
    memo[key] = False
    stack = [node]
    seen = {id(node)}
    hit = False
    while stack and not hit:
        x = stack.pop()
        for a, _ in x.inputs:
            if id(a) in members:
                hit = True
                break
            if id(a) not in seen:
                seen.add(id(a))
                stack.append(a)
    memo[key] = hit
    return hit


def _group_convex(order, selectable, joinable=None):
    """Greedy convex grouping in topological order: a selectable node joins the group of one of its
    inputs when ``joinable(input_node, node, group_members)`` allows it and the group stays convex
    (no path leaves the group and comes back); otherwise it starts a group.  Returns member lists."""
    groups, member_sets, group_of = [], [], {}
    for n in order:
        if n.op is None or not selectable(n):
            continue
        chosen = None
        for a, _ in n.inputs:
            g = group_of.get(id(a))
            if g is None or g == chosen:
                continue
            if joinable is not None and not joinable(a, n, groups[g]):
                continue
            members = member_sets[g]
            memo = {}
            if all(id(b) in members or not _depends_on(b, members, memo) for b, _ in n.inputs):
                chosen = g
                break
        if chosen is None:
            chosen = len(groups)
            groups.append([])
            member_sets.append(set())
        groups[chosen].append(n)
        member_sets[chosen].add(id(n))
        group_of[id(n)] = chosen
    return groups


def describe_groups(sym, order, groups):
    """Per group: its external input entries (``ext``, in the order a depth-first walk of the original
    graph reaches them), the entries used outside it (``outs``), the positions of auxiliary inputs
    among ``ext`` (``aux``) and the subgraph as a JSON-able dict whose inputs are ``data<i>``."""
    group_of = {id(m): gi for gi, g in enumerate(groups) for m in g}
    used_outside = set()
    for n in order:
        for a, j in n.inputs:
            if id(a) in group_of and group_of.get(id(n)) != group_of[id(a)]:
                used_outside.add((id(a), j))
    for n, j in sym._outputs:
        if id(n) in group_of:
            used_outside.add((id(n), j))
    aux_of = _aux_positions(order)
    descs = []
    for gi, g in enumerate(groups):
        members = {id(m) for m in g}
        ext, ext_idx, aux_idx = [], {}, []
        sub_nodes, local = [], {}
        outs = [(m, j) for m in g for j in range(m.num_outputs()) if (id(m), j) in used_outside]
        seen = set()
        for root, _ in outs:
            stack = [(root, 0)]
            while stack:
                m, i = stack.pop()
                if i == 0:
                    if id(m) in seen:
                        continue
                    seen.add(id(m))
                if i >= len(m.inputs):
                    continue
                stack.append((m, i + 1))
                a, j = m.inputs[i]
                if id(a) in members:
                    if id(a) not in seen:
                        stack.append((a, 0))
                elif (id(a), j) not in ext_idx:
                    ext_idx[(id(a), j)] = len(ext)
                    ext.append((a, j))
        for k, (a, j) in enumerate(ext):
            sub_nodes.append({'op': 'null', 'name': 'data%d' % k, 'inputs': []})
            local[('ext', id(a), j)] = len(sub_nodes) - 1
        for m in g:
            ins = []
            for p_, (a, j) in enumerate(m.inputs):
                if id(a) in members:
                    ins.append([local[id(a)], j, 0])
                    continue
                k = ext_idx[(id(a), j)]
                if (id(m), p_) in aux_of and k not in aux_idx:
                    aux_idx.append(k)
                ins.append([local[('ext', id(a), j)], 0, 0])
            attrs = {k: str(v) for k, v in m.attrs.items()}
            sub_nodes.append({'op': m.op, 'name': m.name, 'attrs': attrs, 'inputs': ins})
            local[id(m)] = len(sub_nodes) - 1
        graph = {'nodes': sub_nodes, 'arg_nodes': [i for i, d in enumerate(sub_nodes) if d['op'] == 'null'],
                 'heads': [[local[id(m)], j, 0] for m, j in outs], 'attrs': {}}
        descs.append({'ext': ext, 'outs': outs, 'aux': aux_idx, 'graph': graph})
    return descs


def rebuild(sym, order, groups, descs, make_node):
    """The partitioned Symbol: group ``gi`` becomes ``make_node(gi, desc, input_entries)`` (a new
    node whose outputs are ``desc['outs']`` in order); every other node is copied."""
    from .symbol import Symbol, _Node
    group_of = {id(m): gi for gi, g in enumerate(groups) for m in g}
    last = {gi: g[-1] for gi, g in enumerate(groups)}
    remap = {}

    def entry(a, j):
        r = remap.get((id(a), j))
        return r if r is not None else (remap.get(('node', id(a)), a), j)

    for n in order:
        gi = group_of.get(id(n))
        if gi is None:
            if n.op is None:
                continue
            remap[('node', id(n))] = _Node(n.op, n.name, n.attrs, [entry(a, j) for a, j in n.inputs])
            continue
        if last[gi] is not n:
            continue
        d = descs[gi]
        node = make_node(gi, d, [entry(a, j) for a, j in d['ext']])
        for k, (m, j) in enumerate(d['outs']):
            remap[(id(m), j)] = (node, k)
    new_outs = [entry(n, j) if n.op is not None else (n, j) for n, j in sym._outputs]
    return Symbol(new_outs)


def partition(sym, op_names):
    """Partition ``sym``: every convex group of nodes whose operator is in ``op_names`` becomes one
    ``_CachedOp`` node.  Returns a new Symbol (``sym`` is unchanged)."""
    from .symbol import _Node
    wanted = {id(registry.get(n)) for n in op_names if registry.has(n)}
    if not wanted:
        return sym
    order = sym._topo()
    groups = _group_convex(order, lambda n: id(n.opdef()) in wanted)
    if not groups:
        return sym
    descs = describe_groups(sym, order, groups)

    def make(gi, d, inputs):
        return _Node('_CachedOp', 'sg_%s_%d' % (groups[gi][0].name, gi),
                     {'num_inputs': str(len(d['ext'])), 'num_outputs': str(len(d['outs'])),
                      'aux_indices': ','.join(str(i) for i in d['aux']), 'subgraph': json.dumps(d['graph'])},
                     inputs)
    return rebuild(sym, order, groups, descs, make)


def _aux_positions(order):
    """(id(node), input position) pairs that are auxiliary-state inputs."""
    out = set()
    for n in order:
        if n.op is None:
            continue
        nargs = len(n.opdef().get_arg_names(n.parsed()))
        for p in range(nargs, len(n.inputs)):
            out.add((id(n), p))
        extra = _aux_index_fn(n)
        if extra is not None:
            for p in extra:
                out.add((id(n), p))
    return out


def _aux_index_fn(node):
    if node.op == '_CachedOp':
        s = node.attrs.get('aux_indices', '')
        return [int(x) for x in s.split(',') if x != '']
    return None


def same_shape(node):
    """True when a subgraph node is a one-input one-output chain of same-shape elementwise ops (shape
    inference may then run backwards through it, as through the ops themselves)."""
    from .symbol import _SAME_SHAPE
    if node.attrs.get('num_inputs') != '1' or node.attrs.get('num_outputs') != '1':
        return False
    g = json.loads(node.attrs.get('subgraph', '{}'))
    return all(d['op'] == 'null' or d['op'] in _SAME_SHAPE for d in g.get('nodes', []))


def partition_for_backend(sym, backend):
    names = _BACKENDS.get(backend)
    if names is None:
        return sym
    return partition(sym, names)


def env_partition(sym):
    """Partition for MXNET_SUBGRAPH_BACKEND when that backend has registered operator names."""
    backend = os.environ.get('MXNET_SUBGRAPH_BACKEND')
    if backend and backend in _BACKENDS:
        return partition(sym, _BACKENDS[backend])
    return sym


# ----------------------------------------------------------------------------- the subgraph operator
_PROGS = {}


def _prog(subgraph):
    p = _PROGS.get(subgraph)
    if p is None:
        from .symbol import load_json
        from ..executor import GraphProgram
        sym = load_json(subgraph)
        p = _PROGS[subgraph] = (sym, GraphProgram(sym))
    return p


def user_attrs(attrs):
    """Attributes of a ``_CachedOp`` built by hand from any symbol's JSON (reference
    tests/python/unittest/test_subgraph.py:27: ``mx.sym._internal._CachedOp(*args, subgraph=js)``):
    the positional inputs follow the subgraph's ``list_inputs()``; its variables are renamed
    ``data<i>`` in that order and the auxiliary positions recorded, as a partitioned group's are."""
    from .symbol import load_json
    g = json.loads(attrs['subgraph'])
    sym = load_json(attrs['subgraph'])
    inputs = sym.list_inputs()
    aux = set(sym.list_auxiliary_states())
    idx = {n: i for i, n in enumerate(inputs)}
    for nd in g['nodes']:
        if nd['op'] == 'null' and nd['name'] in idx:
            nd['name'] = 'data%d' % idx[nd['name']]
    out = dict(attrs)
    out['num_inputs'] = len(inputs)
    out['num_outputs'] = len(sym.list_outputs())
    out['aux_indices'] = ','.join(str(i) for i, n in enumerate(inputs) if n in aux)
    out['subgraph'] = json.dumps(g)
    return out


def _cached_args(a):
    n = int(a.get('num_inputs', 0))
    aux = {int(x) for x in str(a.get('aux_indices', '') or '').split(',') if x != ''}
    return ['data%d' % i for i in range(n) if i not in aux]


def _cached_infer(in_shapes, a):
    sym, _ = _prog(a['subgraph'])
    known = {'data%d' % i: tuple(s) for i, s in enumerate(in_shapes) if s is not None}
    arg, _, aux = sym.infer_shape_partial(**known)
    names = sym.list_arguments() + sym.list_auxiliary_states()
    res = {}
    for name, s in zip(names, list(arg) + list(aux)):
        i = int(name[4:])
        if in_shapes[i] is None and s and all(int(d) > 0 for d in s):
            res[i] = tuple(s)
    return res


@register('_CachedOp', aliases=('_subgraph_op', '_default_subgraph_op'), arg_names=_cached_args,
          num_outputs=lambda a: int(a.get('num_outputs', 1)), infer_params=_cached_infer,
          params={'num_inputs': ('int', 0), 'num_outputs': ('int', 1), 'aux_indices': ('str', ''),
                  'subgraph': ('str', '')})
def cached_op(*inputs, num_inputs=0, num_outputs=1, aux_indices='', subgraph=''):
    """Run a partitioned subgraph (its inputs in ``data<i>`` order)."""
    sym, prog = _prog(subgraph)
    outs = prog.run({'data%d' % i: t for i, t in enumerate(inputs)})
    return outs[0] if num_outputs == 1 else tuple(outs)


__all__ += ['cached_op', 'env_partition']
_ = torch
