"""Symbol operators with prefix _contrib_ (mx.sym.contrib)."""
from ..ops import registry as _registry
from .symbol import _op_func
for _n in _registry.list_ops():
    if _n.startswith('_contrib_'):
        globals()[_n[len('_contrib_'):]] = _op_func(_n)


# ---------------------------------------------------------------------------
# control flow (parity: python/mxnet/symbol/contrib.py foreach / while_loop / cond)
# ---------------------------------------------------------------------------
import json as _json


def _as_list(x):
    return (list(x), True) if isinstance(x, (list, tuple)) else ([x], False)


def _flat(x):
    """(flat list of leaves, format) of a possibly nested list of symbols; the format is None for a
    single symbol, else the list of the items' formats (so ``[]`` and ``[[a], b]`` round-trip)."""
    if not isinstance(x, (list, tuple)):
        return [x], None
    leaves, fmt = [], []
    for item in x:
        lv, f = _flat(item)
        leaves.extend(lv)
        fmt.append(f)
    return leaves, fmt


def _unflat(leaves, fmt):
    """Inverse of _flat: (structure, leaves left over)."""
    if fmt is None:
        return leaves[0], leaves[1:]
    out = []
    for f in fmt:
        item, leaves = _unflat(leaves, f)
        out.append(item)
    return out, leaves


def _subgraph_name(base):
    """Unique subgraph name (reference symbol/contrib.py _get_unique_subgraph_name): nested inside
    another subgraph it is prefixed ``outer$``; the n-th subgraph of one name gets suffix n."""
    from ..attribute import AttrScope
    outer = AttrScope.current._attr.get('__subgraph_name__', '')
    if outer:
        base = outer + '$' + base
    AttrScope._subgraph_names[base] += 1
    return base + str(AttrScope._subgraph_names[base] - 1)


def _in_subgraph(base, build):
    """Run ``build()`` (the Python function that creates a subgraph's symbols) under the subgraph's
    unique name; returns (build's result, the name)."""
    from ..attribute import AttrScope
    name = _subgraph_name(base)
    with AttrScope(__subgraph_name__=name):
        return build(), name


def _free_vars(g, exclude):
    from .symbol import Symbol
    out = []
    for n in g._topo():
        if n.op is None and n.name not in exclude:
            out.append(Symbol([(n, 0)]))
    return out


def foreach(body, data, init_states, name='foreach'):
    """Run ``body(data_t, states) -> (outputs, new_states)`` over the leading axis of ``data``.

    ``data``, ``init_states`` and the body's outputs may be (nested) lists; the results keep the
    body's structure (an empty output list stays empty), as the reference's _flatten / _regroup do."""
    from .symbol import var, Group, _create
    data_l, data_fmt = _flat(data)
    states_l, states_fmt = _flat(init_states)
    d_ph = [var('%s_data%d' % (name, i)) for i in range(len(data_l))]
    s_ph = [var('%s_state%d' % (name, i)) for i in range(len(states_l))]
    (outs, new_states), _ = _in_subgraph(name, lambda: body(_unflat(d_ph, data_fmt)[0],
                                                            _unflat(s_ph, states_fmt)[0]))
    outs_l, outs_fmt = _flat(outs if outs is not None else [])
    new_l, new_fmt = _flat(new_states)
    if len(new_l) != len(states_l):
        raise ValueError('foreach: the body returned %d states for %d initial states' % (len(new_l), len(states_l)))
    g = Group(outs_l + new_l)
    # the reference's subgraph contract (python/mxnet/symbol/contrib.py foreach): every data array and
    # every state is an input of the loop body
    used = set(g.list_inputs())
    if any(s.name not in used for s in d_ph):
        raise AssertionError('the data arrays have to be used in the loop body')
    if any(s.name not in used for s in s_ph):
        raise AssertionError('the state arrays have to be used in the loop body')
    ph_names = {s.name for s in d_ph + s_ph}
    remain = _free_vars(g, ph_names)
    attrs = {'subgraph': g.tojson(), 'data_names': _json.dumps([s.name for s in d_ph]),
             'state_names': _json.dumps([s.name for s in s_ph]),
             'remain_names': _json.dumps([s.name for s in remain]), 'num_out_data': len(outs_l)}
    node = _create('_foreach', {'_pos': data_l + states_l + remain}, attrs, name=name)
    res = list(node)
    return _unflat(res[:len(outs_l)], outs_fmt)[0], _unflat(res[len(outs_l):], new_fmt)[0]


def while_loop(cond, func, loop_vars, max_iterations=None, name='while_loop'):
    """Symbolic while loop; per-step outputs are padded to ``max_iterations``.  Loop variables and
    step outputs may be (nested) lists; the results keep their structure."""
    from .symbol import var, Group, _create
    if max_iterations is None:
        raise ValueError('max_iterations should be specified')
    vars_l, vars_fmt = _flat(loop_vars)
    ph = [var('%s_var%d' % (name, i)) for i in range(len(vars_l))]
    arg = _unflat(ph, vars_fmt)[0]
    as_args = isinstance(arg, list)
    c, _ = _in_subgraph(name + '_cond', lambda: cond(*arg) if as_args else cond(arg))
    (outs, new_vars), _ = _in_subgraph(name + '_func', lambda: func(*arg) if as_args else func(arg))
    outs_l, outs_fmt = _flat(outs if outs is not None else [])
    new_l, _ = _flat(new_vars)
    if len(new_l) != len(vars_l):
        raise ValueError('while_loop: func returned %d loop variables for %d' % (len(new_l), len(vars_l)))
    fg = Group(outs_l + new_l)
    cg = Group([c])
    ph_names = {s.name for s in ph}
    remain = {s.name: s for s in _free_vars(fg, ph_names) + _free_vars(cg, ph_names)}
    remain = list(remain.values())
    attrs = {'cond_graph': cg.tojson(), 'func_graph': fg.tojson(), 'var_names': _json.dumps([s.name for s in ph]),
             'remain_names': _json.dumps([s.name for s in remain]), 'num_out_data': len(outs_l),
             'max_iterations': int(max_iterations)}
    node = _create('_while_loop', {'_pos': vars_l + remain}, attrs, name=name)
    res = list(node)
    # final loop variables take the structure of the initial ones (reference symbol/contrib.py)
    return _unflat(res[:len(outs_l)], outs_fmt)[0], _unflat(res[len(outs_l):], vars_fmt)[0]


def cond(pred, then_func, else_func, name='cond'):
    """Symbolic if/else: both branches are subgraphs over the free variables they use."""
    from .symbol import Group, _create
    _subgraph_name(name + '_pred')          # the predicate is a subgraph of its own in the reference
    then_out, _ = _in_subgraph(name + '_then', then_func)
    else_out, _ = _in_subgraph(name + '_else', else_func)
    t_l, t_is_list = _as_list(then_out)
    e_l, _ = _as_list(else_out)
    if len(t_l) != len(e_l):
        raise ValueError('then_func and else_func must return the same number of outputs')
    tg, eg = Group(t_l), Group(e_l)
    inputs = {s.name: s for s in _free_vars(tg, set()) + _free_vars(eg, set())}
    inputs = list(inputs.values())
    attrs = {'then_graph': tg.tojson(), 'else_graph': eg.tojson(),
             'input_names': _json.dumps([s.name for s in inputs]), 'num_outputs': len(t_l)}
    node = _create('_cond', {'_pos': [pred] + inputs}, attrs, name=name)
    res = list(node)
    return res if t_is_list else res[0]


def rand_zipfian(true_classes, num_sampled, range_max):
    """Symbolic log-uniform (Zipfian) candidate sampler: ``(sampled_classes, expected_count_true,
    expected_count_sampled)``, P(k) = log((k+2)/(k+1)) / log(range_max+1) (parity:
    python/mxnet/symbol/contrib.py rand_zipfian; the NDArray twin is ndarray/contrib.py)."""
    import math
    log_range = math.log(range_max + 1)
    rand = _op_func('_random_uniform')(low=0.0, high=log_range, shape=(num_sampled,), dtype='float64')
    sampled = _op_func('_mod_scalar')(_op_func('Cast')(_op_func('exp')(rand) - 1.0, dtype='int64'),
                                      scalar=float(range_max))

    def expected_count(classes):
        c = _op_func('Cast')(classes, dtype='float64')
        return _op_func('log')((c + 2.0) / (c + 1.0)) / log_range * num_sampled
    return sampled, expected_count(true_classes), expected_count(sampled)
