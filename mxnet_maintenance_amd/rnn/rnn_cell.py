"""Symbolic RNN cells (API parity: python/mxnet/rnn/rnn_cell.py).

A cell maps ``(inputs, states) -> (output, new_states)`` on Symbols and can be
``unroll``-ed over time.  Weights are symbol Variables held by an
``RNNParams`` container, named ``<prefix>i2h_weight`` / ``<prefix>h2h_bias``
etc. with all gates fused along the first axis (gate order: LSTM i, f, c, o;
GRU r, z, o -- the same order as the fused ``RNN`` operator, so
``FusedRNNCell`` and stacks of unfused cells exchange parameters through
``unpack_weights`` / ``pack_weights``).
"""
import warnings

from .. import symbol
from .. import initializer as init
from ..base import string_types, numeric_types

__all__ = ['RNNParams', 'BaseRNNCell', 'RNNCell', 'LSTMCell', 'GRUCell', 'FusedRNNCell', 'SequentialRNNCell',
           'DropoutCell', 'ModifierCell', 'ZoneoutCell', 'ResidualCell', 'BidirectionalCell',
           'BaseConvRNNCell', 'ConvRNNCell', 'ConvLSTMCell', 'ConvGRUCell']


def _time_major_split(length, inputs, layout, merge, in_layout=None):
    """Bring ``inputs`` into the requested form and return (inputs, time axis of ``layout``).

    ``merge`` True: one Symbol with time on the layout's T axis; False: a list of ``length``
    per-step Symbols; None: leave whichever form was given.  ``in_layout`` names the layout of a
    merged input when it differs from ``layout``."""
    if inputs is None:
        raise AssertionError('unroll(inputs=None) is not supported; pass the input symbol(s)')
    t_axis = layout.find('T')
    src_axis = t_axis if in_layout is None else in_layout.find('T')
    merged = isinstance(inputs, symbol.Symbol)
    if merged and merge is False:
        if len(inputs.list_outputs()) != 1:
            raise AssertionError('unroll needs a single-output input symbol or a list of symbols')
        steps = symbol.split(inputs, axis=src_axis, num_outputs=length, squeeze_axis=1)
        return list(steps), t_axis
    if not merged:
        if length is not None and len(inputs) != length:
            raise AssertionError('unroll length %s but %d input steps' % (length, len(inputs)))
        if merge is not True:
            return inputs, t_axis
        inputs = symbol.Concat(*[symbol.expand_dims(step, axis=t_axis) for step in inputs], dim=t_axis)
        src_axis = t_axis
    if src_axis != t_axis:
        inputs = symbol.swapaxes(inputs, dim0=t_axis, dim1=src_axis)
    return inputs, t_axis


# kept under the reference's private name for code written against it
_normalize_sequence = _time_major_split


class RNNParams:
    """Container of the Variables of a cell (shared between cells given the same instance)."""

    def __init__(self, prefix=''):
        self._prefix = prefix
        self._params = {}

    def get(self, name, **kwargs):
        """The Variable ``<prefix><name>`` (created on first request with ``kwargs``)."""
        key = self._prefix + name
        var = self._params.get(key)
        if var is None:
            var = self._params[key] = symbol.Variable(key, **kwargs)
        return var


class BaseRNNCell:
    """Abstract cell: subclasses implement ``state_info`` and ``__call__``.

    Subclasses with fused gates list the per-gate name suffixes in ``_GATES`` (their order is the
    row order of the fused i2h / h2h weights)."""

    _GATES = ()

    def __init__(self, prefix='', params=None):
        self._owns_params = params is None
        self._prefix = prefix
        self._params = RNNParams(prefix) if params is None else params
        self._modified = False
        self.reset()

    def reset(self):
        """Forget the time-step counters (call before building a new graph)."""
        self._init_counter = -1
        self._counter = -1
        for child in getattr(self, '_cells', ()):
            child.reset()

    def __call__(self, inputs, states):
        raise NotImplementedError

    @property
    def params(self):
        # once a caller holds the container it may be shared: the cell no longer owns it exclusively
        self._owns_params = False
        return self._params

    @property
    def state_info(self):
        raise NotImplementedError

    @property
    def state_shape(self):
        return [info['shape'] for info in self.state_info]

    @property
    def _gate_names(self):
        return self._GATES

    def _check_unmodified(self):
        if self._modified:
            raise AssertionError('after applying a modifier cell (e.g. ZoneoutCell) the base cell '
                                 'cannot be called directly; call the modifier cell instead')

    def begin_state(self, func=symbol.zeros, **kwargs):
        """Initial states (zeros by default; batch dimension 0 = inferred at bind time)."""
        self._check_unmodified()
        out = []
        for info in self.state_info:
            self._init_counter += 1
            spec = dict(kwargs)
            spec.update(info or {})
            out.append(func(name='%sbegin_state_%d' % (self._prefix, self._init_counter), **spec))
        return out

    def _standard_params(self, i2h_bias_init=None):
        """The four fused-gate Variables of a single-layer cell."""
        get = self.params.get
        self._iW = get('i2h_weight')
        self._hW = get('h2h_weight')
        self._iB = get('i2h_bias') if i2h_bias_init is None else get('i2h_bias', init=i2h_bias_init)
        self._hB = get('h2h_bias')

    def _nc_states(self, count):
        return [{'shape': (0, self._num_hidden), '__layout__': 'NC'} for _ in range(count)]

    # ---------------------------------------------------------------- (un)packing
    def _gate_key(self, group, gate, kind):
        return '%s%s%s_%s' % (self._prefix, group, gate, kind)

    def unpack_weights(self, args):
        """Split fused gate weights/biases in ``args`` into per-gate entries."""
        out = dict(args)
        rows = getattr(self, '_num_hidden', 0)
        for group in ('i2h', 'h2h') if self._gate_names else ():
            for kind in ('weight', 'bias'):
                fused = out.pop(self._gate_key(group, '', kind))
                for j, gate in enumerate(self._gate_names):
                    out[self._gate_key(group, gate, kind)] = fused[j * rows:(j + 1) * rows].copy()
        return out

    def pack_weights(self, args):
        """Inverse of ``unpack_weights``."""
        from .. import ndarray as nd
        out = dict(args)
        for group in ('i2h', 'h2h') if self._gate_names else ():
            for kind in ('weight', 'bias'):
                pieces = [out.pop(self._gate_key(group, gate, kind)) for gate in self._gate_names]
                out[self._gate_key(group, '', kind)] = nd.concat(*pieces, dim=0)
        return out

    # ---------------------------------------------------------------- unrolling
    def unroll(self, length, inputs, begin_state=None, layout='NTC', merge_outputs=None):
        """Apply the cell ``length`` times; returns (outputs, states)."""
        self.reset()
        steps, _ = _time_major_split(length, inputs, layout, False)
        states = begin_state if begin_state is not None else self.begin_state()
        outs = []
        for x in steps:
            y, states = self(x, states)
            outs.append(y)
        outs, _ = _time_major_split(length, outs, layout, merge_outputs)
        return outs, states

    def _get_activation(self, inputs, activation, **kwargs):
        if not isinstance(activation, string_types):
            return activation(inputs, **kwargs)
        return symbol.Activation(inputs, act_type=activation, **kwargs)

    def _fc_pair(self, inputs, prev_h, name):
        """i2h(inputs) and h2h(prev_h) projections for all of the cell's fused gates."""
        width = len(self._gate_names) * self._num_hidden
        return (symbol.FullyConnected(data=inputs, weight=self._iW, bias=self._iB, num_hidden=width,
                                      name=name + 'i2h'),
                symbol.FullyConnected(data=prev_h, weight=self._hW, bias=self._hB, num_hidden=width,
                                      name=name + 'h2h'))

    def _step_name(self):
        self._counter += 1
        return '%st%d_' % (self._prefix, self._counter)


class RNNCell(BaseRNNCell):
    """Elman cell: h' = act(W_i x + b_i + W_h h + b_h)."""

    _GATES = ('',)

    def __init__(self, num_hidden, activation='tanh', prefix='rnn_', params=None):
        super().__init__(prefix=prefix, params=params)
        self._num_hidden = num_hidden
        self._activation = activation
        self._standard_params()

    @property
    def state_info(self):
        return self._nc_states(1)

    def __call__(self, inputs, states):
        tag = self._step_name()
        i2h, h2h = self._fc_pair(inputs, states[0], tag)
        h = self._get_activation(i2h + h2h, self._activation, name=tag + 'out')
        return h, [h]


class LSTMCell(BaseRNNCell):
    """Long short-term memory cell; ``forget_bias`` initialises the forget-gate bias."""

    _GATES = ('_i', '_f', '_c', '_o')

    def __init__(self, num_hidden, prefix='lstm_', params=None, forget_bias=1.0):
        super().__init__(prefix=prefix, params=params)
        self._num_hidden = num_hidden
        self._standard_params(i2h_bias_init=init.LSTMBias(forget_bias=forget_bias))

    @property
    def state_info(self):
        return self._nc_states(2)

    def __call__(self, inputs, states):
        tag = self._step_name()
        i2h, h2h = self._fc_pair(inputs, states[0], tag)
        pre = symbol.SliceChannel(i2h + h2h, num_outputs=4, name=tag + 'slice')
        act = [symbol.Activation(pre[k], act_type='tanh' if k == 2 else 'sigmoid', name=tag + 'ifco'[k])
               for k in range(4)]
        c = symbol._internal._plus(act[1] * states[1], act[0] * act[2], name=tag + 'state')
        h = symbol._internal._mul(act[3], symbol.Activation(c, act_type='tanh'), name=tag + 'out')
        return h, [h, c]


class GRUCell(BaseRNNCell):
    """Gated recurrent unit (Cho et al. 2014), cuDNN / fused-op variant."""

    _GATES = ('_r', '_z', '_o')

    def __init__(self, num_hidden, prefix='gru_', params=None):
        super().__init__(prefix=prefix, params=params)
        self._num_hidden = num_hidden
        self._standard_params()

    @property
    def state_info(self):
        return self._nc_states(1)

    def __call__(self, inputs, states):
        tag = self._step_name()
        h_prev = states[0]
        i2h, h2h = self._fc_pair(inputs, h_prev, tag)
        xr, xz, xn = symbol.SliceChannel(i2h, num_outputs=3, name=tag + 'i2h_slice')
        hr, hz, hn = symbol.SliceChannel(h2h, num_outputs=3, name=tag + 'h2h_slice')
        r = symbol.Activation(xr + hr, act_type='sigmoid', name=tag + 'r_act')
        z = symbol.Activation(xz + hz, act_type='sigmoid', name=tag + 'z_act')
        n = symbol.Activation(xn + r * hn, act_type='tanh', name=tag + 'h_act')
        h = symbol._internal._plus((1. - z) * n, z * h_prev, name=tag + 'out')
        return h, [h]


_MODE_GATES = {'rnn_relu': RNNCell._GATES, 'rnn_tanh': RNNCell._GATES, 'lstm': LSTMCell._GATES,
               'gru': GRUCell._GATES}


class FusedRNNCell(BaseRNNCell):
    """Multi-layer (bi)directional RNN on the fused ``RNN`` operator (one flat parameter Variable)."""

    def __init__(self, num_hidden, num_layers=1, mode='lstm', bidirectional=False, dropout=0., get_next_state=False,
                 forget_bias=1.0, prefix=None, params=None):
        super().__init__(prefix='%s_' % mode if prefix is None else prefix, params=params)
        self._num_hidden = num_hidden
        self._num_layers = num_layers
        self._mode = mode
        self._bidirectional = bidirectional
        self._dropout = dropout
        self._get_next_state = get_next_state
        self._dirs = 'lr' if bidirectional else 'l'
        self._directions = list(self._dirs)
        flat_init = init.FusedRNN(None, num_hidden, num_layers, mode, bidirectional, forget_bias)
        self._parameter = self.params.get('parameters', init=flat_init)

    @property
    def _GATES(self):      # noqa: N802 -- per-instance: depends on the mode
        return _MODE_GATES[self._mode]

    @property
    def state_info(self):
        shape = (len(self._dirs) * self._num_layers, 0, self._num_hidden)
        return [{'shape': shape, '__layout__': 'LNC'} for _ in range(2 if self._mode == 'lstm' else 1)]

    @property
    def _num_gates(self):
        return len(self._GATES)

    def _layout_pieces(self, input_size):
        """(name, offset, shape) of every per-(layer, direction, gate) piece of the flat vector, and
        its total length: all weights (i2h then h2h per layer/direction) first, then all biases."""
        h, nd_ = self._num_hidden, len(self._dirs)
        pieces, pos = [], 0
        for kind in ('weight', 'bias'):
            for layer in range(self._num_layers):
                width = input_size if layer == 0 else h * nd_
                for d in self._dirs:
                    for group, cols in (('i2h', width), ('h2h', h)):
                        for gate in self._GATES:
                            shape = (h, cols) if kind == 'weight' else (h,)
                            name = '%s%s%d_%s%s_%s' % (self._prefix, d, layer, group, gate, kind)
                            pieces.append((name, pos, shape))
                            pos += h * (cols if kind == 'weight' else 1)
        return pieces, pos

    def _slice_weights(self, arr, li, lh):
        """Views of the per-(layer, direction, gate) pieces of ``arr`` keyed by unfused names."""
        del lh    # the hidden size is the cell's own
        pieces, total = self._layout_pieces(li)
        if total != arr.size:
            raise AssertionError('parameter vector of %d elements, expected %d' % (arr.size, total))
        return {name: arr[off:off + _prod(shape)].reshape(shape) for name, off, shape in pieces}

    def _input_size(self, total):
        """Layer-0 input size implied by a flat parameter count."""
        g, h, d = self._num_gates, self._num_hidden, len(self._dirs)
        deeper = (self._num_layers - 1) * d * g * h * (h * d + h + 2)
        return (total - deeper - d * g * h * (h + 2)) // (d * g * h)

    def unpack_weights(self, args):
        out = dict(args)
        flat = out.pop(self._parameter.name)
        for name, view in self._slice_weights(flat, self._input_size(flat.size), self._num_hidden).items():
            out[name] = view.copy()
        return out

    def pack_weights(self, args):
        from .. import ndarray as nd
        out = dict(args)
        first = out['%sl0_i2h%s_weight' % (self._prefix, self._GATES[0])]
        pieces, total = self._layout_pieces(first.shape[1])
        flat = nd.zeros((total,), ctx=first.context, dtype=first.dtype)
        for name, off, shape in pieces:
            flat[off:off + _prod(shape)] = out.pop(name).reshape((-1,))
        out[self._parameter.name] = flat
        return out

    def __call__(self, inputs, states):
        raise NotImplementedError('FusedRNNCell cannot be stepped; use unroll')

    def unroll(self, length, inputs, begin_state=None, layout='NTC', merge_outputs=None):
        self.reset()
        seq, t_axis = _time_major_split(length, inputs, layout, True)
        batch_major = t_axis == 1
        if batch_major:
            warnings.warn('NTC layout detected: FusedRNNCell runs in TNC, inputs are transposed')
            seq = symbol.swapaxes(seq, dim0=0, dim1=1)
        states = begin_state if begin_state is not None else self.begin_state()
        extra = {'state_cell': states[1]} if self._mode == 'lstm' else {}
        res = symbol.RNN(data=seq, parameters=self._parameter, state=states[0], state_size=self._num_hidden,
                         num_layers=self._num_layers, bidirectional=self._bidirectional, p=self._dropout,
                         state_outputs=self._get_next_state, mode=self._mode, name=self._prefix + 'rnn', **extra)
        if self._get_next_state:
            outs = res[0]
            new_states = [res[k] for k in range(1, 3 if self._mode == 'lstm' else 2)]
        else:
            outs, new_states = res, []
        if batch_major:
            outs = symbol.swapaxes(outs, dim0=0, dim1=1)
        outs, _ = _time_major_split(length, outs, layout, merge_outputs)
        return outs, new_states

    def unfuse(self):
        """An equivalent ``SequentialRNNCell`` of unfused cells (weights via unpack_weights)."""
        def cell(pfx):
            if self._mode == 'lstm':
                return LSTMCell(self._num_hidden, prefix=pfx)
            if self._mode == 'gru':
                return GRUCell(self._num_hidden, prefix=pfx)
            return RNNCell(self._num_hidden, activation=self._mode[len('rnn_'):], prefix=pfx)
        stack = SequentialRNNCell()
        for layer in range(self._num_layers):
            fwd = cell('%sl%d_' % (self._prefix, layer))
            if self._bidirectional:
                stack.add(BidirectionalCell(fwd, cell('%sr%d_' % (self._prefix, layer)),
                                            output_prefix='%sbi_l%d_' % (self._prefix, layer)))
            else:
                stack.add(fwd)
            if self._dropout > 0 and layer + 1 < self._num_layers:
                stack.add(DropoutCell(self._dropout, prefix='%s_dropout%d_' % (self._prefix, layer)))
        return stack


def _prod(shape):
    n = 1
    for s in shape:
        n *= s
    return n


class _Container(BaseRNNCell):
    """A cell built from child cells (``self._cells``): states, weights and parameters are the
    concatenation of the children's."""

    def _adopt(self, children, shared):
        """Merge the children's Variables into this container's (and, when this container was given
        ``params``, the container's into every child's first)."""
        for child in children:
            if shared:
                if not child._owns_params:
                    raise AssertionError('with params given to the container, child cells must own theirs')
                child.params._params.update(self._params._params)
        for child in children:
            self._params._params.update(child.params._params)

    @property
    def state_info(self):
        return [info for child in self._cells for info in child.state_info]

    def begin_state(self, **kwargs):
        self._check_unmodified()
        return [st for child in self._cells for st in child.begin_state(**kwargs)]

    def unpack_weights(self, args):
        for child in self._cells:
            args = child.unpack_weights(args)
        return args

    def pack_weights(self, args):
        for child in self._cells:
            args = child.pack_weights(args)
        return args

    def _per_child(self, states):
        """``states`` cut into the children's consecutive slices."""
        cuts, at = [], 0
        for child in self._cells:
            n = len(child.state_info)
            cuts.append(states[at:at + n])
            at += n
        return cuts


class SequentialRNNCell(_Container):
    """Stack of cells: the output of cell i is the input of cell i+1."""

    def __init__(self, params=None):
        super().__init__(prefix='', params=params)
        self._shared = params is not None
        self._cells = []

    def add(self, cell):
        self._cells.append(cell)
        self._adopt([cell], self._shared)

    def __call__(self, inputs, states):
        self._counter += 1
        carried = []
        for child, st in zip(self._cells, self._per_child(states)):
            if isinstance(child, BidirectionalCell):
                raise AssertionError('BidirectionalCell cannot be stepped; unroll the stack instead')
            inputs, st = child(inputs, st)
            carried += st
        return inputs, carried

    def unroll(self, length, inputs, begin_state=None, layout='NTC', merge_outputs=None):
        self.reset()
        states = begin_state if begin_state is not None else self.begin_state()
        carried = []
        depth = len(self._cells)
        for k, (child, st) in enumerate(zip(self._cells, self._per_child(states))):
            merge = merge_outputs if k == depth - 1 else None
            inputs, st = child.unroll(length, inputs=inputs, begin_state=st, layout=layout, merge_outputs=merge)
            carried += st
        return inputs, carried


class DropoutCell(BaseRNNCell):
    """Dropout on the step input (stateless)."""

    def __init__(self, dropout, prefix='dropout_', params=None):
        super().__init__(prefix, params)
        if not isinstance(dropout, numeric_types):
            raise AssertionError('dropout probability must be a number')
        self.dropout = dropout

    @property
    def state_info(self):
        return []

    def __call__(self, inputs, states):
        return (symbol.Dropout(data=inputs, p=self.dropout) if self.dropout > 0 else inputs), states

    def unroll(self, length, inputs, begin_state=None, layout='NTC', merge_outputs=None):
        self.reset()
        seq, _ = _time_major_split(length, inputs, layout, merge_outputs)
        if not isinstance(seq, symbol.Symbol):
            return super().unroll(length, seq, begin_state=begin_state, layout=layout, merge_outputs=merge_outputs)
        return self(seq, [])


class ModifierCell(BaseRNNCell):
    """Base of cells that wrap another cell and change its behaviour."""

    def __init__(self, base_cell):
        super().__init__()
        self.base_cell = base_cell
        base_cell._modified = True

    @property
    def params(self):
        self._owns_params = False
        return self.base_cell.params

    @property
    def state_info(self):
        return self.base_cell.state_info

    def _run_unwrapped(self, fn, *args, **kwargs):
        """Call ``fn`` of the base cell with its 'modified' guard lifted."""
        self.base_cell._modified = False
        try:
            return fn(*args, **kwargs)
        finally:
            self.base_cell._modified = True

    def begin_state(self, init_sym=symbol.zeros, **kwargs):
        self._check_unmodified()
        return self._run_unwrapped(self.base_cell.begin_state, func=init_sym, **kwargs)

    def unpack_weights(self, args):
        return self.base_cell.unpack_weights(args)

    def pack_weights(self, args):
        return self.base_cell.pack_weights(args)

    def __call__(self, inputs, states):
        raise NotImplementedError


class ZoneoutCell(ModifierCell):
    """Zoneout (Krueger et al. 2016): randomly keep previous outputs / states."""

    def __init__(self, base_cell, zoneout_outputs=0., zoneout_states=0.):
        for bad, why in ((FusedRNNCell, 'FusedRNNCell does not support zoneout; unfuse() it first'),
                         (BidirectionalCell, 'BidirectionalCell does not support zoneout; apply it to the inner '
                                             'cells')):
            if isinstance(base_cell, bad):
                raise AssertionError(why)
        super().__init__(base_cell)
        self.zoneout_outputs = zoneout_outputs
        self.zoneout_states = zoneout_states
        self.prev_output = None

    def reset(self):
        super().reset()
        self.prev_output = None

    @staticmethod
    def _keep(p, new, old):
        """Element-wise: ``new`` where a dropout mask of rate ``p`` is set, else ``old``."""
        return symbol.where(symbol.Dropout(symbol.ones_like(new), p=p), new, old)

    def __call__(self, inputs, states):
        y, new_states = self.base_cell(inputs, states)
        if self.zoneout_outputs != 0.:
            last = symbol.zeros_like(y) if self.prev_output is None else self.prev_output
            y = self._keep(self.zoneout_outputs, y, last)
        if self.zoneout_states != 0.:
            new_states = [self._keep(self.zoneout_states, n, o) for n, o in zip(new_states, states)]
        self.prev_output = y
        return y, new_states


class ResidualCell(ModifierCell):
    """Adds the step input to the wrapped cell's output (He et al. 2016 style)."""

    def __call__(self, inputs, states):
        y, states = self.base_cell(inputs, states)
        return symbol.elemwise_add(y, inputs, name='%s_plus_residual' % y.name), states

    def unroll(self, length, inputs, begin_state=None, layout='NTC', merge_outputs=None):
        self.reset()
        ys, states = self._run_unwrapped(self.base_cell.unroll, length, inputs=inputs, begin_state=begin_state,
                                         layout=layout, merge_outputs=merge_outputs)
        merged = isinstance(ys, symbol.Symbol) if merge_outputs is None else merge_outputs
        xs, _ = _time_major_split(length, inputs, layout, merged)
        if merged:
            return symbol.elemwise_add(ys, xs), states
        return [symbol.elemwise_add(y, x) for y, x in zip(ys, xs)], states


class BidirectionalCell(_Container):
    """Runs ``l_cell`` forward and ``r_cell`` backward in time and concatenates their outputs."""

    def __init__(self, l_cell, r_cell, params=None, output_prefix='bi_'):
        super().__init__('', params=params)
        self._output_prefix = output_prefix
        self._adopt([l_cell, r_cell], params is not None)
        self._cells = [l_cell, r_cell]

    def __call__(self, inputs, states):
        raise NotImplementedError('BidirectionalCell cannot be stepped; use unroll')

    def unroll(self, length, inputs, begin_state=None, layout='NTC', merge_outputs=None):
        self.reset()
        steps, t_axis = _time_major_split(length, inputs, layout, False)
        states = begin_state if begin_state is not None else self.begin_state()
        fwd_cell, bwd_cell = self._cells
        split = len(fwd_cell.state_info)
        fwd, fwd_states = fwd_cell.unroll(length, inputs=steps, begin_state=states[:split], layout=layout,
                                          merge_outputs=merge_outputs)
        bwd, bwd_states = bwd_cell.unroll(length, inputs=steps[::-1], begin_state=states[split:], layout=layout,
                                          merge_outputs=merge_outputs)
        if merge_outputs is None:
            merge_outputs = isinstance(fwd, symbol.Symbol) and isinstance(bwd, symbol.Symbol)
            fwd, _ = _time_major_split(None, fwd, layout, merge_outputs)
            bwd, _ = _time_major_split(None, bwd, layout, merge_outputs)
        if merge_outputs:
            outs = symbol.Concat(fwd, symbol.reverse(bwd, axis=t_axis), dim=2, name=self._output_prefix + 'out')
        else:
            outs = [symbol.Concat(f, b, dim=1, name='%st%d' % (self._output_prefix, t))
                    for t, (f, b) in enumerate(zip(fwd, bwd[::-1]))]
        return outs, fwd_states + bwd_states


class BaseConvRNNCell(BaseRNNCell):
    """Convolutional recurrent cells (Shi et al. 2015): i2h / h2h are convolutions."""

    def __init__(self, input_shape, num_hidden, h2h_kernel, h2h_dilate, i2h_kernel, i2h_stride, i2h_pad,
                 i2h_dilate, activation, prefix='', params=None, conv_layout='NCHW'):
        super().__init__(prefix=prefix, params=params)
        if h2h_kernel[0] % 2 != 1 or h2h_kernel[1] % 2 != 1:
            raise AssertionError('only odd h2h kernel sizes are supported, got %s' % (h2h_kernel,))
        self._h2h_kernel = h2h_kernel
        self._h2h_dilate = h2h_dilate
        self._h2h_pad = (h2h_dilate[0] * (h2h_kernel[0] - 1) // 2, h2h_dilate[1] * (h2h_kernel[1] - 1) // 2)
        self._i2h_kernel, self._i2h_stride = i2h_kernel, i2h_stride
        self._i2h_pad, self._i2h_dilate = i2h_pad, i2h_dilate
        self._num_hidden = num_hidden
        self._input_shape = input_shape
        self._conv_layout = conv_layout
        self._activation = activation
        data = symbol.Variable('data')
        conv = symbol.Convolution(data=data, num_filter=num_hidden, kernel=i2h_kernel, stride=i2h_stride,
                                  pad=i2h_pad, dilate=i2h_dilate, layout=conv_layout)
        self._state_shape = conv.infer_shape(data=input_shape)[1][0]
        self._state_shape = (0,) + tuple(self._state_shape[1:])
        self._standard_params()

    @property
    def _num_gates(self):
        return len(self._GATES)

    @property
    def state_info(self):
        return [{'shape': self._state_shape, '__layout__': self._conv_layout}] * self._num_states

    _num_states = 1

    def _conv_forward(self, inputs, states, name):
        n = self._num_hidden * self._num_gates
        i2h = symbol.Convolution(name='%si2h' % name, data=inputs, num_filter=n, kernel=self._i2h_kernel,
                                 stride=self._i2h_stride, pad=self._i2h_pad, dilate=self._i2h_dilate,
                                 weight=self._iW, bias=self._iB, layout=self._conv_layout)
        h2h = symbol.Convolution(name='%sh2h' % name, data=states[0], num_filter=n, kernel=self._h2h_kernel,
                                 dilate=self._h2h_dilate, pad=self._h2h_pad, stride=(1, 1), weight=self._hW,
                                 bias=self._hB, layout=self._conv_layout)
        return i2h, h2h

    def __call__(self, inputs, states):
        raise NotImplementedError


class ConvRNNCell(BaseConvRNNCell):
    def __init__(self, input_shape, num_hidden, h2h_kernel=(3, 3), h2h_dilate=(1, 1), i2h_kernel=(3, 3),
                 i2h_stride=(1, 1), i2h_pad=(1, 1), i2h_dilate=(1, 1), activation='tanh', prefix='ConvRNN_',
                 params=None, conv_layout='NCHW'):
        super().__init__(input_shape, num_hidden, h2h_kernel, h2h_dilate, i2h_kernel, i2h_stride, i2h_pad,
                         i2h_dilate, activation, prefix, params, conv_layout)

    _GATES = ('',)

    def __call__(self, inputs, states):
        tag = self._step_name()
        i2h, h2h = self._conv_forward(inputs, states, tag)
        h = self._get_activation(i2h + h2h, self._activation, name=tag + 'out')
        return h, [h]


class ConvLSTMCell(BaseConvRNNCell):
    _num_states = 2

    def __init__(self, input_shape, num_hidden, h2h_kernel=(3, 3), h2h_dilate=(1, 1), i2h_kernel=(3, 3),
                 i2h_stride=(1, 1), i2h_pad=(1, 1), i2h_dilate=(1, 1), activation='tanh', prefix='ConvLSTM_',
                 params=None, forget_bias=1.0, conv_layout='NCHW'):
        super().__init__(input_shape, num_hidden, h2h_kernel, h2h_dilate, i2h_kernel, i2h_stride, i2h_pad,
                         i2h_dilate, activation, prefix, params, conv_layout)
        self._iB = self.params.get('i2h_bias', init=init.LSTMBias(forget_bias=forget_bias))

    _GATES = ('_i', '_f', '_c', '_o')

    def __call__(self, inputs, states):
        name = self._step_name()
        i2h, h2h = self._conv_forward(inputs, states, name)
        axis = self._conv_layout.find('C')
        g = symbol.SliceChannel(i2h + h2h, num_outputs=4, axis=axis, name=name + 'slice')
        i = symbol.Activation(g[0], act_type='sigmoid')
        f = symbol.Activation(g[1], act_type='sigmoid')
        c = self._get_activation(g[2], self._activation)
        o = symbol.Activation(g[3], act_type='sigmoid')
        next_c = symbol._internal._plus(f * states[1], i * c, name=name + 'state')
        next_h = symbol._internal._mul(o, self._get_activation(next_c, self._activation), name=name + 'out')
        return next_h, [next_h, next_c]


class ConvGRUCell(BaseConvRNNCell):
    def __init__(self, input_shape, num_hidden, h2h_kernel=(3, 3), h2h_dilate=(1, 1), i2h_kernel=(3, 3),
                 i2h_stride=(1, 1), i2h_pad=(1, 1), i2h_dilate=(1, 1), activation='tanh', prefix='ConvGRU_',
                 params=None, conv_layout='NCHW'):
        super().__init__(input_shape, num_hidden, h2h_kernel, h2h_dilate, i2h_kernel, i2h_stride, i2h_pad,
                         i2h_dilate, activation, prefix, params, conv_layout)

    _GATES = ('_r', '_z', '_o')

    def __call__(self, inputs, states):
        name = self._step_name()
        i2h, h2h = self._conv_forward(inputs, states, name)
        axis = self._conv_layout.find('C')
        i_r, i_z, i_n = symbol.SliceChannel(i2h, num_outputs=3, axis=axis, name=name + 'i2h_slice')
        h_r, h_z, h_n = symbol.SliceChannel(h2h, num_outputs=3, axis=axis, name=name + 'h2h_slice')
        r = symbol.Activation(i_r + h_r, act_type='sigmoid')
        z = symbol.Activation(i_z + h_z, act_type='sigmoid')
        n = self._get_activation(i_n + r * h_n, self._activation)
        next_h = symbol._internal._plus((1. - z) * n, z * states[0], name=name + 'out')
        return next_h, [next_h]
