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


def _cells_state_info(cells):
    return [info for c in cells for info in c.state_info]


def _cells_begin_state(cells, **kwargs):
    return [s for c in cells for s in c.begin_state(**kwargs)]


def _cells_unpack_weights(cells, args):
    for c in cells:
        args = c.unpack_weights(args)
    return args


def _cells_pack_weights(cells, args):
    for c in cells:
        args = c.pack_weights(args)
    return args


def _normalize_sequence(length, inputs, layout, merge, in_layout=None):
    """Inputs as either one merged Symbol (time along ``layout``'s T axis) or a list of ``length``
    per-step Symbols; returns (inputs, time_axis)."""
    if inputs is None:
        raise AssertionError('unroll(inputs=None) is not supported; pass the input symbol(s)')
    axis = layout.find('T')
    in_axis = in_layout.find('T') if in_layout is not None else axis
    if isinstance(inputs, symbol.Symbol):
        if merge is False:
            if len(inputs.list_outputs()) != 1:
                raise AssertionError('unroll needs a single-output input symbol or a list of symbols')
            inputs = list(symbol.split(inputs, axis=in_axis, num_outputs=length, squeeze_axis=1))
    else:
        if length is not None and len(inputs) != length:
            raise AssertionError('unroll length %s but %d input steps' % (length, len(inputs)))
        if merge is True:
            inputs = symbol.Concat(*[symbol.expand_dims(i, axis=axis) for i in inputs], dim=axis)
            in_axis = axis
    if isinstance(inputs, symbol.Symbol) and axis != in_axis:
        inputs = symbol.swapaxes(inputs, dim0=axis, dim1=in_axis)
    return inputs, axis


class RNNParams:
    """Container of the Variables of a cell (shared between cells given the same instance)."""

    def __init__(self, prefix=''):
        self._prefix = prefix
        self._params = {}

    def get(self, name, **kwargs):
        """The Variable ``<prefix><name>`` (created on first request with ``kwargs``)."""
        full = self._prefix + name
        if full not in self._params:
            self._params[full] = symbol.Variable(full, **kwargs)
        return self._params[full]


class BaseRNNCell:
    """Abstract cell: subclasses implement ``state_info`` and ``__call__``."""

    def __init__(self, prefix='', params=None):
        if params is None:
            params = RNNParams(prefix)
            self._own_params = True
        else:
            self._own_params = False
        self._prefix = prefix
        self._params = params
        self._modified = False
        self.reset()

    def reset(self):
        """Forget the time-step counters (call before building a new graph)."""
        self._init_counter = -1
        self._counter = -1
        if hasattr(self, '_cells'):
            for c in self._cells:
                c.reset()

    def __call__(self, inputs, states):
        raise NotImplementedError

    @property
    def params(self):
        self._own_params = False
        return self._params

    @property
    def state_info(self):
        raise NotImplementedError

    @property
    def state_shape(self):
        return [info['shape'] for info in self.state_info]

    @property
    def _gate_names(self):
        return ()

    def begin_state(self, func=symbol.zeros, **kwargs):
        """Initial states (zeros by default; batch dimension 0 = inferred at bind time)."""
        if self._modified:
            raise AssertionError('after applying a modifier cell (e.g. ZoneoutCell) the base cell '
                                 'cannot be called directly; call the modifier cell instead')
        states = []
        for info in self.state_info:
            self._init_counter += 1
            name = '%sbegin_state_%d' % (self._prefix, self._init_counter)
            kw = dict(kwargs)
            if info is not None:
                kw.update(info)
            states.append(func(name=name, **kw))
        return states

    # ---------------------------------------------------------------- (un)packing
    def unpack_weights(self, args):
        """Split fused gate weights/biases in ``args`` into per-gate entries."""
        args = dict(args)
        if not self._gate_names:
            return args
        h = self._num_hidden
        for group in ('i2h', 'h2h'):
            w = args.pop('%s%s_weight' % (self._prefix, group))
            b = args.pop('%s%s_bias' % (self._prefix, group))
            for j, gate in enumerate(self._gate_names):
                args['%s%s%s_weight' % (self._prefix, group, gate)] = w[j * h:(j + 1) * h].copy()
                args['%s%s%s_bias' % (self._prefix, group, gate)] = b[j * h:(j + 1) * h].copy()
        return args

    def pack_weights(self, args):
        """Inverse of ``unpack_weights``."""
        from .. import ndarray as nd
        args = dict(args)
        if not self._gate_names:
            return args
        for group in ('i2h', 'h2h'):
            for kind in ('weight', 'bias'):
                parts = [args.pop('%s%s%s_%s' % (self._prefix, group, gate, kind)) for gate in self._gate_names]
                args['%s%s_%s' % (self._prefix, group, kind)] = nd.concat(*parts, dim=0)
        return args

    # ---------------------------------------------------------------- unrolling
    def unroll(self, length, inputs, begin_state=None, layout='NTC', merge_outputs=None):
        """Apply the cell ``length`` times; returns (outputs, states)."""
        self.reset()
        inputs, _ = _normalize_sequence(length, inputs, layout, False)
        states = self.begin_state() if begin_state is None else begin_state
        outputs = []
        for t in range(length):
            out, states = self(inputs[t], states)
            outputs.append(out)
        outputs, _ = _normalize_sequence(length, outputs, layout, merge_outputs)
        return outputs, states

    def _get_activation(self, inputs, activation, **kwargs):
        if isinstance(activation, string_types):
            return symbol.Activation(inputs, act_type=activation, **kwargs)
        return activation(inputs, **kwargs)

    def _fc_pair(self, inputs, prev_h, gates, name):
        """i2h(inputs) and h2h(prev_h) projections for ``gates`` fused gates."""
        n = gates * self._num_hidden
        i2h = symbol.FullyConnected(data=inputs, weight=self._iW, bias=self._iB, num_hidden=n, name=name + 'i2h')
        h2h = symbol.FullyConnected(data=prev_h, weight=self._hW, bias=self._hB, num_hidden=n, name=name + 'h2h')
        return i2h, h2h

    def _step_name(self):
        self._counter += 1
        return '%st%d_' % (self._prefix, self._counter)


class RNNCell(BaseRNNCell):
    """Elman cell: h' = act(W_i x + b_i + W_h h + b_h)."""

    def __init__(self, num_hidden, activation='tanh', prefix='rnn_', params=None):
        super().__init__(prefix=prefix, params=params)
        self._num_hidden = num_hidden
        self._activation = activation
        self._iW = self.params.get('i2h_weight')
        self._iB = self.params.get('i2h_bias')
        self._hW = self.params.get('h2h_weight')
        self._hB = self.params.get('h2h_bias')

    @property
    def state_info(self):
        return [{'shape': (0, self._num_hidden), '__layout__': 'NC'}]

    @property
    def _gate_names(self):
        return ('',)

    def __call__(self, inputs, states):
        name = self._step_name()
        i2h, h2h = self._fc_pair(inputs, states[0], 1, name)
        out = self._get_activation(i2h + h2h, self._activation, name=name + 'out')
        return out, [out]


class LSTMCell(BaseRNNCell):
    """Long short-term memory cell; ``forget_bias`` initialises the forget-gate bias."""

    def __init__(self, num_hidden, prefix='lstm_', params=None, forget_bias=1.0):
        super().__init__(prefix=prefix, params=params)
        self._num_hidden = num_hidden
        self._iW = self.params.get('i2h_weight')
        self._hW = self.params.get('h2h_weight')
        self._iB = self.params.get('i2h_bias', init=init.LSTMBias(forget_bias=forget_bias))
        self._hB = self.params.get('h2h_bias')

    @property
    def state_info(self):
        return [{'shape': (0, self._num_hidden), '__layout__': 'NC'},
                {'shape': (0, self._num_hidden), '__layout__': 'NC'}]

    @property
    def _gate_names(self):
        return ('_i', '_f', '_c', '_o')

    def __call__(self, inputs, states):
        name = self._step_name()
        i2h, h2h = self._fc_pair(inputs, states[0], 4, name)
        gates = symbol.SliceChannel(i2h + h2h, num_outputs=4, name=name + 'slice')
        in_gate = symbol.Activation(gates[0], act_type='sigmoid', name=name + 'i')
        forget_gate = symbol.Activation(gates[1], act_type='sigmoid', name=name + 'f')
        in_transform = symbol.Activation(gates[2], act_type='tanh', name=name + 'c')
        out_gate = symbol.Activation(gates[3], act_type='sigmoid', name=name + 'o')
        next_c = symbol._internal._plus(forget_gate * states[1], in_gate * in_transform, name=name + 'state')
        next_h = symbol._internal._mul(out_gate, symbol.Activation(next_c, act_type='tanh'), name=name + 'out')
        return next_h, [next_h, next_c]


class GRUCell(BaseRNNCell):
    """Gated recurrent unit (Cho et al. 2014), cuDNN / fused-op variant."""

    def __init__(self, num_hidden, prefix='gru_', params=None):
        super().__init__(prefix=prefix, params=params)
        self._num_hidden = num_hidden
        self._iW = self.params.get('i2h_weight')
        self._iB = self.params.get('i2h_bias')
        self._hW = self.params.get('h2h_weight')
        self._hB = self.params.get('h2h_bias')

    @property
    def state_info(self):
        return [{'shape': (0, self._num_hidden), '__layout__': 'NC'}]

    @property
    def _gate_names(self):
        return ('_r', '_z', '_o')

    def __call__(self, inputs, states):
        name = self._step_name()
        prev_h = states[0]
        i2h, h2h = self._fc_pair(inputs, prev_h, 3, name)
        i_r, i_z, i_n = symbol.SliceChannel(i2h, num_outputs=3, name=name + 'i2h_slice')
        h_r, h_z, h_n = symbol.SliceChannel(h2h, num_outputs=3, name=name + 'h2h_slice')
        reset = symbol.Activation(i_r + h_r, act_type='sigmoid', name=name + 'r_act')
        update = symbol.Activation(i_z + h_z, act_type='sigmoid', name=name + 'z_act')
        cand = symbol.Activation(i_n + reset * h_n, act_type='tanh', name=name + 'h_act')
        next_h = symbol._internal._plus((1. - update) * cand, update * prev_h, name=name + 'out')
        return next_h, [next_h]


class FusedRNNCell(BaseRNNCell):
    """Multi-layer (bi)directional RNN on the fused ``RNN`` operator (one flat parameter Variable)."""

    _GATES = {'rnn_relu': ('',), 'rnn_tanh': ('',), 'lstm': ('_i', '_f', '_c', '_o'), 'gru': ('_r', '_z', '_o')}

    def __init__(self, num_hidden, num_layers=1, mode='lstm', bidirectional=False, dropout=0., get_next_state=False,
                 forget_bias=1.0, prefix=None, params=None):
        if prefix is None:
            prefix = '%s_' % mode
        super().__init__(prefix=prefix, params=params)
        self._num_hidden = num_hidden
        self._num_layers = num_layers
        self._mode = mode
        self._bidirectional = bidirectional
        self._dropout = dropout
        self._get_next_state = get_next_state
        self._directions = ['l', 'r'] if bidirectional else ['l']
        initializer = init.FusedRNN(None, num_hidden, num_layers, mode, bidirectional, forget_bias)
        self._parameter = self.params.get('parameters', init=initializer)

    @property
    def state_info(self):
        b = len(self._directions)
        n = 2 if self._mode == 'lstm' else 1
        return [{'shape': (b * self._num_layers, 0, self._num_hidden), '__layout__': 'LNC'}] * n

    @property
    def _gate_names(self):
        return self._GATES[self._mode]

    @property
    def _num_gates(self):
        return len(self._gate_names)

    def _slice_weights(self, arr, li, lh):
        """Views of the per-(layer, direction, gate) pieces of the flat parameter array ``arr``
        (``li``: input size of layer 0, ``lh``: hidden size), keyed by unfused names."""
        out = {}
        g = self._num_gates
        h = self._num_hidden
        pos = 0
        for layer in range(self._num_layers):
            for d in self._directions:
                width = li if layer == 0 else lh * len(self._directions)
                for group, cols in (('i2h', width), ('h2h', lh)):
                    for gate in self._gate_names:
                        name = '%s%s%d_%s%s_weight' % (self._prefix, d, layer, group, gate)
                        out[name] = arr[pos:pos + h * cols].reshape((h, cols))
                        pos += h * cols
        for layer in range(self._num_layers):
            for d in self._directions:
                for group in ('i2h', 'h2h'):
                    for gate in self._gate_names:
                        out['%s%s%d_%s%s_bias' % (self._prefix, d, layer, group, gate)] = arr[pos:pos + h]
                        pos += h
        if pos != arr.size:
            raise AssertionError('parameter vector of %d elements, expected %d' % (arr.size, pos))
        return out

    def _input_size(self, total):
        """Layer-0 input size implied by a flat parameter count."""
        g, h, d, L = self._num_gates, self._num_hidden, len(self._directions), self._num_layers
        rest = (L - 1) * d * g * h * (h * d + h + 2) + d * g * h * (h + 2)
        return (total - rest) // (d * g * h)

    def unpack_weights(self, args):
        args = dict(args)
        arr = args.pop(self._parameter.name)
        li = self._input_size(arr.size)
        for k, v in self._slice_weights(arr, li, self._num_hidden).items():
            args[k] = v.copy()
        return args

    def pack_weights(self, args):
        from .. import ndarray as nd
        args = dict(args)
        w0 = args['%sl0_i2h%s_weight' % (self._prefix, self._gate_names[0])]
        li = w0.shape[1]
        total = self._num_gates * self._num_hidden * len(self._directions) * (
            li + self._num_hidden + 2) + (self._num_layers - 1) * len(self._directions) * self._num_gates * \
            self._num_hidden * (self._num_hidden * len(self._directions) + self._num_hidden + 2)
        arr = nd.zeros((total,), ctx=w0.context, dtype=w0.dtype)
        for k, v in self._slice_weights(arr, li, self._num_hidden).items():
            v[:] = args.pop(k).reshape(v.shape)
        args[self._parameter.name] = arr
        return args

    def __call__(self, inputs, states):
        raise NotImplementedError('FusedRNNCell cannot be stepped; use unroll')

    def unroll(self, length, inputs, begin_state=None, layout='NTC', merge_outputs=None):
        self.reset()
        inputs, axis = _normalize_sequence(length, inputs, layout, True)
        if axis == 1:
            warnings.warn('NTC layout detected: FusedRNNCell runs in TNC, inputs are transposed')
            inputs = symbol.swapaxes(inputs, dim0=0, dim1=1)
        states = self.begin_state() if begin_state is None else begin_state
        kw = {'state_cell': states[1]} if self._mode == 'lstm' else {}
        rnn = symbol.RNN(data=inputs, parameters=self._parameter, state=states[0], state_size=self._num_hidden,
                         num_layers=self._num_layers, bidirectional=self._bidirectional, p=self._dropout,
                         state_outputs=self._get_next_state, mode=self._mode, name=self._prefix + 'rnn', **kw)
        if not self._get_next_state:
            outputs, states = rnn, []
        elif self._mode == 'lstm':
            outputs, states = rnn[0], [rnn[1], rnn[2]]
        else:
            outputs, states = rnn[0], [rnn[1]]
        if axis == 1:
            outputs = symbol.swapaxes(outputs, dim0=0, dim1=1)
        outputs, _ = _normalize_sequence(length, outputs, layout, merge_outputs)
        return outputs, states

    def unfuse(self):
        """An equivalent ``SequentialRNNCell`` of unfused cells (weights via unpack_weights)."""
        make = {'rnn_relu': lambda p: RNNCell(self._num_hidden, activation='relu', prefix=p),
                'rnn_tanh': lambda p: RNNCell(self._num_hidden, activation='tanh', prefix=p),
                'lstm': lambda p: LSTMCell(self._num_hidden, prefix=p),
                'gru': lambda p: GRUCell(self._num_hidden, prefix=p)}[self._mode]
        stack = SequentialRNNCell()
        for i in range(self._num_layers):
            if self._bidirectional:
                stack.add(BidirectionalCell(make('%sl%d_' % (self._prefix, i)), make('%sr%d_' % (self._prefix, i)),
                                            output_prefix='%sbi_l%d_' % (self._prefix, i)))
            else:
                stack.add(make('%sl%d_' % (self._prefix, i)))
            if self._dropout > 0 and i != self._num_layers - 1:
                stack.add(DropoutCell(self._dropout, prefix='%s_dropout%d_' % (self._prefix, i)))
        return stack


class SequentialRNNCell(BaseRNNCell):
    """Stack of cells: the output of cell i is the input of cell i+1."""

    def __init__(self, params=None):
        super().__init__(prefix='', params=params)
        self._override_cell_params = params is not None
        self._cells = []

    def add(self, cell):
        self._cells.append(cell)
        if self._override_cell_params:
            if not cell._own_params:
                raise AssertionError('with params given to SequentialRNNCell, child cells must own theirs')
            cell.params._params.update(self.params._params)
        self.params._params.update(cell.params._params)

    @property
    def state_info(self):
        return _cells_state_info(self._cells)

    def begin_state(self, **kwargs):
        if self._modified:
            raise AssertionError('modified cell: call the modifier instead')
        return _cells_begin_state(self._cells, **kwargs)

    def unpack_weights(self, args):
        return _cells_unpack_weights(self._cells, args)

    def pack_weights(self, args):
        return _cells_pack_weights(self._cells, args)

    def _split_states(self, states):
        out, p = [], 0
        for c in self._cells:
            n = len(c.state_info)
            out.append(states[p:p + n])
            p += n
        return out

    def __call__(self, inputs, states):
        self._counter += 1
        new_states = []
        for cell, st in zip(self._cells, self._split_states(states)):
            if isinstance(cell, BidirectionalCell):
                raise AssertionError('BidirectionalCell cannot be stepped; unroll the stack instead')
            inputs, st = cell(inputs, st)
            new_states.extend(st)
        return inputs, new_states

    def unroll(self, length, inputs, begin_state=None, layout='NTC', merge_outputs=None):
        self.reset()
        states = self.begin_state() if begin_state is None else begin_state
        new_states = []
        last = len(self._cells) - 1
        for i, (cell, st) in enumerate(zip(self._cells, self._split_states(states))):
            inputs, st = cell.unroll(length, inputs=inputs, begin_state=st, layout=layout,
                                     merge_outputs=None if i < last else merge_outputs)
            new_states.extend(st)
        return inputs, new_states


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
        if self.dropout > 0:
            inputs = symbol.Dropout(data=inputs, p=self.dropout)
        return inputs, states

    def unroll(self, length, inputs, begin_state=None, layout='NTC', merge_outputs=None):
        self.reset()
        inputs, _ = _normalize_sequence(length, inputs, layout, merge_outputs)
        if isinstance(inputs, symbol.Symbol):
            return self(inputs, [])
        return super().unroll(length, inputs, begin_state=begin_state, layout=layout, merge_outputs=merge_outputs)


class ModifierCell(BaseRNNCell):
    """Base of cells that wrap another cell and change its behaviour."""

    def __init__(self, base_cell):
        super().__init__()
        base_cell._modified = True
        self.base_cell = base_cell

    @property
    def params(self):
        self._own_params = False
        return self.base_cell.params

    @property
    def state_info(self):
        return self.base_cell.state_info

    def begin_state(self, init_sym=symbol.zeros, **kwargs):
        if self._modified:
            raise AssertionError('modified cell: call the outer modifier instead')
        self.base_cell._modified = False
        try:
            return self.base_cell.begin_state(func=init_sym, **kwargs)
        finally:
            self.base_cell._modified = True

    def unpack_weights(self, args):
        return self.base_cell.unpack_weights(args)

    def pack_weights(self, args):
        return self.base_cell.pack_weights(args)

    def __call__(self, inputs, states):
        raise NotImplementedError


class ZoneoutCell(ModifierCell):
    """Zoneout (Krueger et al. 2016): randomly keep previous outputs / states."""

    def __init__(self, base_cell, zoneout_outputs=0., zoneout_states=0.):
        if isinstance(base_cell, FusedRNNCell):
            raise AssertionError('FusedRNNCell does not support zoneout; unfuse() it first')
        if isinstance(base_cell, BidirectionalCell):
            raise AssertionError('BidirectionalCell does not support zoneout; apply it to the inner cells')
        super().__init__(base_cell)
        self.zoneout_outputs = zoneout_outputs
        self.zoneout_states = zoneout_states
        self.prev_output = None

    def reset(self):
        super().reset()
        self.prev_output = None

    def __call__(self, inputs, states):
        cell = self.base_cell
        next_output, next_states = cell(inputs, states)
        mask = lambda p, like: symbol.Dropout(symbol.ones_like(like), p=p)   # noqa: E731
        prev = self.prev_output if self.prev_output is not None else symbol.zeros_like(next_output)
        out = symbol.where(mask(self.zoneout_outputs, next_output), next_output, prev) \
            if self.zoneout_outputs != 0. else next_output
        if self.zoneout_states != 0.:
            next_states = [symbol.where(mask(self.zoneout_states, n), n, o) for n, o in zip(next_states, states)]
        self.prev_output = out
        return out, next_states


class ResidualCell(ModifierCell):
    """Adds the step input to the wrapped cell's output (He et al. 2016 style)."""

    def __call__(self, inputs, states):
        out, states = self.base_cell(inputs, states)
        return symbol.elemwise_add(out, inputs, name='%s_plus_residual' % out.name), states

    def unroll(self, length, inputs, begin_state=None, layout='NTC', merge_outputs=None):
        self.reset()
        self.base_cell._modified = False
        outputs, states = self.base_cell.unroll(length, inputs=inputs, begin_state=begin_state, layout=layout,
                                                merge_outputs=merge_outputs)
        self.base_cell._modified = True
        merge = isinstance(outputs, symbol.Symbol) if merge_outputs is None else merge_outputs
        inputs, _ = _normalize_sequence(length, inputs, layout, merge)
        if merge:
            outputs = symbol.elemwise_add(outputs, inputs)
        else:
            outputs = [symbol.elemwise_add(o, i) for o, i in zip(outputs, inputs)]
        return outputs, states


class BidirectionalCell(BaseRNNCell):
    """Runs ``l_cell`` forward and ``r_cell`` backward in time and concatenates their outputs."""

    def __init__(self, l_cell, r_cell, params=None, output_prefix='bi_'):
        super().__init__('', params=params)
        self._output_prefix = output_prefix
        self._override_cell_params = params is not None
        if self._override_cell_params:
            if not (l_cell._own_params and r_cell._own_params):
                raise AssertionError('with params given, the inner cells must own theirs')
            l_cell.params._params.update(self.params._params)
            r_cell.params._params.update(self.params._params)
        self.params._params.update(l_cell.params._params)
        self.params._params.update(r_cell.params._params)
        self._cells = [l_cell, r_cell]

    def unpack_weights(self, args):
        return _cells_unpack_weights(self._cells, args)

    def pack_weights(self, args):
        return _cells_pack_weights(self._cells, args)

    def __call__(self, inputs, states):
        raise NotImplementedError('BidirectionalCell cannot be stepped; use unroll')

    @property
    def state_info(self):
        return _cells_state_info(self._cells)

    def begin_state(self, **kwargs):
        if self._modified:
            raise AssertionError('modified cell: call the modifier instead')
        return _cells_begin_state(self._cells, **kwargs)

    def unroll(self, length, inputs, begin_state=None, layout='NTC', merge_outputs=None):
        self.reset()
        inputs, axis = _normalize_sequence(length, inputs, layout, False)
        states = self.begin_state() if begin_state is None else begin_state
        l_cell, r_cell = self._cells
        nl = len(l_cell.state_info)
        l_out, l_states = l_cell.unroll(length, inputs=inputs, begin_state=states[:nl], layout=layout,
                                        merge_outputs=merge_outputs)
        r_out, r_states = r_cell.unroll(length, inputs=list(reversed(inputs)), begin_state=states[nl:],
                                        layout=layout, merge_outputs=merge_outputs)
        if merge_outputs is None:
            merge_outputs = isinstance(l_out, symbol.Symbol) and isinstance(r_out, symbol.Symbol)
            l_out, _ = _normalize_sequence(None, l_out, layout, merge_outputs)
            r_out, _ = _normalize_sequence(None, r_out, layout, merge_outputs)
        if merge_outputs:
            r_out = symbol.reverse(r_out, axis=axis)
            outputs = symbol.Concat(l_out, r_out, dim=2, name='%sout' % self._output_prefix)
        else:
            outputs = [symbol.Concat(l, r, dim=1, name='%st%d' % (self._output_prefix, i))
                       for i, (l, r) in enumerate(zip(l_out, reversed(r_out)))]
        return outputs, l_states + r_states


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
        self._iW = self.params.get('i2h_weight')
        self._hW = self.params.get('h2h_weight')
        self._iB = self.params.get('i2h_bias')
        self._hB = self.params.get('h2h_bias')

    @property
    def _num_gates(self):
        return len(self._gate_names)

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

    @property
    def _gate_names(self):
        return ('',)

    def __call__(self, inputs, states):
        name = self._step_name()
        i2h, h2h = self._conv_forward(inputs, states, name)
        out = self._get_activation(i2h + h2h, self._activation, name=name + 'out')
        return out, [out]


class ConvLSTMCell(BaseConvRNNCell):
    _num_states = 2

    def __init__(self, input_shape, num_hidden, h2h_kernel=(3, 3), h2h_dilate=(1, 1), i2h_kernel=(3, 3),
                 i2h_stride=(1, 1), i2h_pad=(1, 1), i2h_dilate=(1, 1), activation='tanh', prefix='ConvLSTM_',
                 params=None, forget_bias=1.0, conv_layout='NCHW'):
        super().__init__(input_shape, num_hidden, h2h_kernel, h2h_dilate, i2h_kernel, i2h_stride, i2h_pad,
                         i2h_dilate, activation, prefix, params, conv_layout)
        self._iB = self.params.get('i2h_bias', init=init.LSTMBias(forget_bias=forget_bias))

    @property
    def _gate_names(self):
        return ('_i', '_f', '_c', '_o')

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

    @property
    def _gate_names(self):
        return ('_r', '_z', '_o')

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
