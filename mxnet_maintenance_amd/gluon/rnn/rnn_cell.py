"""Recurrent cells (parity: python/mxnet/gluon/rnn/rnn_cell.py).

A cell computes one time step ``(output, new_states) = cell(input, states)``;
``unroll`` applies it over a sequence (NTC/TNC, optional ``valid_length``
masking).  The fused multi-layer path lives in rnn_layer.py (RNN op); cells
are for custom recurrences, decoders and the unfused reference semantics.
"""
from ... import ndarray, symbol
from ...ndarray.ndarray import NDArray
from ...symbol.symbol import Symbol
from ..block import Block, HybridBlock
from ..utils import _indent

__all__ = ['RecurrentCell', 'HybridRecurrentCell', 'RNNCell', 'LSTMCell', 'GRUCell', 'SequentialRNNCell',
           'HybridSequentialRNNCell', 'DropoutCell', 'ModifierCell', 'ZoneoutCell', 'ResidualCell',
           'BidirectionalCell', 'LSTMPCell', 'VariationalDropoutCell']

tensor_types = (Symbol, NDArray)


def _as_list(x):
    return list(x) if isinstance(x, (list, tuple)) else [x]


def _cells_state_info(cells, batch_size):
    return sum([c.state_info(batch_size) for c in cells], [])


def _cells_begin_state(cells, **kwargs):
    return sum([c.begin_state(**kwargs) for c in cells], [])


def _get_begin_state(cell, F, begin_state, inputs, batch_size):
    if begin_state is None:
        if F is ndarray:
            ctx = inputs.context if isinstance(inputs, tensor_types) else inputs[0].context
            begin_state = cell.begin_state(func=F.zeros, batch_size=batch_size, ctx=ctx)
        else:
            begin_state = cell.begin_state(func=F.zeros, batch_size=batch_size)
    return begin_state


def _format_sequence(length, inputs, layout, merge, in_layout=None):
    """Normalise ``inputs`` to a list of per-step tensors (merge False) or one tensor (merge True)."""
    assert inputs is not None, 'unroll(inputs=None) has been deprecated.'
    axis = layout.find('T')
    batch_axis = layout.find('N')
    batch_size = 0
    in_axis = in_layout.find('T') if in_layout is not None else axis
    if isinstance(inputs, Symbol):
        F = symbol
        if merge is False:
            inputs = list(symbol.split(inputs, axis=in_axis, num_outputs=length, squeeze_axis=1))
    elif isinstance(inputs, NDArray):
        F = ndarray
        batch_size = inputs.shape[batch_axis]
        if merge is False:
            assert length is None or length == inputs.shape[in_axis]
            inputs = _as_list(ndarray.split(inputs, axis=in_axis, num_outputs=inputs.shape[in_axis],
                                            squeeze_axis=1))
    else:
        assert length is None or len(inputs) == length
        if isinstance(inputs[0], Symbol):
            F = symbol
        else:
            F = ndarray
            batch_size = inputs[0].shape[0]
        if merge is True:
            inputs = F.stack(*inputs, axis=axis)
            in_axis = axis
    if isinstance(inputs, tensor_types) and axis != in_axis:
        inputs = F.swapaxes(inputs, dim1=axis, dim2=in_axis)
    return inputs, axis, F, batch_size


def _mask_sequence_variable_length(F, data, length, valid_length, time_axis, merge):
    assert valid_length is not None
    if not isinstance(data, tensor_types):
        data = F.stack(*data, axis=time_axis)
    outputs = F.SequenceMask(data, sequence_length=valid_length, use_sequence_length=True, axis=time_axis)
    if not merge:
        outputs = _as_list(F.split(outputs, num_outputs=length, axis=time_axis, squeeze_axis=True))
    return outputs


def _reverse_sequences(sequences, unroll_step, valid_length=None):
    F = symbol if isinstance(sequences[0], Symbol) else ndarray
    if valid_length is None:
        return list(reversed(sequences))
    rev = F.SequenceReverse(F.stack(*sequences, axis=0), sequence_length=valid_length, use_sequence_length=True)
    if unroll_step > 1 or F is symbol:
        return _as_list(F.split(rev, axis=0, num_outputs=unroll_step, squeeze_axis=True))
    return [rev[0]]


class RecurrentCell(Block):
    """Abstract base class for RNN cells."""

    def __init__(self, prefix=None, params=None):
        super().__init__(prefix=prefix, params=params)
        self._modified = False
        self.reset()

    def reset(self):
        self._init_counter = -1
        self._counter = -1
        for cell in self._children.values():
            cell.reset()

    def state_info(self, batch_size=0):
        raise NotImplementedError()

    def begin_state(self, batch_size=0, func=ndarray.zeros, **kwargs):
        assert not self._modified, \
            'After applying modifier cells (e.g. ZoneoutCell) the base cell cannot be called directly. ' \
            'Call the modifier cell instead.'
        states = []
        for info in self.state_info(batch_size):
            self._init_counter += 1
            if info is not None:
                info = dict(info)
                info.update(kwargs)
            else:
                info = dict(kwargs)
            info.pop('__layout__', None)
            if 'symbol' in getattr(func, '__module__', ''):
                info.pop('ctx', None)
            state = func(name='%sbegin_state_%d' % (self._prefix, self._init_counter), **info)
            states.append(state)
        return states

    def unroll(self, length, inputs, begin_state=None, layout='NTC', merge_outputs=None, valid_length=None):
        self.reset()
        inputs, axis, F, batch_size = _format_sequence(length, inputs, layout, False)
        begin_state = _get_begin_state(self, F, begin_state, inputs, batch_size)
        states = begin_state
        outputs = []
        all_states = []
        for i in range(length):
            output, states = self(inputs[i], states)
            outputs.append(output)
            if valid_length is not None:
                all_states.append(states)
        if valid_length is not None:
            states = [F.SequenceLast(F.stack(*ele_list, axis=0), sequence_length=valid_length,
                                     use_sequence_length=True, axis=0) for ele_list in zip(*all_states)]
            outputs = _mask_sequence_variable_length(F, outputs, length, valid_length, axis, True)
            if not merge_outputs:
                outputs = _as_list(F.split(outputs, num_outputs=length, axis=axis, squeeze_axis=True))
            return outputs, states
        outputs, _, _, _ = _format_sequence(length, outputs, layout, merge_outputs)
        return outputs, states

    def _get_activation(self, F, inputs, activation, **kwargs):
        func = {'tanh': F.tanh, 'relu': F.relu, 'sigmoid': F.sigmoid, 'softsign': F.softsign}.get(activation)
        if func:
            return func(inputs, **kwargs)
        if isinstance(activation, str):
            return F.Activation(inputs, act_type=activation, **kwargs)
        if isinstance(activation, Block) or callable(activation):
            return activation(inputs, **kwargs)
        return activation

    def forward(self, inputs, states):
        self._counter += 1
        return super().forward(inputs, states)


class HybridRecurrentCell(RecurrentCell, HybridBlock):
    """RecurrentCell that supports hybridize()."""

    def __init__(self, prefix=None, params=None):
        super().__init__(prefix=prefix, params=params)

    def forward(self, x, *args):
        self._counter += 1
        return HybridBlock.forward(self, x, *args)

    def hybrid_forward(self, F, x, *args, **kwargs):
        raise NotImplementedError


class RNNCell(HybridRecurrentCell):
    r"""Elman RNN cell: ``h' = act(W_ih x + b_ih + W_hh h + b_hh)``."""

    def __init__(self, hidden_size, activation='tanh', i2h_weight_initializer=None, h2h_weight_initializer=None,
                 i2h_bias_initializer='zeros', h2h_bias_initializer='zeros', input_size=0, prefix=None,
                 params=None):
        super().__init__(prefix=prefix, params=params)
        self._hidden_size = hidden_size
        self._activation = activation
        self._input_size = input_size
        self.i2h_weight = self.params.get('i2h_weight', shape=(hidden_size, input_size),
                                          init=i2h_weight_initializer, allow_deferred_init=True)
        self.h2h_weight = self.params.get('h2h_weight', shape=(hidden_size, hidden_size),
                                          init=h2h_weight_initializer, allow_deferred_init=True)
        self.i2h_bias = self.params.get('i2h_bias', shape=(hidden_size,), init=i2h_bias_initializer,
                                        allow_deferred_init=True)
        self.h2h_bias = self.params.get('h2h_bias', shape=(hidden_size,), init=h2h_bias_initializer,
                                        allow_deferred_init=True)

    def state_info(self, batch_size=0):
        return [{'shape': (batch_size, self._hidden_size), '__layout__': 'NC'}]

    def _alias(self):
        return 'rnn'

    def __repr__(self):
        shape = self.i2h_weight.shape
        return '{name}({mapping}, {_activation})'.format(
            name=self.__class__.__name__, mapping='{0} -> {1}'.format(shape[1] if shape[1] else None, shape[0]),
            **self.__dict__)

    def hybrid_forward(self, F, inputs, states, i2h_weight, h2h_weight, i2h_bias, h2h_bias):
        prefix = 't%d_' % self._counter
        i2h = F.FullyConnected(data=inputs, weight=i2h_weight, bias=i2h_bias, num_hidden=self._hidden_size,
                               name=prefix + 'i2h')
        h2h = F.FullyConnected(data=states[0], weight=h2h_weight, bias=h2h_bias, num_hidden=self._hidden_size,
                               name=prefix + 'h2h')
        i2h_plus_h2h = F.elemwise_add(i2h, h2h, name=prefix + 'plus0')
        output = self._get_activation(F, i2h_plus_h2h, self._activation, name=prefix + 'out')
        return output, [output]


class LSTMCell(HybridRecurrentCell):
    r"""LSTM cell; gates ordered (i, f, c, o) in the fused weight like the reference."""

    def __init__(self, hidden_size, i2h_weight_initializer=None, h2h_weight_initializer=None,
                 i2h_bias_initializer='zeros', h2h_bias_initializer='zeros', input_size=0, prefix=None,
                 params=None, activation='tanh', recurrent_activation='sigmoid'):
        super().__init__(prefix=prefix, params=params)
        self._hidden_size = hidden_size
        self._input_size = input_size
        self.i2h_weight = self.params.get('i2h_weight', shape=(4 * hidden_size, input_size),
                                          init=i2h_weight_initializer, allow_deferred_init=True)
        self.h2h_weight = self.params.get('h2h_weight', shape=(4 * hidden_size, hidden_size),
                                          init=h2h_weight_initializer, allow_deferred_init=True)
        self.i2h_bias = self.params.get('i2h_bias', shape=(4 * hidden_size,), init=i2h_bias_initializer,
                                        allow_deferred_init=True)
        self.h2h_bias = self.params.get('h2h_bias', shape=(4 * hidden_size,), init=h2h_bias_initializer,
                                        allow_deferred_init=True)
        self._activation = activation
        self._recurrent_activation = recurrent_activation

    def state_info(self, batch_size=0):
        return [{'shape': (batch_size, self._hidden_size), '__layout__': 'NC'},
                {'shape': (batch_size, self._hidden_size), '__layout__': 'NC'}]

    def _alias(self):
        return 'lstm'

    def __repr__(self):
        shape = self.i2h_weight.shape
        return '{name}({mapping})'.format(name=self.__class__.__name__,
                                          mapping='{0} -> {1}'.format(shape[1] if shape[1] else None, shape[0]))

    def hybrid_forward(self, F, inputs, states, i2h_weight, h2h_weight, i2h_bias, h2h_bias):
        prefix = 't%d_' % self._counter
        i2h = F.FullyConnected(data=inputs, weight=i2h_weight, bias=i2h_bias, num_hidden=self._hidden_size * 4,
                               name=prefix + 'i2h')
        h2h = F.FullyConnected(data=states[0], weight=h2h_weight, bias=h2h_bias,
                               num_hidden=self._hidden_size * 4, name=prefix + 'h2h')
        gates = F.elemwise_add(i2h, h2h, name=prefix + 'plus0')
        slice_gates = F.SliceChannel(gates, num_outputs=4, name=prefix + 'slice')
        in_gate = self._get_activation(F, slice_gates[0], self._recurrent_activation, name=prefix + 'i')
        forget_gate = self._get_activation(F, slice_gates[1], self._recurrent_activation, name=prefix + 'f')
        in_transform = self._get_activation(F, slice_gates[2], self._activation, name=prefix + 'c')
        out_gate = self._get_activation(F, slice_gates[3], self._recurrent_activation, name=prefix + 'o')
        next_c = F.elemwise_add(F.elemwise_mul(forget_gate, states[1], name=prefix + 'mul0'),
                                F.elemwise_mul(in_gate, in_transform, name=prefix + 'mul1'), name=prefix + 'state')
        next_h = F.elemwise_mul(out_gate, self._get_activation(F, next_c, self._activation, name=prefix + 'activation0'),
                                name=prefix + 'out')
        return next_h, [next_h, next_c]


class GRUCell(HybridRecurrentCell):
    r"""GRU cell (reset gate applied after the h2h matmul, as cuDNN/the reference)."""

    def __init__(self, hidden_size, i2h_weight_initializer=None, h2h_weight_initializer=None,
                 i2h_bias_initializer='zeros', h2h_bias_initializer='zeros', input_size=0, prefix=None,
                 params=None, activation='tanh', recurrent_activation='sigmoid'):
        super().__init__(prefix=prefix, params=params)
        self._hidden_size = hidden_size
        self._input_size = input_size
        self._activation = activation
        self._recurrent_activation = recurrent_activation
        self.i2h_weight = self.params.get('i2h_weight', shape=(3 * hidden_size, input_size),
                                          init=i2h_weight_initializer, allow_deferred_init=True)
        self.h2h_weight = self.params.get('h2h_weight', shape=(3 * hidden_size, hidden_size),
                                          init=h2h_weight_initializer, allow_deferred_init=True)
        self.i2h_bias = self.params.get('i2h_bias', shape=(3 * hidden_size,), init=i2h_bias_initializer,
                                        allow_deferred_init=True)
        self.h2h_bias = self.params.get('h2h_bias', shape=(3 * hidden_size,), init=h2h_bias_initializer,
                                        allow_deferred_init=True)

    def state_info(self, batch_size=0):
        return [{'shape': (batch_size, self._hidden_size), '__layout__': 'NC'}]

    def _alias(self):
        return 'gru'

    def __repr__(self):
        shape = self.i2h_weight.shape
        return '{name}({mapping})'.format(name=self.__class__.__name__,
                                          mapping='{0} -> {1}'.format(shape[1] if shape[1] else None, shape[0]))

    def hybrid_forward(self, F, inputs, states, i2h_weight, h2h_weight, i2h_bias, h2h_bias):
        prefix = 't%d_' % self._counter
        prev_state_h = states[0]
        i2h = F.FullyConnected(data=inputs, weight=i2h_weight, bias=i2h_bias, num_hidden=self._hidden_size * 3,
                               name=prefix + 'i2h')
        h2h = F.FullyConnected(data=prev_state_h, weight=h2h_weight, bias=h2h_bias,
                               num_hidden=self._hidden_size * 3, name=prefix + 'h2h')
        i2h_r, i2h_z, i2h = F.SliceChannel(i2h, num_outputs=3, name=prefix + 'i2h_slice')
        h2h_r, h2h_z, h2h = F.SliceChannel(h2h, num_outputs=3, name=prefix + 'h2h_slice')
        reset_gate = self._get_activation(F, F.elemwise_add(i2h_r, h2h_r, name=prefix + 'plus0'),
                                          self._recurrent_activation, name=prefix + 'r_act')
        update_gate = self._get_activation(F, F.elemwise_add(i2h_z, h2h_z, name=prefix + 'plus1'),
                                           self._recurrent_activation, name=prefix + 'z_act')
        next_h_tmp = self._get_activation(F, F.elemwise_add(i2h, F.elemwise_mul(reset_gate, h2h,
                                                                                 name=prefix + 'mul0'),
                                                            name=prefix + 'plus2'),
                                          self._activation, name=prefix + 'h_act')
        ones = F.ones_like(update_gate, name=prefix + 'ones_like0')
        next_h = F.elemwise_add(F.elemwise_mul(F.elemwise_sub(ones, update_gate, name=prefix + 'minus0'),
                                               next_h_tmp, name=prefix + 'mul1'),
                                F.elemwise_mul(update_gate, prev_state_h, name=prefix + 'mul20'),
                                name=prefix + 'out')
        return next_h, [next_h]


class SequentialRNNCell(RecurrentCell):
    """Stack of cells; the output of one feeds the next."""

    def __init__(self, prefix=None, params=None):
        super().__init__(prefix=prefix, params=params)

    def __repr__(self):
        s = '{name}(\n{modstr}\n)'
        return s.format(name=self.__class__.__name__,
                        modstr='\n'.join(['({i}): {m}'.format(i=i, m=_indent(m.__repr__(), 2))
                                          for i, m in self._children.items()]))

    def add(self, cell):
        self.register_child(cell)

    def state_info(self, batch_size=0):
        return _cells_state_info(self._children.values(), batch_size)

    def begin_state(self, **kwargs):
        assert not self._modified, 'After applying modifier cells the base cell cannot be called directly.'
        return _cells_begin_state(self._children.values(), **kwargs)

    def unroll(self, length, inputs, begin_state=None, layout='NTC', merge_outputs=None, valid_length=None):
        self.reset()
        inputs, _, F, batch_size = _format_sequence(length, inputs, layout, None)
        num_cells = len(self._children)
        begin_state = _get_begin_state(self, F, begin_state, inputs, batch_size)
        p = 0
        next_states = []
        for i, cell in enumerate(self._children.values()):
            n = len(cell.state_info())
            states = begin_state[p:p + n]
            p += n
            inputs, states = cell.unroll(length, inputs=inputs, begin_state=states, layout=layout,
                                         merge_outputs=None if i < num_cells - 1 else merge_outputs,
                                         valid_length=valid_length)
            next_states.extend(states)
        return inputs, next_states

    def __getitem__(self, i):
        return list(self._children.values())[i]

    def __len__(self):
        return len(self._children)

    def __call__(self, inputs, states):
        self._counter += 1
        next_states = []
        p = 0
        assert all(not isinstance(cell, BidirectionalCell) for cell in self._children.values())
        for cell in self._children.values():
            n = len(cell.state_info())
            state = states[p:p + n]
            p += n
            inputs, state = cell(inputs, state)
            next_states.append(state)
        return inputs, sum(next_states, [])

    def hybrid_forward(self, *args, **kwargs):
        raise NotImplementedError


class HybridSequentialRNNCell(HybridRecurrentCell):
    """Hybridizable stack of cells."""

    def __init__(self, prefix=None, params=None):
        super().__init__(prefix=prefix, params=params)

    __repr__ = SequentialRNNCell.__repr__
    add = SequentialRNNCell.add
    state_info = SequentialRNNCell.state_info
    begin_state = SequentialRNNCell.begin_state
    unroll = SequentialRNNCell.unroll
    __getitem__ = SequentialRNNCell.__getitem__
    __len__ = SequentialRNNCell.__len__

    def __call__(self, inputs, states):
        self._counter += 1
        next_states = []
        p = 0
        for cell in self._children.values():
            n = len(cell.state_info())
            state = states[p:p + n]
            p += n
            inputs, state = cell(inputs, state)
            next_states.append(state)
        return inputs, sum(next_states, [])

    def hybrid_forward(self, F, inputs, states):
        return self.__call__(inputs, states)


class DropoutCell(HybridRecurrentCell):
    """Apply dropout on the input (no state)."""

    def __init__(self, rate, axes=(), prefix=None, params=None):
        super().__init__(prefix, params)
        assert isinstance(rate, (int, float)), 'rate must be a number'
        self._rate = rate
        self._axes = axes

    def __repr__(self):
        return '{name}(rate={_rate}, axes={_axes})'.format(name=self.__class__.__name__, **self.__dict__)

    def state_info(self, batch_size=0):
        return []

    def _alias(self):
        return 'dropout'

    def hybrid_forward(self, F, inputs, states):
        if self._rate > 0:
            inputs = F.Dropout(data=inputs, p=self._rate, axes=self._axes, name='t%d_fwd' % self._counter)
        return inputs, states

    def unroll(self, length, inputs, begin_state=None, layout='NTC', merge_outputs=None, valid_length=None):
        self.reset()
        inputs, _, F, _ = _format_sequence(length, inputs, layout, merge_outputs)
        if isinstance(inputs, tensor_types):
            return self.hybrid_forward(F, inputs, begin_state if begin_state else [])
        return super().unroll(length, inputs, begin_state=begin_state, layout=layout,
                              merge_outputs=merge_outputs, valid_length=None)


class ModifierCell(HybridRecurrentCell):
    """Base class for cells that wrap (modify) another cell."""

    def __init__(self, base_cell):
        assert not base_cell._modified, 'Cell %s is already modified. One cell cannot be modified twice' \
            % base_cell.name
        base_cell._modified = True
        super().__init__(prefix=base_cell.prefix + self._alias(), params=None)
        self.base_cell = base_cell

    @property
    def params(self):
        return self.base_cell.params

    def state_info(self, batch_size=0):
        return self.base_cell.state_info(batch_size)

    def begin_state(self, func=ndarray.zeros, **kwargs):
        assert not self._modified, 'After applying modifier cells the base cell cannot be called directly.'
        self.base_cell._modified = False
        begin = self.base_cell.begin_state(func=func, **kwargs)
        self.base_cell._modified = True
        return begin

    def hybrid_forward(self, F, inputs, states):
        raise NotImplementedError

    def __repr__(self):
        return '{name}({base_cell})'.format(name=self.__class__.__name__, **self.__dict__)


class ZoneoutCell(ModifierCell):
    """Zoneout regularisation (Krueger et al. 2016) on outputs and/or states."""

    def __init__(self, base_cell, zoneout_outputs=0., zoneout_states=0.):
        assert not isinstance(base_cell, BidirectionalCell), \
            'BidirectionalCell doesn\'t support zoneout since it doesn\'t support step. ' \
            'Please add ZoneoutCell to the cells underneath instead.'
        assert not isinstance(base_cell, SequentialRNNCell) or not base_cell._bidirectional if hasattr(
            base_cell, '_bidirectional') else True
        super().__init__(base_cell)
        self.zoneout_outputs = zoneout_outputs
        self.zoneout_states = zoneout_states
        self._prev_output = None

    def __repr__(self):
        return '{name}(p_out={zoneout_outputs}, p_state={zoneout_states}, {base_cell})'.format(
            name=self.__class__.__name__, **self.__dict__)

    def _alias(self):
        return 'zoneout'

    def reset(self):
        super().reset()
        self._prev_output = None

    def hybrid_forward(self, F, inputs, states):
        cell, p_outputs, p_states = self.base_cell, self.zoneout_outputs, self.zoneout_states
        next_output, next_states = cell(inputs, states)

        def mask(p, like):
            return F.Dropout(F.ones_like(like), p=p)
        prev_output = self._prev_output
        if prev_output is None:
            prev_output = F.zeros_like(next_output)
        output = F.where(mask(p_outputs, next_output), next_output, prev_output) if p_outputs != 0. \
            else next_output
        states = [F.where(mask(p_states, new_s), new_s, old_s) for new_s, old_s in zip(next_states, states)] \
            if p_states != 0. else next_states
        self._prev_output = output
        return output, states


class ResidualCell(ModifierCell):
    """Adds the input to the output of the wrapped cell."""

    def __init__(self, base_cell):
        super().__init__(base_cell)

    def hybrid_forward(self, F, inputs, states):
        output, states = self.base_cell(inputs, states)
        output = F.elemwise_add(output, inputs, name='t%d_fwd' % self._counter)
        return output, states

    def unroll(self, length, inputs, begin_state=None, layout='NTC', merge_outputs=None, valid_length=None):
        self.reset()
        self.base_cell._modified = False
        outputs, states = self.base_cell.unroll(length, inputs=inputs, begin_state=begin_state, layout=layout,
                                                merge_outputs=merge_outputs, valid_length=valid_length)
        self.base_cell._modified = True
        merge_outputs = isinstance(outputs, tensor_types) if merge_outputs is None else merge_outputs
        inputs, axis, F, _ = _format_sequence(length, inputs, layout, merge_outputs)
        if valid_length is not None:
            inputs = _mask_sequence_variable_length(F, inputs, length, valid_length, axis, merge_outputs)
        if merge_outputs:
            outputs = F.elemwise_add(outputs, inputs)
        else:
            outputs = [F.elemwise_add(i, j) for i, j in zip(outputs, inputs)]
        return outputs, states


class BidirectionalCell(HybridRecurrentCell):
    """Run ``l_cell`` forward and ``r_cell`` backward over time and concatenate outputs."""

    def __init__(self, l_cell, r_cell, output_prefix='bi_'):
        super().__init__(prefix='', params=None)
        self.register_child(l_cell, 'l_cell')
        self.register_child(r_cell, 'r_cell')
        self._output_prefix = output_prefix

    def __call__(self, inputs, states):
        raise NotImplementedError('Bidirectional cannot be stepped. Please use unroll')

    def __repr__(self):
        return '{name}(forward={l_cell}, backward={r_cell})'.format(
            name=self.__class__.__name__, l_cell=self._children['l_cell'], r_cell=self._children['r_cell'])

    def state_info(self, batch_size=0):
        return _cells_state_info(self._children.values(), batch_size)

    def begin_state(self, **kwargs):
        assert not self._modified, 'After applying modifier cells the base cell cannot be called directly.'
        return _cells_begin_state(self._children.values(), **kwargs)

    def unroll(self, length, inputs, begin_state=None, layout='NTC', merge_outputs=None, valid_length=None):
        self.reset()
        inputs, axis, F, batch_size = _format_sequence(length, inputs, layout, False)
        reversed_inputs = list(_reverse_sequences(inputs, length, valid_length))
        begin_state = _get_begin_state(self, F, begin_state, inputs, batch_size)
        states = begin_state
        l_cell, r_cell = self._children['l_cell'], self._children['r_cell']
        l_outputs, l_states = l_cell.unroll(length, inputs=inputs,
                                            begin_state=states[:len(l_cell.state_info(batch_size))],
                                            layout=layout, merge_outputs=merge_outputs, valid_length=valid_length)
        r_outputs, r_states = r_cell.unroll(length, inputs=reversed_inputs,
                                            begin_state=states[len(l_cell.state_info(batch_size)):],
                                            layout=layout, merge_outputs=False, valid_length=valid_length)
        reversed_r_outputs = _reverse_sequences(r_outputs, length, valid_length)
        if merge_outputs is None:
            merge_outputs = isinstance(l_outputs, tensor_types)
            l_outputs, _, _, _ = _format_sequence(None, l_outputs, layout, merge_outputs)
            reversed_r_outputs, _, _, _ = _format_sequence(None, reversed_r_outputs, layout, merge_outputs)
        if merge_outputs:
            reversed_r_outputs = F.stack(*reversed_r_outputs, axis=axis)
            outputs = F.concat(l_outputs, reversed_r_outputs, dim=2, name='%sout' % self._output_prefix)
        else:
            outputs = [F.concat(l_o, r_o, dim=1, name='%st%d' % (self._output_prefix, i))
                       for i, (l_o, r_o) in enumerate(zip(l_outputs, reversed_r_outputs))]
        if valid_length is not None:
            outputs = _mask_sequence_variable_length(F, outputs, length, valid_length, axis, merge_outputs)
        states = l_states + r_states
        return outputs, states


class LSTMPCell(HybridRecurrentCell):
    """LSTM with a recurrent projection layer (Sak et al. 2014): ``r = W_hr h``."""

    def __init__(self, hidden_size, projection_size, i2h_weight_initializer=None, h2h_weight_initializer=None,
                 h2r_weight_initializer=None, i2h_bias_initializer='zeros', h2h_bias_initializer='zeros',
                 input_size=0, prefix=None, params=None):
        super().__init__(prefix=prefix, params=params)
        self._hidden_size = hidden_size
        self._input_size = input_size
        self._projection_size = projection_size
        self.i2h_weight = self.params.get('i2h_weight', shape=(4 * hidden_size, input_size),
                                          init=i2h_weight_initializer, allow_deferred_init=True)
        self.h2h_weight = self.params.get('h2h_weight', shape=(4 * hidden_size, projection_size),
                                          init=h2h_weight_initializer, allow_deferred_init=True)
        self.h2r_weight = self.params.get('h2r_weight', shape=(projection_size, hidden_size),
                                          init=h2r_weight_initializer, allow_deferred_init=True)
        self.i2h_bias = self.params.get('i2h_bias', shape=(4 * hidden_size,), init=i2h_bias_initializer,
                                        allow_deferred_init=True)
        self.h2h_bias = self.params.get('h2h_bias', shape=(4 * hidden_size,), init=h2h_bias_initializer,
                                        allow_deferred_init=True)

    def state_info(self, batch_size=0):
        return [{'shape': (batch_size, self._projection_size), '__layout__': 'NC'},
                {'shape': (batch_size, self._hidden_size), '__layout__': 'NC'}]

    def _alias(self):
        return 'lstmp'

    def hybrid_forward(self, F, inputs, states, i2h_weight, h2h_weight, h2r_weight, i2h_bias, h2h_bias):
        prefix = 't%d_' % self._counter
        i2h = F.FullyConnected(data=inputs, weight=i2h_weight, bias=i2h_bias, num_hidden=self._hidden_size * 4,
                               name=prefix + 'i2h')
        h2h = F.FullyConnected(data=states[0], weight=h2h_weight, bias=h2h_bias,
                               num_hidden=self._hidden_size * 4, name=prefix + 'h2h')
        gates = i2h + h2h
        slice_gates = F.SliceChannel(gates, num_outputs=4, name=prefix + 'slice')
        in_gate = F.Activation(slice_gates[0], act_type='sigmoid', name=prefix + 'i')
        forget_gate = F.Activation(slice_gates[1], act_type='sigmoid', name=prefix + 'f')
        in_transform = F.Activation(slice_gates[2], act_type='tanh', name=prefix + 'c')
        out_gate = F.Activation(slice_gates[3], act_type='sigmoid', name=prefix + 'o')
        next_c = F.elemwise_add(forget_gate * states[1], in_gate * in_transform, name=prefix + 'state')
        hidden = F.elemwise_mul(out_gate, F.Activation(next_c, act_type='tanh'), name=prefix + 'hidden')
        next_r = F.FullyConnected(data=hidden, num_hidden=self._projection_size, weight=h2r_weight, no_bias=True,
                                  name=prefix + 'out')
        return next_r, [next_r, next_c]


class VariationalDropoutCell(ModifierCell):
    """Variational dropout (Gal & Ghahramani 2016): one dropout mask per sequence for inputs/states/outputs."""

    def __init__(self, base_cell, drop_inputs=0., drop_states=0., drop_outputs=0.):
        assert not drop_states or not isinstance(base_cell, BidirectionalCell), \
            'BidirectionalCell doesn\'t support variational state dropout.'
        super().__init__(base_cell)
        self.drop_inputs = drop_inputs
        self.drop_states = drop_states
        self.drop_outputs = drop_outputs
        self.drop_inputs_mask = None
        self.drop_states_mask = None
        self.drop_outputs_mask = None

    def _alias(self):
        return 'vardrop'

    def reset(self):
        super().reset()
        self.drop_inputs_mask = None
        self.drop_states_mask = None
        self.drop_outputs_mask = None

    def _initialize_input_masks(self, F, inputs, states):
        if self.drop_states and self.drop_states_mask is None:
            self.drop_states_mask = F.Dropout(F.ones_like(states[0]), p=self.drop_states)
        if self.drop_inputs and self.drop_inputs_mask is None:
            self.drop_inputs_mask = F.Dropout(F.ones_like(inputs), p=self.drop_inputs)

    def _initialize_output_mask(self, F, output):
        if self.drop_outputs and self.drop_outputs_mask is None:
            self.drop_outputs_mask = F.Dropout(F.ones_like(output), p=self.drop_outputs)

    def hybrid_forward(self, F, inputs, states):
        cell = self.base_cell
        self._initialize_input_masks(F, inputs, states)
        if self.drop_states:
            states = list(states)
            states[0] = states[0] * self.drop_states_mask
        if self.drop_inputs:
            inputs = inputs * self.drop_inputs_mask
        next_output, next_states = cell(inputs, states)
        self._initialize_output_mask(F, next_output)
        if self.drop_outputs:
            next_output = next_output * self.drop_outputs_mask
        return next_output, next_states

    def __repr__(self):
        return '{name}(p_out = {drop_outputs}, p_state = {drop_states})'.format(name=self.__class__.__name__,
                                                                               **self.__dict__)
