"""Fused recurrent layers RNN / LSTM / GRU (parity: python/mxnet/gluon/rnn/rnn_layer.py).

Per-layer/direction parameters ``{l,r}{i}_{i2h,h2h,h2r}_{weight,bias}`` are
concatenated (weights first, then biases — the reference's flat layout) and
fed to the fused ``RNN`` operator, which runs MIOpen-backed torch RNN kernels
on the MI355X (or the explicit loop for clipping / variable lengths).
"""
import re

from ... import ndarray, symbol
from ...ndarray.ndarray import NDArray
from ..block import HybridBlock
from . import rnn_cell

__all__ = ['RNN', 'LSTM', 'GRU']


class _RNNLayer(HybridBlock):
    def __init__(self, hidden_size, num_layers, layout, dropout, bidirectional, input_size,
                 i2h_weight_initializer, h2h_weight_initializer, i2h_bias_initializer, h2h_bias_initializer, mode,
                 projection_size, h2r_weight_initializer, lstm_state_clip_min, lstm_state_clip_max,
                 lstm_state_clip_nan, dtype, use_sequence_length=False, **kwargs):
        super().__init__(**kwargs)
        assert layout in ('TNC', 'NTC'), "Invalid layout %s; must be one of ['TNC' or 'NTC']" % layout
        self._hidden_size = hidden_size
        self._projection_size = projection_size if projection_size else None
        self._num_layers = num_layers
        self._mode = mode
        self._layout = layout
        self._dropout = dropout
        self._dir = 2 if bidirectional else 1
        self._input_size = input_size
        self._i2h_weight_initializer = i2h_weight_initializer
        self._h2h_weight_initializer = h2h_weight_initializer
        self._i2h_bias_initializer = i2h_bias_initializer
        self._h2h_bias_initializer = h2h_bias_initializer
        self._h2r_weight_initializer = h2r_weight_initializer
        self._lstm_state_clip_min = lstm_state_clip_min
        self._lstm_state_clip_max = lstm_state_clip_max
        self._lstm_state_clip_nan = lstm_state_clip_nan
        self._dtype = dtype
        self._use_sequence_length = use_sequence_length
        self.skip_states = None
        self._gates = {'rnn_relu': 1, 'rnn_tanh': 1, 'lstm': 4, 'gru': 3}[mode]
        ng, ni, nh = self._gates, input_size, hidden_size
        npj = self._projection_size
        for i in range(num_layers):
            for j in ['l', 'r'][:self._dir]:
                self._register_param('{}{}_i2h_weight'.format(j, i), (ng * nh, ni), i2h_weight_initializer, dtype)
                self._register_param('{}{}_h2h_weight'.format(j, i), (ng * nh, npj or nh), h2h_weight_initializer,
                                     dtype)
                self._register_param('{}{}_i2h_bias'.format(j, i), (ng * nh,), i2h_bias_initializer, dtype)
                self._register_param('{}{}_h2h_bias'.format(j, i), (ng * nh,), h2h_bias_initializer, dtype)
                if npj:
                    self._register_param('{}{}_h2r_weight'.format(j, i), (npj, nh), h2r_weight_initializer, dtype)
            ni = (npj or nh) * self._dir

    def _register_param(self, name, shape, init, dtype):
        p = self.params.get(name, shape=shape, init=init, allow_deferred_init=True, dtype=dtype)
        setattr(self, name, p)
        return p

    def __repr__(self):
        s = '{name}({mapping}, {_layout}'
        if self._num_layers != 1:
            s += ', num_layers={_num_layers}'
        if self._dropout != 0:
            s += ', dropout={_dropout}'
        if self._dir == 2:
            s += ', bidirectional'
        s += ')'
        shape = self.l0_i2h_weight.shape
        mapping = '{0} -> {1}'.format(shape[1] if shape[1] else None, shape[0] // self._gates)
        return s.format(name=self.__class__.__name__, mapping=mapping, **self.__dict__)

    def _collect_params_with_prefix(self, prefix=''):
        # parameter-file names follow the unfused cell layout for compatibility with the reference
        if prefix:
            prefix += '.'
        pattern = re.compile(r'(l|r)(\d+)_(i2h|h2h|h2r)_(weight|bias)\Z')

        def convert_key(m, bidirectional):
            d, l, g, t = [m.group(i) for i in range(1, 5)]
            if bidirectional:
                return '_unfused.{}.{}_cell.{}_{}'.format(l, d, g, t)
            return '_unfused.{}.{}_{}'.format(l, g, t)
        bidirectional = any(pattern.match(k).group(1) == 'r' for k in self._reg_params)
        ret = {prefix + convert_key(pattern.match(key), bidirectional): val for key, val in self._reg_params.items()}
        for name, child in self._children.items():
            ret.update(child._collect_params_with_prefix(prefix + name))
        return ret

    def state_info(self, batch_size=0):
        raise NotImplementedError

    def _unfuse(self):
        """Equivalent stack of cells sharing this layer's parameters."""
        assert not self._projection_size, '_unfuse does not support projection layer yet!'
        assert not self._lstm_state_clip_min and not self._lstm_state_clip_max, \
            '_unfuse does not support state clipping yet!'
        get_cell = {'rnn_relu': lambda **kw: rnn_cell.RNNCell(self._hidden_size, activation='relu', **kw),
                    'rnn_tanh': lambda **kw: rnn_cell.RNNCell(self._hidden_size, activation='tanh', **kw),
                    'lstm': lambda **kw: rnn_cell.LSTMCell(self._hidden_size, **kw),
                    'gru': lambda **kw: rnn_cell.GRUCell(self._hidden_size, **kw)}[self._mode]
        stack = rnn_cell.HybridSequentialRNNCell(prefix=self.prefix, params=self.params)
        with stack.name_scope():
            ni = self._input_size
            for i in range(self._num_layers):
                kwargs = {'input_size': ni, 'i2h_weight_initializer': self._i2h_weight_initializer,
                          'h2h_weight_initializer': self._h2h_weight_initializer,
                          'i2h_bias_initializer': self._i2h_bias_initializer,
                          'h2h_bias_initializer': self._h2h_bias_initializer}
                if self._dir == 2:
                    stack.add(rnn_cell.BidirectionalCell(get_cell(prefix='l%d_' % i, **kwargs),
                                                         get_cell(prefix='r%d_' % i, **kwargs)))
                else:
                    stack.add(get_cell(prefix='l%d_' % i, **kwargs))
                if self._dropout > 0 and i != self._num_layers - 1:
                    stack.add(rnn_cell.DropoutCell(self._dropout))
                ni = self._hidden_size * self._dir
        return stack

    def cast(self, dtype):
        super().cast(dtype)
        self._dtype = dtype

    def begin_state(self, batch_size=0, func=ndarray.zeros, **kwargs):
        states = []
        for i, info in enumerate(self.state_info(batch_size)):
            if info is not None:
                info = dict(info)
                info.update(kwargs)
            else:
                info = dict(kwargs)
            info.pop('__layout__', None)
            if 'symbol' in getattr(func, '__module__', ''):
                info.pop('ctx', None)
            states.append(func(name='%sh0_%d' % (self.prefix, i), **info))
        return states

    def __call__(self, inputs, states=None, sequence_length=None, **kwargs):
        self.skip_states = states is None
        if states is None:
            if isinstance(inputs, NDArray):
                batch_size = inputs.shape[self._layout.find('N')]
                states = self.begin_state(batch_size, ctx=inputs.context, dtype=inputs.dtype)
            else:
                states = self.begin_state(0, func=symbol.zeros)
        if isinstance(states, (NDArray, symbol.Symbol)):
            states = [states]
        if self._use_sequence_length:
            return super().__call__(inputs, states, sequence_length, **kwargs)
        return super().__call__(inputs, states, **kwargs)

    def hybrid_forward(self, F, inputs, states, sequence_length=None, **kwargs):
        if F is ndarray:
            batch_size = inputs.shape[self._layout.find('N')]
            for state, info in zip(states, self.state_info(batch_size)):
                if state.shape != info['shape']:
                    raise ValueError('Invalid recurrent state shape. Expecting %s, got %s.'
                                     % (str(info['shape']), str(state.shape)))
        out = self._forward_kernel(F, inputs, states, sequence_length, **kwargs)
        return out[0] if self.skip_states else out

    def _forward_kernel(self, F, inputs, states, sequence_length, **kwargs):
        if self._layout == 'NTC':
            inputs = F.swapaxes(inputs, dim1=0, dim2=1)
        groups = ['i2h', 'h2h', 'h2r'] if self._projection_size else ['i2h', 'h2h']
        params = [kwargs['{}{}_{}_{}'.format(d, l, g, t)].reshape(-1)
                  for t in ['weight', 'bias']
                  for l in range(self._num_layers)
                  for d in ['l', 'r'][:self._dir]
                  for g in groups if g != 'h2r' or t != 'bias']
        params = F._internal._rnn_param_concat(*params, dim=0)
        rnn_args = list(states) + ([sequence_length] if self._use_sequence_length else [])
        rnn = F.RNN(inputs, params, *rnn_args, use_sequence_length=self._use_sequence_length,
                    state_size=self._hidden_size, projection_size=self._projection_size,
                    num_layers=self._num_layers, bidirectional=self._dir == 2, p=self._dropout, state_outputs=True,
                    mode=self._mode, lstm_state_clip_min=self._lstm_state_clip_min,
                    lstm_state_clip_max=self._lstm_state_clip_max, lstm_state_clip_nan=self._lstm_state_clip_nan)
        if self._mode == 'lstm':
            outputs, states = rnn[0], [rnn[1], rnn[2]]
        else:
            outputs, states = rnn[0], [rnn[1]]
        if self._layout == 'NTC':
            outputs = F.swapaxes(outputs, dim1=0, dim2=1)
        return outputs, states


class RNN(_RNNLayer):
    """Multi-layer Elman RNN with tanh or ReLU non-linearity."""

    def __init__(self, hidden_size, num_layers=1, activation='relu', layout='TNC', dropout=0, bidirectional=False,
                 i2h_weight_initializer=None, h2h_weight_initializer=None, i2h_bias_initializer='zeros',
                 h2h_bias_initializer='zeros', input_size=0, dtype='float32', **kwargs):
        super().__init__(hidden_size, num_layers, layout, dropout, bidirectional, input_size,
                         i2h_weight_initializer, h2h_weight_initializer, i2h_bias_initializer, h2h_bias_initializer,
                         'rnn_' + activation, None, None, None, None, False, dtype, **kwargs)

    def state_info(self, batch_size=0):
        return [{'shape': (self._num_layers * self._dir, batch_size, self._hidden_size), '__layout__': 'LNC',
                 'dtype': self._dtype}]


class LSTM(_RNNLayer):
    """Multi-layer LSTM (optionally projected: LSTMP, with state clipping)."""

    def __init__(self, hidden_size, num_layers=1, layout='TNC', dropout=0, bidirectional=False, input_size=0,
                 i2h_weight_initializer=None, h2h_weight_initializer=None, i2h_bias_initializer='zeros',
                 h2h_bias_initializer='zeros', projection_size=None, h2r_weight_initializer=None,
                 state_clip_min=None, state_clip_max=None, state_clip_nan=False, dtype='float32', **kwargs):
        super().__init__(hidden_size, num_layers, layout, dropout, bidirectional, input_size,
                         i2h_weight_initializer, h2h_weight_initializer, i2h_bias_initializer, h2h_bias_initializer,
                         'lstm', projection_size, h2r_weight_initializer, state_clip_min, state_clip_max,
                         state_clip_nan, dtype, **kwargs)

    def state_info(self, batch_size=0):
        if self._projection_size is None:
            return [{'shape': (self._num_layers * self._dir, batch_size, self._hidden_size), '__layout__': 'LNC',
                     'dtype': self._dtype},
                    {'shape': (self._num_layers * self._dir, batch_size, self._hidden_size), '__layout__': 'LNC',
                     'dtype': self._dtype}]
        return [{'shape': (self._num_layers * self._dir, batch_size, self._projection_size), '__layout__': 'LNC',
                 'dtype': self._dtype},
                {'shape': (self._num_layers * self._dir, batch_size, self._hidden_size), '__layout__': 'LNC',
                 'dtype': self._dtype}]


class GRU(_RNNLayer):
    """Multi-layer GRU."""

    def __init__(self, hidden_size, num_layers=1, layout='TNC', dropout=0, bidirectional=False, input_size=0,
                 i2h_weight_initializer=None, h2h_weight_initializer=None, i2h_bias_initializer='zeros',
                 h2h_bias_initializer='zeros', dtype='float32', **kwargs):
        super().__init__(hidden_size, num_layers, layout, dropout, bidirectional, input_size,
                         i2h_weight_initializer, h2h_weight_initializer, i2h_bias_initializer, h2h_bias_initializer,
                         'gru', None, None, None, None, False, dtype, **kwargs)

    def state_info(self, batch_size=0):
        return [{'shape': (self._num_layers * self._dir, batch_size, self._hidden_size), '__layout__': 'LNC',
                 'dtype': self._dtype}]
