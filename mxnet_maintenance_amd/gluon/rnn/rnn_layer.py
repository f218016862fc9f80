"""Fused recurrent layers RNN / LSTM / GRU (parity: python/mxnet/gluon/rnn/rnn_layer.py).

Each (layer, direction) owns ``{l,r}{layer}_{i2h,h2h[,h2r]}_{weight,bias}``
parameters.  The forward flattens them into the fused ``RNN`` operator's single
parameter vector -- every weight (layer-major, direction, group) first, then
every bias -- which is the layout the reference's cuDNN path uses, so
``.params`` files interchange.  The operator itself runs the in-tree gfx950
recurrent kernels (ops/rnn_fns.py) on the GPU.
"""
import re

from ... import ndarray, symbol
from ...ndarray.ndarray import NDArray
from ..block import HybridBlock
from . import rnn_cell

__all__ = ['RNN', 'LSTM', 'GRU']

_GATES = {'rnn_relu': 1, 'rnn_tanh': 1, 'lstm': 4, 'gru': 3}
_PARAM_RE = re.compile(r'(?P<dir>[lr])(?P<layer>\d+)_(?P<group>i2h|h2h|h2r)_(?P<kind>weight|bias)\Z')


class _RNNLayer(HybridBlock):
    """Shared machinery of the fused layers; subclasses only describe their recurrent state."""

    def __init__(self, hidden_size, num_layers, layout, dropout, bidirectional, input_size,
                 i2h_weight_initializer, h2h_weight_initializer, i2h_bias_initializer, h2h_bias_initializer, mode,
                 projection_size, h2r_weight_initializer, lstm_state_clip_min, lstm_state_clip_max,
                 lstm_state_clip_nan, dtype, use_sequence_length=False, **kwargs):
        super().__init__(**kwargs)
        if layout not in ('TNC', 'NTC'):
            raise AssertionError("Invalid layout %s; must be one of ['TNC' or 'NTC']" % layout)
        self._mode = mode
        self._gates = _GATES[mode]
        self._hidden_size = hidden_size
        self._projection_size = projection_size or None
        self._num_layers = num_layers
        self._layout = layout
        self._dropout = dropout
        self._dir = 2 if bidirectional else 1
        self._input_size = input_size
        self._inits = {'i2h_weight': i2h_weight_initializer, 'h2h_weight': h2h_weight_initializer,
                       'i2h_bias': i2h_bias_initializer, 'h2h_bias': h2h_bias_initializer,
                       'h2r_weight': h2r_weight_initializer}
        # attribute names kept for code that introspects them (the reference exposes these)
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
        for name, shape in self._param_specs():
            kind = name.split('_', 1)[1]
            p = self.params.get(name, shape=shape, init=self._inits[kind], allow_deferred_init=True, dtype=dtype)
            setattr(self, name, p)

    # ------------------------------------------------------------------ parameter layout
    def _directions(self):
        return 'lr'[:self._dir]

    def _param_specs(self):
        """(name, shape) of every parameter, in registration order."""
        rows = self._gates * self._hidden_size
        rec = self._projection_size or self._hidden_size
        width = self._input_size
        specs = []
        for layer in range(self._num_layers):
            for d in self._directions():
                tag = '%s%d_' % (d, layer)
                specs += [(tag + 'i2h_weight', (rows, width)), (tag + 'h2h_weight', (rows, rec)),
                          (tag + 'i2h_bias', (rows,)), (tag + 'h2h_bias', (rows,))]
                if self._projection_size:
                    specs.append((tag + 'h2r_weight', (self._projection_size, self._hidden_size)))
            width = rec * self._dir
        return specs

    def _flat_order(self):
        """Parameter names in the fused operator's flat order: all weights, then all biases."""
        groups = ('i2h', 'h2h', 'h2r') if self._projection_size else ('i2h', 'h2h')
        names = []
        for kind in ('weight', 'bias'):
            for layer in range(self._num_layers):
                for d in self._directions():
                    names += ['%s%d_%s_%s' % (d, layer, g, kind) for g in groups
                              if not (g == 'h2r' and kind == 'bias')]
        return names

    def __repr__(self):
        w = self.l0_i2h_weight.shape
        parts = ['%s -> %s' % (w[1] or None, w[0] // self._gates), self._layout]
        if self._num_layers != 1:
            parts.append('num_layers=%d' % self._num_layers)
        if self._dropout != 0:
            parts.append('dropout=%s' % self._dropout)
        if self._dir == 2:
            parts.append('bidirectional')
        return '%s(%s)' % (type(self).__name__, ', '.join(parts))

    def _collect_params_with_prefix(self, prefix=''):
        # saved names follow the unfused cell stack (`_unfused.<layer>[.<dir>_cell].<group>_<kind>`), the
        # naming the reference writes, so checkpoints load into either form
        lead = prefix + '.' if prefix else ''
        bidir = self._dir == 2
        out = {}
        for key, val in self._reg_params.items():
            m = _PARAM_RE.match(key)
            cell = '%s.%s_cell' % (m.group('layer'), m.group('dir')) if bidir else m.group('layer')
            out['%s_unfused.%s.%s_%s' % (lead, cell, m.group('group'), m.group('kind'))] = val
        for name, child in self._children.items():
            out.update(child._collect_params_with_prefix(lead + name))
        return out

    def state_info(self, batch_size=0):
        raise NotImplementedError

    def _symbol_begin_state(self, inputs):
        """Zero initial states of a traced graph, sized by the batch of ``inputs`` on every call:
        a (1, N, 1) zero slice of the input broadcast to (layers * directions, N, width) -- unlike
        zeros with an unknown batch dim, it stays right when a cached graph sees another batch size."""
        t_axis, c_axis = self._layout.index('T'), self._layout.index('C')
        z = symbol.slice_axis(symbol.slice_axis(inputs, axis=t_axis, begin=0, end=1), axis=c_axis, begin=0, end=1)
        z = symbol.reshape(symbol.zeros_like(z), shape=(1, -1, 1))
        return [symbol.broadcast_to(z, shape=(info['shape'][0], 0, info['shape'][2]))
                for info in self.state_info(0)]

    def _state_spec(self, batch_size, width):
        return {'shape': (self._num_layers * self._dir, batch_size, width), '__layout__': 'LNC',
                'dtype': self._dtype}

    # ------------------------------------------------------------------ unfused equivalent
    def _make_cell(self, prefix, input_size):
        kw = dict(prefix=prefix, input_size=input_size,
                  i2h_weight_initializer=self._inits['i2h_weight'], h2h_weight_initializer=self._inits['h2h_weight'],
                  i2h_bias_initializer=self._inits['i2h_bias'], h2h_bias_initializer=self._inits['h2h_bias'])
        if self._mode == 'lstm':
            return rnn_cell.LSTMCell(self._hidden_size, **kw)
        if self._mode == 'gru':
            return rnn_cell.GRUCell(self._hidden_size, **kw)
        return rnn_cell.RNNCell(self._hidden_size, activation=self._mode[len('rnn_'):], **kw)

    def _unfuse(self):
        """A HybridSequentialRNNCell computing the same function with this layer's parameters."""
        if self._projection_size:
            raise AssertionError('projection layers have no unfused cell equivalent')
        if self._lstm_state_clip_min or self._lstm_state_clip_max:
            raise AssertionError('state clipping has no unfused cell equivalent')
        stack = rnn_cell.HybridSequentialRNNCell(prefix=self.prefix, params=self.params)
        with stack.name_scope():
            width = self._input_size
            last = self._num_layers - 1
            for layer in range(self._num_layers):
                cells = [self._make_cell('%s%d_' % (d, layer), width) for d in self._directions()]
                stack.add(rnn_cell.BidirectionalCell(*cells) if len(cells) == 2 else cells[0])
                if self._dropout > 0 and layer < last:
                    stack.add(rnn_cell.DropoutCell(self._dropout))
                width = self._hidden_size * self._dir
        return stack

    # ------------------------------------------------------------------ execution
    def cast(self, dtype):
        super().cast(dtype)
        self._dtype = dtype

    def begin_state(self, batch_size=0, func=ndarray.zeros, **kwargs):
        symbolic = 'symbol' in getattr(func, '__module__', '')
        states = []
        for i, info in enumerate(self.state_info(batch_size)):
            spec = dict(info or {})
            spec.update(kwargs)
            spec.pop('__layout__', None)
            if symbolic:
                spec.pop('ctx', None)
            states.append(func(name='%sh0_%d' % (self.prefix, i), **spec))
        return states

    def __call__(self, inputs, states=None, sequence_length=None, **kwargs):
        self.skip_states = states is None
        if states is None:
            if isinstance(inputs, NDArray):
                n = inputs.shape[self._layout.index('N')]
                states = self.begin_state(n, ctx=inputs.context, dtype=inputs.dtype)
            else:
                states = self._symbol_begin_state(inputs)
        if isinstance(states, (NDArray, symbol.Symbol)):
            states = [states]
        extra = (sequence_length,) if self._use_sequence_length else ()
        return super().__call__(inputs, states, *extra, **kwargs)

    def hybrid_forward(self, F, inputs, states, sequence_length=None, **kwargs):
        if F is ndarray:
            n = inputs.shape[self._layout.index('N')]
            for got, want in zip(states, self.state_info(n)):
                if got.shape != want['shape']:
                    raise ValueError('Invalid recurrent state shape. Expecting %s, got %s.'
                                     % (str(want['shape']), str(got.shape)))
        out = self._forward_kernel(F, inputs, states, sequence_length, **kwargs)
        return out[0] if self.skip_states else out

    def _forward_kernel(self, F, inputs, states, sequence_length, **kwargs):
        time_major = self._layout == 'TNC'
        if not time_major:
            inputs = F.swapaxes(inputs, dim1=0, dim2=1)
        flat = F._internal._rnn_param_concat(*[kwargs[n].reshape(-1) for n in self._flat_order()], dim=0)
        args = list(states)
        if self._use_sequence_length:
            args.append(sequence_length)
        res = F.RNN(inputs, flat, *args, use_sequence_length=self._use_sequence_length,
                    state_size=self._hidden_size, projection_size=self._projection_size,
                    num_layers=self._num_layers, bidirectional=self._dir == 2, p=self._dropout, state_outputs=True,
                    mode=self._mode, lstm_state_clip_min=self._lstm_state_clip_min,
                    lstm_state_clip_max=self._lstm_state_clip_max, lstm_state_clip_nan=self._lstm_state_clip_nan)
        nstate = 2 if self._mode == 'lstm' else 1
        outputs, new_states = res[0], [res[1 + i] for i in range(nstate)]
        if not time_major:
            outputs = F.swapaxes(outputs, dim1=0, dim2=1)
        return outputs, new_states


class RNN(_RNNLayer):
    """Multi-layer Elman RNN with tanh or ReLU non-linearity."""

    def __init__(self, hidden_size, num_layers=1, activation='relu', layout='TNC', dropout=0, bidirectional=False,
                 i2h_weight_initializer=None, h2h_weight_initializer=None, i2h_bias_initializer='zeros',
                 h2h_bias_initializer='zeros', input_size=0, dtype='float32', **kwargs):
        super().__init__(hidden_size, num_layers, layout, dropout, bidirectional, input_size,
                         i2h_weight_initializer, h2h_weight_initializer, i2h_bias_initializer, h2h_bias_initializer,
                         'rnn_' + activation, None, None, None, None, False, dtype, **kwargs)

    def state_info(self, batch_size=0):
        return [self._state_spec(batch_size, self._hidden_size)]


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
        h = self._projection_size or self._hidden_size
        return [self._state_spec(batch_size, h), self._state_spec(batch_size, self._hidden_size)]


class GRU(_RNNLayer):
    """Multi-layer GRU."""

    def __init__(self, hidden_size, num_layers=1, layout='TNC', dropout=0, bidirectional=False, input_size=0,
                 i2h_weight_initializer=None, h2h_weight_initializer=None, i2h_bias_initializer='zeros',
                 h2h_bias_initializer='zeros', dtype='float32', **kwargs):
        super().__init__(hidden_size, num_layers, layout, dropout, bidirectional, input_size,
                         i2h_weight_initializer, h2h_weight_initializer, i2h_bias_initializer, h2h_bias_initializer,
                         'gru', None, None, None, None, False, dtype, **kwargs)

    def state_info(self, batch_size=0):
        return [self._state_spec(batch_size, self._hidden_size)]
