"""Convolutional recurrent cells (parity: python/mxnet/gluon/contrib/rnn/conv_rnn_cell.py).

ConvRNN / ConvLSTM (Shi et al. 2015) / ConvGRU in 1, 2 and 3 spatial dims: the
input-to-hidden and hidden-to-hidden transforms are convolutions; the h2h
convolution is 'same'-padded (odd kernel) so the state keeps its spatial shape.
"""
from ...rnn.rnn_cell import HybridRecurrentCell

__all__ = ['Conv1DRNNCell', 'Conv2DRNNCell', 'Conv3DRNNCell', 'Conv1DLSTMCell', 'Conv2DLSTMCell',
           'Conv3DLSTMCell', 'Conv1DGRUCell', 'Conv2DGRUCell', 'Conv3DGRUCell']


def _tup(v, n):
    return (v,) * n if isinstance(v, int) else tuple(v)


class _BaseConvRNNCell(HybridRecurrentCell):
    def __init__(self, input_shape, hidden_channels, i2h_kernel, h2h_kernel, i2h_pad, i2h_dilate, h2h_dilate,
                 i2h_weight_initializer, h2h_weight_initializer, i2h_bias_initializer, h2h_bias_initializer, dims,
                 conv_layout, activation, prefix=None, params=None, num_gates=1):
        super().__init__(prefix=prefix, params=params)
        self._hidden_channels = hidden_channels
        self._input_shape = tuple(input_shape)
        self._conv_layout = conv_layout
        self._activation = activation
        self._dims = dims
        self._i2h_kernel = _tup(i2h_kernel, dims)
        self._h2h_kernel = _tup(h2h_kernel, dims)
        assert all(k % 2 == 1 for k in self._h2h_kernel), \
            'Only support odd number, get h2h_kernel= %s' % str(self._h2h_kernel)
        self._i2h_pad = _tup(i2h_pad, dims)
        self._i2h_dilate = _tup(i2h_dilate, dims)
        self._h2h_dilate = _tup(h2h_dilate, dims)
        self._h2h_pad = tuple(d * (k - 1) // 2 for d, k in zip(self._h2h_dilate, self._h2h_kernel))
        channel_axis = conv_layout.find('C')
        in_channels = self._input_shape[channel_axis - 1] if channel_axis > 0 else self._input_shape[0]
        spatial = [s for i, s in enumerate(self._input_shape) if i != channel_axis - 1]
        self._state_spatial = tuple((s + 2 * p - d * (k - 1) - 1) + 1 for s, p, d, k in
                                    zip(spatial, self._i2h_pad, self._i2h_dilate, self._i2h_kernel))
        ng = num_gates
        self.i2h_weight = self.params.get('i2h_weight', shape=(hidden_channels * ng, in_channels) + self._i2h_kernel,
                                          init=i2h_weight_initializer, allow_deferred_init=True)
        self.h2h_weight = self.params.get('h2h_weight',
                                          shape=(hidden_channels * ng, hidden_channels) + self._h2h_kernel,
                                          init=h2h_weight_initializer, allow_deferred_init=True)
        self.i2h_bias = self.params.get('i2h_bias', shape=(hidden_channels * ng,), init=i2h_bias_initializer,
                                        allow_deferred_init=True)
        self.h2h_bias = self.params.get('h2h_bias', shape=(hidden_channels * ng,), init=h2h_bias_initializer,
                                        allow_deferred_init=True)
        self._num_gates = ng

    def _state_shape(self, batch_size):
        if self._conv_layout.find('C') == 1:
            return (batch_size, self._hidden_channels) + self._state_spatial
        return (batch_size,) + self._state_spatial + (self._hidden_channels,)

    def state_info(self, batch_size=0):
        return [{'shape': self._state_shape(batch_size), '__layout__': self._conv_layout}]

    def _conv_forward(self, F, inputs, states, i2h_weight, h2h_weight, i2h_bias, h2h_bias, name):
        nf = self._hidden_channels * self._num_gates
        i2h = F.Convolution(data=inputs, num_filter=nf, kernel=self._i2h_kernel, pad=self._i2h_pad,
                            dilate=self._i2h_dilate, weight=i2h_weight, bias=i2h_bias, layout=self._conv_layout,
                            name=name + 'i2h')
        h2h = F.Convolution(data=states[0], num_filter=nf, kernel=self._h2h_kernel, pad=self._h2h_pad,
                            dilate=self._h2h_dilate, weight=h2h_weight, bias=h2h_bias, layout=self._conv_layout,
                            name=name + 'h2h')
        return i2h, h2h

    def _caxis(self):
        return self._conv_layout.find('C')


class _ConvRNNCell(_BaseConvRNNCell):
    def _alias(self):
        return 'conv_rnn'

    def hybrid_forward(self, F, inputs, states, i2h_weight, h2h_weight, i2h_bias, h2h_bias):
        prefix = 't%d_' % self._counter
        i2h, h2h = self._conv_forward(F, inputs, states, i2h_weight, h2h_weight, i2h_bias, h2h_bias, prefix)
        output = self._get_activation(F, i2h + h2h, self._activation, name=prefix + 'out')
        return output, [output]


class _ConvLSTMCell(_BaseConvRNNCell):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, num_gates=4, **kwargs)

    def _alias(self):
        return 'conv_lstm'

    def state_info(self, batch_size=0):
        s = self._state_shape(batch_size)
        return [{'shape': s, '__layout__': self._conv_layout}, {'shape': s, '__layout__': self._conv_layout}]

    def hybrid_forward(self, F, inputs, states, i2h_weight, h2h_weight, i2h_bias, h2h_bias):
        prefix = 't%d_' % self._counter
        i2h, h2h = self._conv_forward(F, inputs, states, i2h_weight, h2h_weight, i2h_bias, h2h_bias, prefix)
        gates = i2h + h2h
        sg = F.SliceChannel(gates, num_outputs=4, axis=self._caxis(), name=prefix + 'slice')
        in_gate = F.Activation(sg[0], act_type='sigmoid')
        forget_gate = F.Activation(sg[1], act_type='sigmoid')
        in_transform = self._get_activation(F, sg[2], self._activation)
        out_gate = F.Activation(sg[3], act_type='sigmoid')
        next_c = forget_gate * states[1] + in_gate * in_transform
        next_h = F.elemwise_mul(out_gate, self._get_activation(F, next_c, self._activation), name=prefix + 'out')
        return next_h, [next_h, next_c]


class _ConvGRUCell(_BaseConvRNNCell):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, num_gates=3, **kwargs)

    def _alias(self):
        return 'conv_gru'

    def hybrid_forward(self, F, inputs, states, i2h_weight, h2h_weight, i2h_bias, h2h_bias):
        prefix = 't%d_' % self._counter
        i2h, h2h = self._conv_forward(F, inputs, states, i2h_weight, h2h_weight, i2h_bias, h2h_bias, prefix)
        ax = self._caxis()
        i2h_r, i2h_z, i2h = F.SliceChannel(i2h, num_outputs=3, axis=ax, name=prefix + 'i2h_slice')
        h2h_r, h2h_z, h2h = F.SliceChannel(h2h, num_outputs=3, axis=ax, name=prefix + 'h2h_slice')
        reset_gate = F.Activation(i2h_r + h2h_r, act_type='sigmoid')
        update_gate = F.Activation(i2h_z + h2h_z, act_type='sigmoid')
        next_h_tmp = self._get_activation(F, i2h + reset_gate * h2h, self._activation)
        next_h = F.elemwise_add((1. - update_gate) * next_h_tmp, update_gate * states[0], name=prefix + 'out')
        return next_h, [next_h]


def _make(base, dims, layout, default_act):
    class Cell(base):
        def __init__(self, input_shape, hidden_channels, i2h_kernel, h2h_kernel, i2h_pad=(0,) * dims,
                     i2h_dilate=(1,) * dims, h2h_dilate=(1,) * dims, i2h_weight_initializer=None,
                     h2h_weight_initializer=None, i2h_bias_initializer='zeros', h2h_bias_initializer='zeros',
                     conv_layout=layout, activation=default_act, prefix=None, params=None):
            super().__init__(input_shape=input_shape, hidden_channels=hidden_channels, i2h_kernel=i2h_kernel,
                             h2h_kernel=h2h_kernel, i2h_pad=i2h_pad, i2h_dilate=i2h_dilate, h2h_dilate=h2h_dilate,
                             i2h_weight_initializer=i2h_weight_initializer,
                             h2h_weight_initializer=h2h_weight_initializer, i2h_bias_initializer=i2h_bias_initializer,
                             h2h_bias_initializer=h2h_bias_initializer, dims=dims, conv_layout=conv_layout,
                             activation=activation, prefix=prefix, params=params)
    return Cell


Conv1DRNNCell = _make(_ConvRNNCell, 1, 'NCW', 'tanh')
Conv2DRNNCell = _make(_ConvRNNCell, 2, 'NCHW', 'tanh')
Conv3DRNNCell = _make(_ConvRNNCell, 3, 'NCDHW', 'tanh')
Conv1DLSTMCell = _make(_ConvLSTMCell, 1, 'NCW', 'tanh')
Conv2DLSTMCell = _make(_ConvLSTMCell, 2, 'NCHW', 'tanh')
Conv3DLSTMCell = _make(_ConvLSTMCell, 3, 'NCDHW', 'tanh')
Conv1DGRUCell = _make(_ConvGRUCell, 1, 'NCW', 'tanh')
Conv2DGRUCell = _make(_ConvGRUCell, 2, 'NCHW', 'tanh')
Conv3DGRUCell = _make(_ConvGRUCell, 3, 'NCDHW', 'tanh')
for _n in __all__:
    globals()[_n].__name__ = _n
    globals()[_n].__qualname__ = _n
