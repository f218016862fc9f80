"""Convolution and pooling layers.

Parity: python/mxnet/gluon/nn/conv_layers.py (_Conv, Conv1D/2D/3D,
Conv1D/2D/3DTranspose, _Pooling, Max/Avg/GlobalMax/GlobalAvg Pool 1/2/3D,
ReflectionPad2D).  ``layout='NHWC'`` (weights OHWI) is the MI355X fast path.
"""
from ..block import HybridBlock
from .activations import Activation

__all__ = ['Conv1D', 'Conv2D', 'Conv3D', 'Conv1DTranspose', 'Conv2DTranspose', 'Conv3DTranspose',
           'MaxPool1D', 'MaxPool2D', 'MaxPool3D', 'AvgPool1D', 'AvgPool2D', 'AvgPool3D',
           'GlobalMaxPool1D', 'GlobalMaxPool2D', 'GlobalMaxPool3D', 'GlobalAvgPool1D', 'GlobalAvgPool2D',
           'GlobalAvgPool3D', 'ReflectionPad2D']


def _infer_weight_shape(op_name, data_shape, kwargs):
    from ... import symbol
    op = getattr(symbol, op_name)
    sym = op(symbol.var('data', shape=data_shape), **kwargs)
    return sym.infer_shape_partial()[0]


class _Conv(HybridBlock):
    def __init__(self, channels, kernel_size, strides, padding, dilation, groups, layout, in_channels=0,
                 activation=None, use_bias=True, weight_initializer=None, bias_initializer='zeros',
                 op_name='Convolution', adj=None, prefix=None, params=None):
        super().__init__(prefix=prefix, params=params)
        with self.name_scope():
            self._channels = channels
            self._in_channels = in_channels
            if isinstance(strides, int):
                strides = (strides,) * len(kernel_size)
            if isinstance(padding, int):
                padding = (padding,) * len(kernel_size)
            if isinstance(dilation, int):
                dilation = (dilation,) * len(kernel_size)
            self._op_name = op_name
            self._kwargs = {'kernel': kernel_size, 'stride': strides, 'dilate': dilation, 'pad': padding,
                            'num_filter': channels, 'num_group': groups, 'no_bias': not use_bias,
                            'layout': layout}
            if adj is not None:
                self._kwargs['adj'] = adj
            nsp = len(kernel_size)
            if layout.endswith('C'):
                if op_name == 'Convolution':
                    wshape = (channels,) + tuple(kernel_size) + (in_channels // groups if in_channels else 0,)
                else:
                    wshape = (in_channels,) + tuple(kernel_size) + (channels // groups,)
            else:
                if op_name == 'Convolution':
                    wshape = (channels, in_channels // groups if in_channels else 0) + tuple(kernel_size)
                else:
                    wshape = (in_channels, channels // groups) + tuple(kernel_size)
            self.weight = self.params.get('weight', shape=wshape, init=weight_initializer,
                                          allow_deferred_init=True)
            if use_bias:
                self.bias = self.params.get('bias', shape=(channels,), init=bias_initializer,
                                            allow_deferred_init=True)
            else:
                self.bias = None
            if activation is not None:
                self.act = Activation(activation, prefix=activation + '_')
            else:
                self.act = None

    def hybrid_forward(self, F, x, weight, bias=None):
        if getattr(self, '_tee', False) and bias is None and self.act is None:
            # (conv(x), x): identity-shortcut pass-through fused into the backward GEMM
            return F.contrib.ConvolutionTee(x, weight, name='fwd', inplace_shortcut_grad=True, **self._kwargs)
        if bias is None:
            act = getattr(F, self._op_name)(x, weight, name='fwd', **self._kwargs)
        else:
            act = getattr(F, self._op_name)(x, weight, bias, name='fwd', **self._kwargs)
        if self.act is not None:
            act = self.act(act)
        return act

    def _alias(self):
        return 'conv'

    def __repr__(self):
        s = '{name}({mapping}, kernel_size={kernel}, stride={stride}'
        len_kernel_size = len(self._kwargs['kernel'])
        if self._kwargs['pad'] != (0,) * len_kernel_size:
            s += ', padding={pad}'
        if self._kwargs['dilate'] != (1,) * len_kernel_size:
            s += ', dilation={dilate}'
        if hasattr(self, 'out_pad') and self.out_pad != (0,) * len_kernel_size:
            s += ', output_padding={out_pad}'.format(out_pad=self.out_pad)
        if self._kwargs['num_group'] != 1:
            s += ', groups={num_group}'
        if self.bias is None:
            s += ', bias=False'
        if self.act:
            s += ', {}'.format(self.act)
        s += ')'
        shape = self.weight.shape
        in_c = shape[-1] if self._kwargs['layout'].endswith('C') else shape[1]
        return s.format(name=self.__class__.__name__,
                        mapping='{0} -> {1}'.format(in_c if in_c else None, shape[0]), **self._kwargs)


class Conv1D(_Conv):
    def __init__(self, channels, kernel_size, strides=1, padding=0, dilation=1, groups=1, layout='NCW',
                 activation=None, use_bias=True, weight_initializer=None, bias_initializer='zeros',
                 in_channels=0, **kwargs):
        assert layout in ('NCW', 'NWC'), 'Only supports NCW and NWC layout for now'
        if isinstance(kernel_size, int):
            kernel_size = (kernel_size,)
        assert len(kernel_size) == 1, 'kernel_size must be a number or a list of 1 ints'
        super().__init__(channels, kernel_size, strides, padding, dilation, groups, layout, in_channels,
                         activation, use_bias, weight_initializer, bias_initializer, **kwargs)


class Conv2D(_Conv):
    def __init__(self, channels, kernel_size, strides=(1, 1), padding=(0, 0), dilation=(1, 1), groups=1,
                 layout='NCHW', activation=None, use_bias=True, weight_initializer=None, bias_initializer='zeros',
                 in_channels=0, **kwargs):
        assert layout in ('NCHW', 'NHWC'), 'Only supports NCHW and NHWC layout for now'
        if isinstance(kernel_size, int):
            kernel_size = (kernel_size,) * 2
        assert len(kernel_size) == 2, 'kernel_size must be a number or a list of 2 ints'
        super().__init__(channels, kernel_size, strides, padding, dilation, groups, layout, in_channels,
                         activation, use_bias, weight_initializer, bias_initializer, **kwargs)


class Conv3D(_Conv):
    def __init__(self, channels, kernel_size, strides=(1, 1, 1), padding=(0, 0, 0), dilation=(1, 1, 1), groups=1,
                 layout='NCDHW', activation=None, use_bias=True, weight_initializer=None, bias_initializer='zeros',
                 in_channels=0, **kwargs):
        assert layout in ('NCDHW', 'NDHWC'), 'Only supports NCDHW and NDHWC layout for now'
        if isinstance(kernel_size, int):
            kernel_size = (kernel_size,) * 3
        assert len(kernel_size) == 3, 'kernel_size must be a number or a list of 3 ints'
        super().__init__(channels, kernel_size, strides, padding, dilation, groups, layout, in_channels,
                         activation, use_bias, weight_initializer, bias_initializer, **kwargs)


class Conv1DTranspose(_Conv):
    def __init__(self, channels, kernel_size, strides=1, padding=0, output_padding=0, dilation=1, groups=1,
                 layout='NCW', activation=None, use_bias=True, weight_initializer=None, bias_initializer='zeros',
                 in_channels=0, **kwargs):
        assert layout in ('NCW', 'NWC'), 'Only supports NCW and NWC layout for now'
        if isinstance(kernel_size, int):
            kernel_size = (kernel_size,)
        if isinstance(output_padding, int):
            output_padding = (output_padding,)
        super().__init__(channels, kernel_size, strides, padding, dilation, groups, layout, in_channels,
                         activation, use_bias, weight_initializer, bias_initializer, op_name='Deconvolution',
                         adj=output_padding, **kwargs)
        self.outpad = output_padding


class Conv2DTranspose(_Conv):
    def __init__(self, channels, kernel_size, strides=(1, 1), padding=(0, 0), output_padding=(0, 0),
                 dilation=(1, 1), groups=1, layout='NCHW', activation=None, use_bias=True, weight_initializer=None,
                 bias_initializer='zeros', in_channels=0, **kwargs):
        assert layout in ('NCHW', 'NHWC'), 'Only supports NCHW and NHWC layout for now'
        if isinstance(kernel_size, int):
            kernel_size = (kernel_size,) * 2
        if isinstance(output_padding, int):
            output_padding = (output_padding,) * 2
        super().__init__(channels, kernel_size, strides, padding, dilation, groups, layout, in_channels,
                         activation, use_bias, weight_initializer, bias_initializer, op_name='Deconvolution',
                         adj=output_padding, **kwargs)
        self.outpad = output_padding


class Conv3DTranspose(_Conv):
    def __init__(self, channels, kernel_size, strides=(1, 1, 1), padding=(0, 0, 0), output_padding=(0, 0, 0),
                 dilation=(1, 1, 1), groups=1, layout='NCDHW', activation=None, use_bias=True,
                 weight_initializer=None, bias_initializer='zeros', in_channels=0, **kwargs):
        assert layout in ('NCDHW', 'NDHWC'), 'Only supports NCDHW and NDHWC layout for now'
        if isinstance(kernel_size, int):
            kernel_size = (kernel_size,) * 3
        if isinstance(output_padding, int):
            output_padding = (output_padding,) * 3
        super().__init__(channels, kernel_size, strides, padding, dilation, groups, layout, in_channels,
                         activation, use_bias, weight_initializer, bias_initializer, op_name='Deconvolution',
                         adj=output_padding, **kwargs)
        self.outpad = output_padding


class _Pooling(HybridBlock):
    def __init__(self, pool_size, strides, padding, ceil_mode, global_pool, pool_type, layout,
                 count_include_pad=None, **kwargs):
        super().__init__(**kwargs)
        if strides is None:
            strides = pool_size
        if isinstance(strides, int):
            strides = (strides,) * len(pool_size)
        if isinstance(padding, int):
            padding = (padding,) * len(pool_size)
        self._kwargs = {'kernel': pool_size, 'stride': strides, 'pad': padding, 'global_pool': global_pool,
                        'pool_type': pool_type, 'layout': layout,
                        'pooling_convention': 'full' if ceil_mode else 'valid'}
        if count_include_pad is not None:
            self._kwargs['count_include_pad'] = count_include_pad

    def _alias(self):
        return 'pool'

    def hybrid_forward(self, F, x):
        return F.Pooling(x, name='fwd', **self._kwargs)

    def __repr__(self):
        s = '{name}(size={kernel}, stride={stride}, padding={pad}, ceil_mode={ceil_mode}'
        s += ', global_pool={global_pool}, pool_type={pool_type}, layout={layout})'
        return s.format(name=self.__class__.__name__,
                        ceil_mode=self._kwargs['pooling_convention'] == 'full', **self._kwargs)


def _pool_cls(nsp, pool_type, name, default_layout, glob=False):
    if glob:
        def __init__(self, layout=default_layout, **kwargs):
            _Pooling.__init__(self, (1,) * nsp, None, 0, True, True, pool_type, layout, **kwargs)
    elif pool_type == 'avg':
        def __init__(self, pool_size=(2,) * nsp if nsp > 1 else 2, strides=None, padding=0, ceil_mode=False,
                     layout=default_layout, count_include_pad=True, **kwargs):
            if isinstance(pool_size, int):
                pool_size = (pool_size,) * nsp
            _Pooling.__init__(self, pool_size, strides, padding, ceil_mode, False, 'avg', layout,
                              count_include_pad, **kwargs)
    else:
        def __init__(self, pool_size=(2,) * nsp if nsp > 1 else 2, strides=None, padding=0, layout=default_layout,
                     ceil_mode=False, **kwargs):
            if isinstance(pool_size, int):
                pool_size = (pool_size,) * nsp
            _Pooling.__init__(self, pool_size, strides, padding, ceil_mode, False, 'max', layout, **kwargs)
    return type(name, (_Pooling,), {'__init__': __init__, '__doc__': '%s pooling (%dD).' % (pool_type, nsp)})


MaxPool1D = _pool_cls(1, 'max', 'MaxPool1D', 'NCW')
MaxPool2D = _pool_cls(2, 'max', 'MaxPool2D', 'NCHW')
MaxPool3D = _pool_cls(3, 'max', 'MaxPool3D', 'NCDHW')
AvgPool1D = _pool_cls(1, 'avg', 'AvgPool1D', 'NCW')
AvgPool2D = _pool_cls(2, 'avg', 'AvgPool2D', 'NCHW')
AvgPool3D = _pool_cls(3, 'avg', 'AvgPool3D', 'NCDHW')
GlobalMaxPool1D = _pool_cls(1, 'max', 'GlobalMaxPool1D', 'NCW', glob=True)
GlobalMaxPool2D = _pool_cls(2, 'max', 'GlobalMaxPool2D', 'NCHW', glob=True)
GlobalMaxPool3D = _pool_cls(3, 'max', 'GlobalMaxPool3D', 'NCDHW', glob=True)
GlobalAvgPool1D = _pool_cls(1, 'avg', 'GlobalAvgPool1D', 'NCW', glob=True)
GlobalAvgPool2D = _pool_cls(2, 'avg', 'GlobalAvgPool2D', 'NCHW', glob=True)
GlobalAvgPool3D = _pool_cls(3, 'avg', 'GlobalAvgPool3D', 'NCDHW', glob=True)


class ReflectionPad2D(HybridBlock):
    def __init__(self, padding=0, **kwargs):
        super().__init__(**kwargs)
        if isinstance(padding, int):
            padding = (0, 0, 0, 0, padding, padding, padding, padding)
        assert len(padding) == 8
        self._padding = padding

    def hybrid_forward(self, F, x):
        return F.pad(x, mode='reflect', pad_width=self._padding)
