"""Deformable convolution blocks (parity: python/mxnet/gluon/contrib/cnn/conv_layers.py).

The offsets (and, for v2, modulation masks) are predicted by a regular
convolution from the same input, initialised to zero so training starts from a
plain convolution.
"""
from ...block import HybridBlock
from ... import nn as _nn

__all__ = ['DeformableConvolution', 'ModulatedDeformableConvolution']


def _tup(v, n=2):
    return (v,) * n if isinstance(v, int) else tuple(v)


class DeformableConvolution(HybridBlock):
    def __init__(self, channels, kernel_size=(1, 1), strides=(1, 1), padding=(0, 0), dilation=(1, 1), groups=1,
                 num_deformable_group=1, layout='NCHW', use_bias=True, in_channels=0, activation=None,
                 weight_initializer=None, bias_initializer='zeros', offset_weight_initializer='zeros',
                 offset_bias_initializer='zeros', offset_use_bias=True, op_name='DeformableConvolution',
                 adj=None, prefix=None, params=None):
        super().__init__(prefix=prefix, params=params)
        assert layout == 'NCHW', 'Only supports NCHW layout for now'
        kernel_size, strides, padding, dilation = (_tup(kernel_size), _tup(strides), _tup(padding), _tup(dilation))
        self._channels = channels
        self._in_channels = in_channels
        offset_channels = 2 * kernel_size[0] * kernel_size[1] * num_deformable_group
        self._kwargs_offset = {'kernel': kernel_size, 'stride': strides, 'dilate': dilation, 'pad': padding,
                               'num_filter': offset_channels, 'num_group': groups, 'no_bias': not offset_use_bias,
                               'layout': layout}
        self._kwargs_deformable_conv = {'kernel': kernel_size, 'stride': strides, 'dilate': dilation,
                                        'pad': padding, 'num_filter': channels, 'num_group': groups,
                                        'num_deformable_group': num_deformable_group, 'no_bias': not use_bias,
                                        'layout': layout}
        wshapes = [(offset_channels, in_channels // groups if in_channels else 0) + kernel_size,
                   (channels, in_channels // groups if in_channels else 0) + kernel_size]
        self.offset_weight = self.params.get('offset_weight', shape=wshapes[0], init=offset_weight_initializer,
                                             allow_deferred_init=True)
        self.offset_bias = self.params.get('offset_bias', shape=(offset_channels,), init=offset_bias_initializer,
                                           allow_deferred_init=True) if offset_use_bias else None
        self.deformable_conv_weight = self.params.get('deformable_conv_weight', shape=wshapes[1],
                                                      init=weight_initializer, allow_deferred_init=True)
        self.deformable_conv_bias = self.params.get('deformable_conv_bias', shape=(channels,),
                                                    init=bias_initializer, allow_deferred_init=True) \
            if use_bias else None
        self.act = _nn.Activation(activation, prefix=activation + '_') if activation else None

    def hybrid_forward(self, F, x, offset_weight, deformable_conv_weight, offset_bias=None,
                       deformable_conv_bias=None):
        if offset_bias is None:
            offset = F.Convolution(x, offset_weight, cudnn_off=True, **self._kwargs_offset)
        else:
            offset = F.Convolution(x, offset_weight, offset_bias, cudnn_off=True, **self._kwargs_offset)
        if deformable_conv_bias is None:
            act = F.contrib.DeformableConvolution(data=x, offset=offset, weight=deformable_conv_weight, name='fwd',
                                                  **self._kwargs_deformable_conv)
        else:
            act = F.contrib.DeformableConvolution(data=x, offset=offset, weight=deformable_conv_weight,
                                                  bias=deformable_conv_bias, name='fwd',
                                                  **self._kwargs_deformable_conv)
        if self.act:
            act = self.act(act)
        return act


class ModulatedDeformableConvolution(HybridBlock):
    def __init__(self, channels, kernel_size=(1, 1), strides=(1, 1), padding=(0, 0), dilation=(1, 1), groups=1,
                 num_deformable_group=1, layout='NCHW', use_bias=True, in_channels=0, activation=None,
                 weight_initializer=None, bias_initializer='zeros', offset_weight_initializer='zeros',
                 offset_bias_initializer='zeros', offset_use_bias=True, op_name='ModulatedDeformableConvolution',
                 adj=None, prefix=None, params=None):
        super().__init__(prefix=prefix, params=params)
        assert layout == 'NCHW', 'Only supports NCHW layout for now'
        kernel_size, strides, padding, dilation = (_tup(kernel_size), _tup(strides), _tup(padding), _tup(dilation))
        self._channels = channels
        K = kernel_size[0] * kernel_size[1]
        self._offset_channels = 3 * K * num_deformable_group
        self._split = 2 * K * num_deformable_group
        self._kwargs_offset = {'kernel': kernel_size, 'stride': strides, 'dilate': dilation, 'pad': padding,
                               'num_filter': self._offset_channels, 'num_group': groups,
                               'no_bias': not offset_use_bias, 'layout': layout}
        self._kwargs_deformable_conv = {'kernel': kernel_size, 'stride': strides, 'dilate': dilation,
                                        'pad': padding, 'num_filter': channels, 'num_group': groups,
                                        'num_deformable_group': num_deformable_group, 'no_bias': not use_bias,
                                        'layout': layout}
        ic = in_channels // groups if in_channels else 0
        self.offset_weight = self.params.get('offset_weight', shape=(self._offset_channels, ic) + kernel_size,
                                             init=offset_weight_initializer, allow_deferred_init=True)
        self.offset_bias = self.params.get('offset_bias', shape=(self._offset_channels,),
                                           init=offset_bias_initializer, allow_deferred_init=True) \
            if offset_use_bias else None
        self.deformable_conv_weight = self.params.get('deformable_conv_weight', shape=(channels, ic) + kernel_size,
                                                      init=weight_initializer, allow_deferred_init=True)
        self.deformable_conv_bias = self.params.get('deformable_conv_bias', shape=(channels,),
                                                    init=bias_initializer, allow_deferred_init=True) \
            if use_bias else None
        self.act = _nn.Activation(activation, prefix=activation + '_') if activation else None

    def hybrid_forward(self, F, x, offset_weight, deformable_conv_weight, offset_bias=None,
                       deformable_conv_bias=None):
        if offset_bias is None:
            om = F.Convolution(x, offset_weight, cudnn_off=True, **self._kwargs_offset)
        else:
            om = F.Convolution(x, offset_weight, offset_bias, cudnn_off=True, **self._kwargs_offset)
        offset = F.slice_axis(om, axis=1, begin=0, end=self._split)
        mask = F.sigmoid(F.slice_axis(om, axis=1, begin=self._split, end=None)) * 2
        kw = dict(data=x, offset=offset, mask=mask, weight=deformable_conv_weight, name='fwd',
                  **self._kwargs_deformable_conv)
        if deformable_conv_bias is not None:
            kw['bias'] = deformable_conv_bias
        act = F.contrib.ModulatedDeformableConvolution(**kw)
        if self.act:
            act = self.act(act)
        return act
