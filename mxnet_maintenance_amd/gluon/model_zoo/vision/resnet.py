"""ResNet V1 / V1b / V2 (18, 34, 50, 101, 152).

Parity: python/mxnet/gluon/model_zoo/vision/resnet.py (BasicBlockV1/V2,
BottleneckV1/V2, ResNetV1/V2, get_resnet, resnet{18..152}_v{1,2}); V1b (stride
on the 3x3 conv of the bottleneck, as in GluonCV) is the benchmark model.

MI355X options (not in the reference signature, defaults keep its behaviour):
``layout='NHWC'`` builds the whole network channel-last (convolutions with OHWI
weights, BatchNorm over the last axis, NHWC pooling) which is the layout the
gfx950 conv/BN kernels are written for; ``fuse=True`` folds every BN+ReLU into
one ``BatchNormWithReLU`` and every bottleneck tail ``relu(BN(x) + shortcut)``
into one ``BatchNormAddReLU`` kernel.
"""
from ... import nn
from ...block import HybridBlock
from ...nn.basic_layers import _BatchNorm
from ....context import cpu

__all__ = ['ResNetV1', 'ResNetV2', 'BasicBlockV1', 'BasicBlockV2', 'BottleneckV1', 'BottleneckV2',
           'BottleneckV1b', 'resnet18_v1', 'resnet34_v1', 'resnet50_v1', 'resnet101_v1', 'resnet152_v1',
           'resnet18_v2', 'resnet34_v2', 'resnet50_v2', 'resnet101_v2', 'resnet152_v2', 'resnet50_v1b',
           'resnet101_v1b', 'resnet152_v1b', 'resnet18_v1b', 'resnet34_v1b', 'get_resnet']


def _bn_axis(layout):
    return 3 if layout == 'NHWC' else 1


def _conv(channels, k, stride, pad, in_channels, layout, use_bias=False):
    return nn.Conv2D(channels, kernel_size=k, strides=stride, padding=pad, use_bias=use_bias,
                     in_channels=in_channels, layout=layout)


def _bn(layout, relu=False, fuse=False, **kw):
    if relu and fuse:
        return nn.BatchNormReLU(axis=_bn_axis(layout), **kw)
    return nn.BatchNorm(axis=_bn_axis(layout), **kw)


class _StemBNReLUPool(nn.BatchNormReLU):
    """The stem's BatchNorm + ReLU + 3x3/2 max pooling as one operator (``fuse=True``, NHWC): the pooling
    kernel normalises each window tap itself, so the 112x112 normalised activation is never written or
    re-read (ops/nn.py ``_contrib_BatchNormReLUMaxPool``). Same parameters as BatchNormReLU."""

    def hybrid_forward(self, F, x, gamma, beta, running_mean, running_var):
        return F.contrib.BatchNormReLUMaxPool(x, gamma, beta, running_mean, running_var, name='fwd',
                                              kernel=(3, 3), stride=(2, 2), pad=(1, 1), **self._kwargs)


def _stem_tail(features, layout, fuse):
    """BatchNorm + ReLU + max pooling after the 7x7 stem convolution."""
    if fuse and layout == 'NHWC':
        features.add(_StemBNReLUPool(axis=_bn_axis(layout)))
        return
    features.add(_bn(layout, True, fuse))
    if not fuse:
        features.add(nn.Activation('relu'))
    features.add(nn.MaxPool2D(3, 2, 1, layout=layout))


class _ResidualTail(_BatchNorm):
    """relu(BN(x) + shortcut) of a residual block: one fused HIP kernel when ``fuse``; otherwise this
    block is the plain BN and the owning residual block adds and activates (``_finish``), so the
    add / relu symbols are named in the stage's scope as in the reference model zoo
    (``..._stage1_activation0``)."""

    def __init__(self, layout, fuse, **kwargs):
        super().__init__(axis=_bn_axis(layout), **kwargs)
        self._fuse_add = fuse

    def _alias(self):
        return 'batchnorm'

    def hybrid_forward(self, F, x, shortcut, gamma, beta, running_mean, running_var):
        if self._fuse_add:
            return F.contrib.BatchNormAddReLU(x, shortcut, gamma, beta, running_mean, running_var, name='fwd',
                                              **self._kwargs)
        return F.BatchNorm(x, gamma, beta, running_mean, running_var, name='fwd', **self._kwargs)


def _finish(F, tail, out, shortcut):
    y = tail(out, shortcut)
    return y if tail._fuse_add else F.Activation(y + shortcut, act_type='relu')


class BasicBlockV1(HybridBlock):
    """Two 3x3 convs + identity/projection shortcut (ResNet-18/34 V1)."""

    def __init__(self, channels, stride, downsample=False, in_channels=0, layout='NCHW', fuse=False, **kwargs):
        super().__init__(**kwargs)
        self.body = nn.HybridSequential(prefix='')
        self.body.add(_conv(channels, 3, stride, 1, in_channels, layout),
                      _bn(layout, True, fuse))
        if not fuse:
            self.body.add(nn.Activation('relu'))
        self.body.add(_conv(channels, 3, 1, 1, channels, layout))
        self.tail = _ResidualTail(layout, fuse)
        self.downsample = None
        if downsample:
            self.downsample = nn.HybridSequential(prefix='')
            self.downsample.add(_conv(channels, 1, stride, 0, in_channels, layout), _bn(layout))

    def hybrid_forward(self, F, x):
        shortcut = self.downsample(x) if self.downsample is not None else x
        return _finish(F, self.tail, self.body(x), shortcut)


class BottleneckV1(HybridBlock):
    """1x1 -> 3x3 -> 1x1 bottleneck (ResNet-50+ V1).  ``stride_on_3x3`` gives V1b."""

    def __init__(self, channels, stride, downsample=False, in_channels=0, layout='NCHW', fuse=False,
                 stride_on_3x3=False, **kwargs):
        super().__init__(**kwargs)
        mid = channels // 4
        s1, s3 = (1, stride) if stride_on_3x3 else (stride, 1)
        self.body = nn.HybridSequential(prefix='')
        self.body.add(_conv(mid, 1, s1, 0, in_channels, layout), _bn(layout, True, fuse))
        if not fuse:
            self.body.add(nn.Activation('relu'))
        self.body.add(_conv(mid, 3, s3, 1, mid, layout), _bn(layout, True, fuse))
        if not fuse:
            self.body.add(nn.Activation('relu'))
        self.body.add(_conv(channels, 1, 1, 0, mid, layout))
        self.tail = _ResidualTail(layout, fuse)
        self.downsample = None
        if downsample:
            self.downsample = nn.HybridSequential(prefix='')
            self.downsample.add(_conv(channels, 1, stride, 0, in_channels, layout), _bn(layout))
        # channel-last 1x1/stride-1 first conv: that conv also emits x for the shortcut branch, so
        # the shortcut's gradient (identity: the tail's d_addend; projection: the downsample conv's
        # dgrad) is folded into this conv's dgrad GEMM (ConvolutionTee, beta = 1) instead of autograd
        # adding two activation-sized gradients in a separate kernel
        self._tee = fuse and s1 == 1 and layout == 'NHWC'
        if self._tee:
            self.body[0]._tee = True

    def hybrid_forward(self, F, x):
        if self._tee:
            blocks = list(self.body._children.values())
            out, passthrough = blocks[0](x)
            for b in blocks[1:]:
                out = b(out)
            shortcut = self.downsample(passthrough) if self.downsample is not None else passthrough
            return _finish(F, self.tail, out, shortcut)
        shortcut = self.downsample(x) if self.downsample is not None else x
        return _finish(F, self.tail, self.body(x), shortcut)


class BottleneckV1b(BottleneckV1):
    def __init__(self, channels, stride, downsample=False, in_channels=0, layout='NCHW', fuse=False, **kwargs):
        super().__init__(channels, stride, downsample, in_channels, layout, fuse, stride_on_3x3=True, **kwargs)


class BasicBlockV2(HybridBlock):
    """Pre-activation basic block (ResNet V2)."""

    def __init__(self, channels, stride, downsample=False, in_channels=0, layout='NCHW', fuse=False, **kwargs):
        super().__init__(**kwargs)
        self.bn1 = _bn(layout, True, fuse)
        self.conv1 = _conv(channels, 3, stride, 1, in_channels, layout)
        self.bn2 = _bn(layout, True, fuse)
        self.conv2 = _conv(channels, 3, 1, 1, channels, layout)
        self._fused = fuse
        self.downsample = _conv(channels, 1, stride, 0, in_channels, layout) if downsample else None

    def _act(self, F, x, bn):
        x = bn(x)
        return x if self._fused else F.Activation(x, act_type='relu')

    def hybrid_forward(self, F, x):
        shortcut = x
        x = self._act(F, x, self.bn1)
        if self.downsample is not None:
            shortcut = self.downsample(x)
        x = self.conv1(x)
        x = self.conv2(self._act(F, x, self.bn2))
        return x + shortcut


class BottleneckV2(HybridBlock):
    """Pre-activation bottleneck (ResNet V2, 50+ layers)."""

    def __init__(self, channels, stride, downsample=False, in_channels=0, layout='NCHW', fuse=False, **kwargs):
        super().__init__(**kwargs)
        mid = channels // 4
        self.bn1 = _bn(layout, True, fuse)
        self.conv1 = _conv(mid, 1, 1, 0, 0, layout)
        self.bn2 = _bn(layout, True, fuse)
        self.conv2 = _conv(mid, 3, stride, 1, mid, layout)
        self.bn3 = _bn(layout, True, fuse)
        self.conv3 = _conv(channels, 1, 1, 0, 0, layout)
        self._fused = fuse
        self.downsample = _conv(channels, 1, stride, 0, in_channels, layout) if downsample else None

    def _act(self, F, x, bn):
        x = bn(x)
        return x if self._fused else F.Activation(x, act_type='relu')

    def hybrid_forward(self, F, x):
        shortcut = x
        x = self._act(F, x, self.bn1)
        if self.downsample is not None:
            shortcut = self.downsample(x)
        x = self.conv1(x)
        x = self.conv2(self._act(F, x, self.bn2))
        x = self.conv3(self._act(F, x, self.bn3))
        return x + shortcut


class _ResNetBase(HybridBlock):
    def _stage(self, block, n, channels, stride, index, in_channels, layout, fuse):
        stage = nn.HybridSequential(prefix='stage%d_' % index)
        with stage.name_scope():
            stage.add(block(channels, stride, channels != in_channels, in_channels=in_channels, layout=layout,
                            fuse=fuse, prefix=''))
            for _ in range(n - 1):
                stage.add(block(channels, 1, False, in_channels=channels, layout=layout, fuse=fuse, prefix=''))
        return stage


class ResNetV1(_ResNetBase):
    """ResNet V1 (He et al. 2015)."""

    def __init__(self, block, layers, channels, classes=1000, thumbnail=False, layout='NCHW', fuse=False,
                 **kwargs):
        super().__init__(**kwargs)
        assert len(layers) == len(channels) - 1
        self._layout = layout
        with self.name_scope():
            self.features = nn.HybridSequential(prefix='')
            if thumbnail:
                self.features.add(_conv(channels[0], 3, 1, 1, 0, layout))
            else:
                self.features.add(_conv(channels[0], 7, 2, 3, 0, layout))
                _stem_tail(self.features, layout, fuse)
            for i, n in enumerate(layers):
                self.features.add(self._stage(block, n, channels[i + 1], 1 if i == 0 else 2, i + 1,
                                              channels[i], layout, fuse))
            self.features.add(nn.GlobalAvgPool2D(layout=layout))
            self.output = nn.Dense(classes, in_units=channels[-1])

    def hybrid_forward(self, F, x):
        return self.output(self.features(x))


class ResNetV2(_ResNetBase):
    """ResNet V2 (He et al. 2016, pre-activation)."""

    def __init__(self, block, layers, channels, classes=1000, thumbnail=False, layout='NCHW', fuse=False,
                 **kwargs):
        super().__init__(**kwargs)
        assert len(layers) == len(channels) - 1
        with self.name_scope():
            self.features = nn.HybridSequential(prefix='')
            self.features.add(nn.BatchNorm(scale=False, center=False, axis=_bn_axis(layout)))
            if thumbnail:
                self.features.add(_conv(channels[0], 3, 1, 1, 0, layout))
            else:
                self.features.add(_conv(channels[0], 7, 2, 3, 0, layout))
                _stem_tail(self.features, layout, fuse)
            in_channels = channels[0]
            for i, n in enumerate(layers):
                self.features.add(self._stage(block, n, channels[i + 1], 1 if i == 0 else 2, i + 1,
                                              in_channels, layout, fuse))
                in_channels = channels[i + 1]
            self.features.add(_bn(layout, True, fuse))
            if not fuse:
                self.features.add(nn.Activation('relu'))
            self.features.add(nn.GlobalAvgPool2D(layout=layout))
            self.features.add(nn.Flatten())
            self.output = nn.Dense(classes, in_units=in_channels)

    def hybrid_forward(self, F, x):
        return self.output(self.features(x))


resnet_spec = {18: ('basic_block', [2, 2, 2, 2], [64, 64, 128, 256, 512]),
               34: ('basic_block', [3, 4, 6, 3], [64, 64, 128, 256, 512]),
               50: ('bottle_neck', [3, 4, 6, 3], [64, 256, 512, 1024, 2048]),
               101: ('bottle_neck', [3, 4, 23, 3], [64, 256, 512, 1024, 2048]),
               152: ('bottle_neck', [3, 8, 36, 3], [64, 256, 512, 1024, 2048])}
resnet_net_versions = [ResNetV1, ResNetV2]
resnet_block_versions = [{'basic_block': BasicBlockV1, 'bottle_neck': BottleneckV1},
                         {'basic_block': BasicBlockV2, 'bottle_neck': BottleneckV2}]


def get_resnet(version, num_layers, pretrained=False, ctx=cpu(), root='~/.mxnet/models', v1b=False, **kwargs):
    assert num_layers in resnet_spec, 'Invalid number of layers: %d. Options are %s' % (
        num_layers, str(resnet_spec.keys()))
    block_type, layers, channels = resnet_spec[num_layers]
    assert 1 <= version <= 2, 'Invalid resnet version: %d. Options are 1 and 2.' % version
    resnet_class = resnet_net_versions[version - 1]
    block_class = resnet_block_versions[version - 1][block_type]
    if v1b and block_type == 'bottle_neck':
        block_class = BottleneckV1b
    net = resnet_class(block_class, layers, channels, **kwargs)
    if pretrained:
        from ..model_store import get_model_file
        net.load_parameters(get_model_file('resnet%d_v%d' % (num_layers, version), root=root), ctx=ctx)
    return net


def resnet18_v1(**kwargs):
    return get_resnet(1, 18, **kwargs)


def resnet34_v1(**kwargs):
    return get_resnet(1, 34, **kwargs)


def resnet50_v1(**kwargs):
    return get_resnet(1, 50, **kwargs)


def resnet101_v1(**kwargs):
    return get_resnet(1, 101, **kwargs)


def resnet152_v1(**kwargs):
    return get_resnet(1, 152, **kwargs)


def resnet18_v2(**kwargs):
    return get_resnet(2, 18, **kwargs)


def resnet34_v2(**kwargs):
    return get_resnet(2, 34, **kwargs)


def resnet50_v2(**kwargs):
    return get_resnet(2, 50, **kwargs)


def resnet101_v2(**kwargs):
    return get_resnet(2, 101, **kwargs)


def resnet152_v2(**kwargs):
    return get_resnet(2, 152, **kwargs)


def resnet18_v1b(**kwargs):
    return get_resnet(1, 18, v1b=True, **kwargs)


def resnet34_v1b(**kwargs):
    return get_resnet(1, 34, v1b=True, **kwargs)


def resnet50_v1b(**kwargs):
    return get_resnet(1, 50, v1b=True, **kwargs)


def resnet101_v1b(**kwargs):
    return get_resnet(1, 101, v1b=True, **kwargs)


def resnet152_v1b(**kwargs):
    return get_resnet(1, 152, v1b=True, **kwargs)
