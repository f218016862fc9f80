"""AlexNet, VGG, SqueezeNet, DenseNet, Inception V3, MobileNet V1/V2.

Parity: python/mxnet/gluon/model_zoo/vision/{alexnet,vgg,squeezenet,densenet,
inception,mobilenet}.py — same architectures, constructors and factory names.
"""
from ... import nn
from ...block import HybridBlock
from ....context import cpu

__all__ = ['AlexNet', 'alexnet', 'VGG', 'vgg11', 'vgg13', 'vgg16', 'vgg19', 'vgg11_bn', 'vgg13_bn', 'vgg16_bn',
           'vgg19_bn', 'get_vgg', 'SqueezeNet', 'squeezenet1_0', 'squeezenet1_1', 'get_squeezenet', 'DenseNet',
           'densenet121', 'densenet161', 'densenet169', 'densenet201', 'get_densenet', 'Inception3',
           'inception_v3', 'MobileNet', 'MobileNetV2', 'mobilenet1_0', 'mobilenet0_75', 'mobilenet0_5',
           'mobilenet0_25', 'mobilenet_v2_1_0', 'mobilenet_v2_0_75', 'mobilenet_v2_0_5', 'mobilenet_v2_0_25',
           'get_mobilenet', 'get_mobilenet_v2']


def _load_pretrained(net, name, pretrained, ctx, root):
    if pretrained:
        from ..model_store import get_model_file
        net.load_parameters(get_model_file(name, root=root), ctx=ctx)
    return net


# ------------------------------------------------------------------ AlexNet
class AlexNet(HybridBlock):
    def __init__(self, classes=1000, **kwargs):
        super().__init__(**kwargs)
        with self.name_scope():
            self.features = nn.HybridSequential(prefix='')
            with self.features.name_scope():
                for ch, k, s, p, pool in [(64, 11, 4, 2, True), (192, 5, 1, 2, True), (384, 3, 1, 1, False),
                                          (256, 3, 1, 1, False), (256, 3, 1, 1, True)]:
                    self.features.add(nn.Conv2D(ch, kernel_size=k, strides=s, padding=p, activation='relu'))
                    if pool:
                        self.features.add(nn.MaxPool2D(pool_size=3, strides=2))
                self.features.add(nn.Flatten())
                for _ in range(2):
                    self.features.add(nn.Dense(4096, activation='relu'))
                    self.features.add(nn.Dropout(0.5))
            self.output = nn.Dense(classes)

    def hybrid_forward(self, F, x):
        return self.output(self.features(x))


def alexnet(pretrained=False, ctx=cpu(), root='~/.mxnet/models', **kwargs):
    return _load_pretrained(AlexNet(**kwargs), 'alexnet', pretrained, ctx, root)


# ---------------------------------------------------------------------- VGG
vgg_spec = {11: ([1, 1, 2, 2, 2], [64, 128, 256, 512, 512]),
            13: ([2, 2, 2, 2, 2], [64, 128, 256, 512, 512]),
            16: ([2, 2, 3, 3, 3], [64, 128, 256, 512, 512]),
            19: ([2, 2, 4, 4, 4], [64, 128, 256, 512, 512])}


class VGG(HybridBlock):
    def __init__(self, layers, filters, classes=1000, batch_norm=False, **kwargs):
        super().__init__(**kwargs)
        assert len(layers) == len(filters)
        with self.name_scope():
            self.features = nn.HybridSequential(prefix='')
            for n, f in zip(layers, filters):
                for _ in range(n):
                    self.features.add(nn.Conv2D(f, kernel_size=3, padding=1, weight_initializer='xavier',
                                                bias_initializer='zeros'))
                    if batch_norm:
                        self.features.add(nn.BatchNorm())
                    self.features.add(nn.Activation('relu'))
                self.features.add(nn.MaxPool2D(strides=2))
            for _ in range(2):
                self.features.add(nn.Dense(4096, activation='relu', weight_initializer='normal',
                                           bias_initializer='zeros'))
                self.features.add(nn.Dropout(rate=0.5))
            self.output = nn.Dense(classes, weight_initializer='normal', bias_initializer='zeros')

    def hybrid_forward(self, F, x):
        return self.output(self.features(x))


def get_vgg(num_layers, pretrained=False, ctx=cpu(), root='~/.mxnet/models', **kwargs):
    layers, filters = vgg_spec[num_layers]
    net = VGG(layers, filters, **kwargs)
    bn = '_bn' if kwargs.get('batch_norm') else ''
    return _load_pretrained(net, 'vgg%d%s' % (num_layers, bn), pretrained, ctx, root)


def vgg11(**kw):
    return get_vgg(11, **kw)


def vgg13(**kw):
    return get_vgg(13, **kw)


def vgg16(**kw):
    return get_vgg(16, **kw)


def vgg19(**kw):
    return get_vgg(19, **kw)


def vgg11_bn(**kw):
    kw['batch_norm'] = True
    return get_vgg(11, **kw)


def vgg13_bn(**kw):
    kw['batch_norm'] = True
    return get_vgg(13, **kw)


def vgg16_bn(**kw):
    kw['batch_norm'] = True
    return get_vgg(16, **kw)


def vgg19_bn(**kw):
    kw['batch_norm'] = True
    return get_vgg(19, **kw)


# --------------------------------------------------------------- SqueezeNet
def _fire(squeeze, e1, e3):
    out = nn.HybridSequential(prefix='')
    out.add(nn.Conv2D(squeeze, kernel_size=1), nn.Activation('relu'))
    paths = _HybridConcat()
    left = nn.HybridSequential(prefix='')
    left.add(nn.Conv2D(e1, kernel_size=1), nn.Activation('relu'))
    right = nn.HybridSequential(prefix='')
    right.add(nn.Conv2D(e3, kernel_size=3, padding=1), nn.Activation('relu'))
    paths.add(left, right)
    out.add(paths)
    return out


class _HybridConcat(nn.HybridSequential):
    """Run children on the same input and concatenate along channels."""

    def __init__(self, axis=1, **kwargs):
        super().__init__(prefix='', **kwargs)
        self._axis = axis

    def hybrid_forward(self, F, x):
        return F.Concat(*[b(x) for b in self._children.values()], dim=self._axis)


class SqueezeNet(HybridBlock):
    def __init__(self, version, classes=1000, **kwargs):
        super().__init__(**kwargs)
        assert version in ['1.0', '1.1']
        with self.name_scope():
            self.features = nn.HybridSequential(prefix='')
            if version == '1.0':
                self.features.add(nn.Conv2D(96, kernel_size=7, strides=2), nn.Activation('relu'),
                                  nn.MaxPool2D(pool_size=3, strides=2, ceil_mode=True))
                spec = [(16, 64, 64), (16, 64, 64), (32, 128, 128), 'pool', (32, 128, 128), (48, 192, 192),
                        (48, 192, 192), (64, 256, 256), 'pool', (64, 256, 256)]
            else:
                self.features.add(nn.Conv2D(64, kernel_size=3, strides=2), nn.Activation('relu'),
                                  nn.MaxPool2D(pool_size=3, strides=2, ceil_mode=True))
                spec = [(16, 64, 64), (16, 64, 64), 'pool', (32, 128, 128), (32, 128, 128), 'pool',
                        (48, 192, 192), (48, 192, 192), (64, 256, 256), (64, 256, 256)]
            for s in spec:
                if s == 'pool':
                    self.features.add(nn.MaxPool2D(pool_size=3, strides=2, ceil_mode=True))
                else:
                    self.features.add(_fire(*s))
            self.features.add(nn.Dropout(0.5))
            self.output = nn.HybridSequential(prefix='')
            self.output.add(nn.Conv2D(classes, kernel_size=1), nn.Activation('relu'),
                            nn.AvgPool2D(13), nn.Flatten())

    def hybrid_forward(self, F, x):
        return self.output(self.features(x))


def get_squeezenet(version, pretrained=False, ctx=cpu(), root='~/.mxnet/models', **kwargs):
    return _load_pretrained(SqueezeNet(version, **kwargs), 'squeezenet%s' % version, pretrained, ctx, root)


def squeezenet1_0(**kw):
    return get_squeezenet('1.0', **kw)


def squeezenet1_1(**kw):
    return get_squeezenet('1.1', **kw)


# ----------------------------------------------------------------- DenseNet
class _DenseLayer(HybridBlock):
    def __init__(self, growth_rate, bn_size, dropout, **kwargs):
        super().__init__(**kwargs)
        self.body = nn.HybridSequential(prefix='')
        self.body.add(nn.BatchNorm(), nn.Activation('relu'),
                      nn.Conv2D(bn_size * growth_rate, kernel_size=1, use_bias=False),
                      nn.BatchNorm(), nn.Activation('relu'),
                      nn.Conv2D(growth_rate, kernel_size=3, padding=1, use_bias=False))
        if dropout:
            self.body.add(nn.Dropout(dropout))

    def hybrid_forward(self, F, x):
        return F.Concat(x, self.body(x), dim=1)


def _dense_block(num_layers, bn_size, growth_rate, dropout, stage_index):
    out = nn.HybridSequential(prefix='stage%d_' % stage_index)
    with out.name_scope():
        for _ in range(num_layers):
            out.add(_DenseLayer(growth_rate, bn_size, dropout, prefix=''))
    return out


def _transition(num_output_features):
    out = nn.HybridSequential(prefix='')
    out.add(nn.BatchNorm(), nn.Activation('relu'), nn.Conv2D(num_output_features, kernel_size=1, use_bias=False),
            nn.AvgPool2D(pool_size=2, strides=2))
    return out


class DenseNet(HybridBlock):
    def __init__(self, num_init_features, growth_rate, block_config, bn_size=4, dropout=0, classes=1000,
                 **kwargs):
        super().__init__(**kwargs)
        with self.name_scope():
            self.features = nn.HybridSequential(prefix='')
            self.features.add(nn.Conv2D(num_init_features, kernel_size=7, strides=2, padding=3, use_bias=False),
                              nn.BatchNorm(), nn.Activation('relu'), nn.MaxPool2D(pool_size=3, strides=2, padding=1))
            num_features = num_init_features
            for i, num_layers in enumerate(block_config):
                self.features.add(_dense_block(num_layers, bn_size, growth_rate, dropout, i + 1))
                num_features = num_features + num_layers * growth_rate
                if i != len(block_config) - 1:
                    self.features.add(_transition(num_features // 2))
                    num_features = num_features // 2
            self.features.add(nn.BatchNorm(), nn.Activation('relu'), nn.AvgPool2D(pool_size=7), nn.Flatten())
            self.output = nn.Dense(classes)

    def hybrid_forward(self, F, x):
        return self.output(self.features(x))


densenet_spec = {121: (64, 32, [6, 12, 24, 16]), 161: (96, 48, [6, 12, 36, 24]),
                 169: (64, 32, [6, 12, 32, 32]), 201: (64, 32, [6, 12, 48, 32])}


def get_densenet(num_layers, pretrained=False, ctx=cpu(), root='~/.mxnet/models', **kwargs):
    init, growth, cfg = densenet_spec[num_layers]
    return _load_pretrained(DenseNet(init, growth, cfg, **kwargs), 'densenet%d' % num_layers, pretrained, ctx, root)


def densenet121(**kw):
    return get_densenet(121, **kw)


def densenet161(**kw):
    return get_densenet(161, **kw)


def densenet169(**kw):
    return get_densenet(169, **kw)


def densenet201(**kw):
    return get_densenet(201, **kw)


# -------------------------------------------------------------- Inception V3
def _bconv(channels, kernel_size, strides=1, padding=0):
    out = nn.HybridSequential(prefix='')
    out.add(nn.Conv2D(channels, kernel_size=kernel_size, strides=strides, padding=padding, use_bias=False),
            nn.BatchNorm(epsilon=0.001), nn.Activation('relu'))
    return out


def _branch(pool, *convs):
    out = nn.HybridSequential(prefix='')
    if pool == 'avg':
        out.add(nn.AvgPool2D(pool_size=3, strides=1, padding=1))
    elif pool == 'max':
        out.add(nn.MaxPool2D(pool_size=3, strides=2))
    for c in convs:
        out.add(_bconv(*c))
    return out


class _Concat(HybridBlock):
    def __init__(self, branches, **kwargs):
        super().__init__(**kwargs)
        for i, b in enumerate(branches):
            self.register_child(b, str(i))

    def hybrid_forward(self, F, x):
        return F.Concat(*[b(x) for b in self._children.values()], dim=1)


class _SplitConcat(HybridBlock):
    """stem -> two parallel convs, concatenated (Inception E-block branch)."""

    def __init__(self, stem, a, b, **kwargs):
        super().__init__(**kwargs)
        self.stem, self.a, self.b = stem, a, b

    def hybrid_forward(self, F, x):
        x = self.stem(x) if self.stem is not None else x
        return F.Concat(self.a(x), self.b(x), dim=1)


def _make_A(pool_features, prefix):
    return _Concat([_branch(None, (64, 1)), _branch(None, (48, 1), (64, 5, 1, 2)),
                    _branch(None, (64, 1), (96, 3, 1, 1), (96, 3, 1, 1)), _branch('avg', (pool_features, 1))],
                   prefix=prefix)


def _make_B(prefix):
    return _Concat([_branch(None, (384, 3, 2)), _branch(None, (64, 1), (96, 3, 1, 1), (96, 3, 2)),
                    _branch('max')], prefix=prefix)


def _make_C(c7, prefix):
    return _Concat([_branch(None, (192, 1)), _branch(None, (c7, 1), (c7, (1, 7), 1, (0, 3)), (192, (7, 1), 1, (3, 0))),
                    _branch(None, (c7, 1), (c7, (7, 1), 1, (3, 0)), (c7, (1, 7), 1, (0, 3)), (c7, (7, 1), 1, (3, 0)),
                            (192, (1, 7), 1, (0, 3))), _branch('avg', (192, 1))], prefix=prefix)


def _make_D(prefix):
    return _Concat([_branch(None, (192, 1), (320, 3, 2)),
                    _branch(None, (192, 1), (192, (1, 7), 1, (0, 3)), (192, (7, 1), 1, (3, 0)), (192, 3, 2)),
                    _branch('max')], prefix=prefix)


def _make_E(prefix):
    b1 = _branch(None, (320, 1))
    b2 = _SplitConcat(_branch(None, (384, 1)), _branch(None, (384, (1, 3), 1, (0, 1))),
                      _branch(None, (384, (3, 1), 1, (1, 0))))
    b3 = _SplitConcat(_branch(None, (448, 1), (384, 3, 1, 1)), _branch(None, (384, (1, 3), 1, (0, 1))),
                      _branch(None, (384, (3, 1), 1, (1, 0))))
    b4 = _branch('avg', (192, 1))
    return _Concat([b1, b2, b3, b4], prefix=prefix)


class Inception3(HybridBlock):
    def __init__(self, classes=1000, **kwargs):
        super().__init__(**kwargs)
        with self.name_scope():
            self.features = nn.HybridSequential(prefix='')
            self.features.add(_bconv(32, 3, 2), _bconv(32, 3), _bconv(64, 3, 1, 1),
                              nn.MaxPool2D(pool_size=3, strides=2), _bconv(80, 1), _bconv(192, 3),
                              nn.MaxPool2D(pool_size=3, strides=2),
                              _make_A(32, 'A1_'), _make_A(64, 'A2_'), _make_A(64, 'A3_'), _make_B('B_'),
                              _make_C(128, 'C1_'), _make_C(160, 'C2_'), _make_C(160, 'C3_'), _make_C(192, 'C4_'),
                              _make_D('D_'), _make_E('E1_'), _make_E('E2_'), nn.AvgPool2D(pool_size=8),
                              nn.Dropout(0.5))
            self.output = nn.Dense(classes)

    def hybrid_forward(self, F, x):
        return self.output(self.features(x))


def inception_v3(pretrained=False, ctx=cpu(), root='~/.mxnet/models', **kwargs):
    return _load_pretrained(Inception3(**kwargs), 'inceptionv3', pretrained, ctx, root)


# ---------------------------------------------------------------- MobileNet
class _ReLU6(HybridBlock):
    def hybrid_forward(self, F, x):
        return F.clip(x, 0, 6, name='relu6')


def _add_conv(out, channels=1, kernel=1, stride=1, pad=0, num_group=1, active=True, relu6=False):
    out.add(nn.Conv2D(channels, kernel, stride, pad, groups=num_group, use_bias=False))
    out.add(nn.BatchNorm(scale=True))
    if active:
        out.add(_ReLU6() if relu6 else nn.Activation('relu'))


def _add_conv_dw(out, dw_channels, channels, stride, relu6=False):
    _add_conv(out, channels=dw_channels, kernel=3, stride=stride, pad=1, num_group=dw_channels, relu6=relu6)
    _add_conv(out, channels=channels, relu6=relu6)


class _LinearBottleneck(HybridBlock):
    def __init__(self, in_channels, channels, t, stride, **kwargs):
        super().__init__(**kwargs)
        self.use_shortcut = stride == 1 and in_channels == channels
        with self.name_scope():
            self.out = nn.HybridSequential()
            _add_conv(self.out, in_channels * t, relu6=True)
            _add_conv(self.out, in_channels * t, kernel=3, stride=stride, pad=1, num_group=in_channels * t,
                      relu6=True)
            _add_conv(self.out, channels, active=False, relu6=True)

    def hybrid_forward(self, F, x):
        out = self.out(x)
        if self.use_shortcut:
            out = F.elemwise_add(out, x)
        return out


class MobileNet(HybridBlock):
    def __init__(self, multiplier=1.0, classes=1000, **kwargs):
        super().__init__(**kwargs)
        with self.name_scope():
            self.features = nn.HybridSequential(prefix='')
            with self.features.name_scope():
                _add_conv(self.features, channels=int(32 * multiplier), kernel=3, pad=1, stride=2)
                dw_channels = [int(x * multiplier) for x in [32, 64] + [128] * 2 + [256] * 2 + [512] * 6 + [1024]]
                channels = [int(x * multiplier) for x in [64] + [128] * 2 + [256] * 2 + [512] * 6 + [1024] * 2]
                strides = [1, 2] * 3 + [1] * 5 + [2, 1]
                for dwc, c, s in zip(dw_channels, channels, strides):
                    _add_conv_dw(self.features, dw_channels=dwc, channels=c, stride=s)
                self.features.add(nn.GlobalAvgPool2D())
                self.features.add(nn.Flatten())
            self.output = nn.Dense(classes)

    def hybrid_forward(self, F, x):
        return self.output(self.features(x))


class MobileNetV2(HybridBlock):
    def __init__(self, multiplier=1.0, classes=1000, **kwargs):
        super().__init__(**kwargs)
        with self.name_scope():
            self.features = nn.HybridSequential(prefix='features_')
            with self.features.name_scope():
                _add_conv(self.features, int(32 * multiplier), kernel=3, stride=2, pad=1, relu6=True)
                in_channels_group = [int(x * multiplier) for x in [32] + [16] + [24] * 2 + [32] * 3 + [64] * 4 +
                                     [96] * 3 + [160] * 3]
                channels_group = [int(x * multiplier) for x in [16] + [24] * 2 + [32] * 3 + [64] * 4 + [96] * 3 +
                                  [160] * 3 + [320]]
                ts = [1] + [6] * 16
                strides = [1, 2] * 2 + [1, 1, 2] + [1] * 6 + [2] + [1] * 3
                for in_c, c, t, s in zip(in_channels_group, channels_group, ts, strides):
                    self.features.add(_LinearBottleneck(in_channels=in_c, channels=c, t=t, stride=s))
                last_channels = int(1280 * multiplier) if multiplier > 1.0 else 1280
                _add_conv(self.features, last_channels, relu6=True)
                self.features.add(nn.GlobalAvgPool2D())
            self.output = nn.HybridSequential(prefix='output_')
            with self.output.name_scope():
                self.output.add(nn.Conv2D(classes, 1, use_bias=False, prefix='pred_'), nn.Flatten())

    def hybrid_forward(self, F, x):
        return self.output(self.features(x))


def get_mobilenet(multiplier, pretrained=False, ctx=cpu(), root='~/.mxnet/models', **kwargs):
    ver = '%.2f' % multiplier
    ver = {'1.00': '1.0', '0.50': '0.5'}.get(ver, ver)
    return _load_pretrained(MobileNet(multiplier, **kwargs), 'mobilenet%s' % ver, pretrained, ctx, root)


def get_mobilenet_v2(multiplier, pretrained=False, ctx=cpu(), root='~/.mxnet/models', **kwargs):
    ver = '%.2f' % multiplier
    ver = {'1.00': '1.0', '0.50': '0.5'}.get(ver, ver)
    return _load_pretrained(MobileNetV2(multiplier, **kwargs), 'mobilenetv2_%s' % ver, pretrained, ctx, root)


def mobilenet1_0(**kw):
    return get_mobilenet(1.0, **kw)


def mobilenet0_75(**kw):
    return get_mobilenet(0.75, **kw)


def mobilenet0_5(**kw):
    return get_mobilenet(0.5, **kw)


def mobilenet0_25(**kw):
    return get_mobilenet(0.25, **kw)


def mobilenet_v2_1_0(**kw):
    return get_mobilenet_v2(1.0, **kw)


def mobilenet_v2_0_75(**kw):
    return get_mobilenet_v2(0.75, **kw)


def mobilenet_v2_0_5(**kw):
    return get_mobilenet_v2(0.5, **kw)


def mobilenet_v2_0_25(**kw):
    return get_mobilenet_v2(0.25, **kw)
