"""SSD (Single Shot MultiBox Detector) on a ResNet-50 backbone, NHWC.

Parity: example/ssd/symbol/symbol_factory.py (``resnet50`` entry: features at
the end of stage 3 and stage 4, four extra 1x1->3x3/s2 feature layers with
512/256/256/128 filters, per-layer anchor sizes/ratios),
example/ssd/symbol/common.py (multi_layer_feature, multibox_layer) and
example/ssd/symbol/symbol_builder.py (MultiBoxTarget -> softmax CE with
ignore label + smooth-L1 location loss, MultiBoxDetection for inference).

MI355X design: the backbone is the fused-BN NHWC ResNet of the model zoo
(MFMA implicit-GEMM convs, NHWC BN kernels); the prediction heads emit NHWC
maps so flattening them already gives the reference's (location, anchor,
class) order with no transpose; anchors are a constant computed once per
input size; targets come from the gfx950 MultiBoxTarget kernel (one workgroup
per image, src/kernels/detection.hip) so the training step never leaves the
GPU.
"""
import torch

from ..gluon import nn
from ..gluon.block import HybridBlock
from .. import ndarray as nd
from .. import autograd

__all__ = ['SSD', 'ssd_512_resnet50_v1', 'ssd_300_resnet50_v1', 'SSDMultiBoxLoss', 'SSDTrainStep']

# example/ssd/symbol/symbol_factory.py, network == 'resnet50'
_RESNET50_SIZES = [[.1, .141], [.2, .272], [.37, .447], [.54, .619], [.71, .79], [.88, .961]]
_RESNET50_RATIOS = [[1, 2, .5], [1, 2, .5, 3, 1. / 3], [1, 2, .5, 3, 1. / 3], [1, 2, .5, 3, 1. / 3],
                    [1, 2, .5], [1, 2, .5]]


class _DeformBlock(HybridBlock):
    """ReLU(deformable 3x3 conv) on an NHWC or NCHW feature map (the deformable op itself is NCHW)."""

    def __init__(self, channels, stride, pad, layout, **kwargs):
        super().__init__(**kwargs)
        from ..gluon.contrib.cnn import DeformableConvolution
        self.layout = layout
        self._kwargs = {'kernel': (3, 3), 'stride': (stride, stride), 'pad': (pad, pad)}
        with self.name_scope():
            self.conv = DeformableConvolution(channels, kernel_size=(3, 3), strides=(stride, stride),
                                              padding=(pad, pad), activation='relu')

    def hybrid_forward(self, F, x):
        if self.layout == 'NHWC':
            return F.transpose(self.conv(F.transpose(x, axes=(0, 3, 1, 2))), axes=(0, 2, 3, 1))
        return self.conv(x)


class SSD(HybridBlock):
    """SSD detector.  ``forward(x)`` -> (cls_preds [B, A, C+1], loc_preds [B, A*4]).

    ``x`` is NHWC when ``layout='NHWC'`` (the MI355X default) or NCHW.
    """

    def __init__(self, base='resnet50_v1b', classes=20, sizes=None, ratios=None, num_filters=(512, 256, 256, 128),
                 strides=(2, 2, 2, 2), pads=(1, 1, 1, 1), min_filter=128, layout='NHWC', fuse=True,
                 deformable=False, **kwargs):
        super().__init__(**kwargs)
        from ..gluon.model_zoo import vision
        self.classes = classes
        self.layout = layout
        self.sizes = [list(s) for s in (sizes or _RESNET50_SIZES)]
        self.ratios = [list(r) for r in (ratios or _RESNET50_RATIOS)]
        nfeat = 2 + len(num_filters)
        assert len(self.sizes) == len(self.ratios) == nfeat, 'one size/ratio list per feature map'
        self.num_anchors = [len(s) + len(r) - 1 for s, r in zip(self.sizes, self.ratios)]
        self._anchor_cache = {}
        with self.name_scope():
            backbone = vision.get_model(base, layout=layout, fuse=fuse)
            # stage-3 output (stride 16) and stage-4 output (stride 32): the features end with
            # ... stage3, stage4, global pooling (the stem's layer count depends on ``fuse``)
            nf_ = len(backbone.features)
            self.stage3 = backbone.features[:nf_ - 2]
            self.stage4 = backbone.features[nf_ - 2]
            self.extras = nn.HybridSequential(prefix='extras_')
            with self.extras.name_scope():
                for k, (nf, s, p) in enumerate(zip(num_filters, strides, pads)):
                    blk = nn.HybridSequential(prefix='multi_feat_%d_' % (k + 2))
                    with blk.name_scope():
                        blk.add(nn.Conv2D(max(min_filter, nf // 2), 1, layout=layout, activation='relu'))
                        if deformable:
                            # the config's deformable / im2col conv: 3x3 taps displaced by learned offsets
                            # (contrib DeformableConvolution, in-tree HIP sampling kernels on the GPU)
                            blk.add(_DeformBlock(nf, s, p, layout))
                        else:
                            blk.add(nn.Conv2D(nf, 3, strides=s, padding=p, layout=layout, activation='relu'))
                    self.extras.add(blk)
            self.cls_preds = nn.HybridSequential(prefix='cls_')
            self.loc_preds = nn.HybridSequential(prefix='loc_')
            with self.cls_preds.name_scope():
                for na in self.num_anchors:
                    self.cls_preds.add(nn.Conv2D(na * (classes + 1), 3, padding=1, layout=layout))
            with self.loc_preds.name_scope():
                for na in self.num_anchors:
                    self.loc_preds.add(nn.Conv2D(na * 4, 3, padding=1, layout=layout))

    def _features(self, x):
        feats = []
        y = self.stage3(x)
        feats.append(y)
        y = self.stage4(y)
        feats.append(y)
        for blk in self.extras:
            y = blk(y)
            feats.append(y)
        return feats

    def hybrid_forward(self, F, x):
        feats = self._features(x)
        cls, loc = [], []
        for f, cp, lp in zip(feats, self.cls_preds, self.loc_preds):
            c = cp(f)
            l_ = lp(f)
            if self.layout == 'NCHW':
                c = F.transpose(c, axes=(0, 2, 3, 1))
                l_ = F.transpose(l_, axes=(0, 2, 3, 1))
            cls.append(F.flatten(c))
            loc.append(F.flatten(l_))
        cls = F.reshape(F.concat(*cls, dim=1), shape=(0, -1, self.classes + 1))
        loc = F.concat(*loc, dim=1)
        return cls, loc

    def feature_shapes(self, data_shape):
        """Spatial (H, W) of every prediction map for a square/rect input of ``data_shape`` (H, W)."""
        h, w = data_shape
        shapes = []
        h, w = -(-h // 16), -(-w // 16)       # stride 16 (stage 3)
        shapes.append((h, w))
        h, w = -(-h // 2), -(-w // 2)         # stride 32 (stage 4)
        shapes.append((h, w))
        for blk in self.extras:
            conv = blk[1]
            k, s, p = conv._kwargs['kernel'][0], conv._kwargs['stride'][0], conv._kwargs['pad'][0]
            h, w = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
            shapes.append((h, w))
        return shapes

    def anchors(self, data_shape, ctx=None):
        """[1, A, 4] corner anchors (normalised) — MultiBoxPrior per map, concatenated."""
        key = (tuple(data_shape), str(ctx))
        if key not in self._anchor_cache:
            parts = []
            for (h, w), s, r in zip(self.feature_shapes(data_shape), self.sizes, self.ratios):
                dummy = nd.zeros((1, 1, h, w), ctx=ctx)
                parts.append(nd.contrib.MultiBoxPrior(dummy, sizes=s, ratios=r).reshape((1, -1, 4)))
            self._anchor_cache[key] = nd.concat(*parts, dim=1)
        return self._anchor_cache[key]

    def detect(self, x, data_shape, nms_threshold=0.45, threshold=0.01, nms_topk=400):
        """Inference: MultiBoxDetection over softmax class probabilities -> [B, A, 6]."""
        cls, loc = self(x)
        prob = nd.softmax(cls.astype('float32'), axis=-1).transpose((0, 2, 1))
        return nd.contrib.MultiBoxDetection(prob, loc.astype('float32'), self.anchors(data_shape, x.context),
                                            nms_threshold=nms_threshold, threshold=threshold, nms_topk=nms_topk)


def ssd_512_resnet50_v1(classes=20, **kwargs):
    return SSD('resnet50_v1b', classes=classes, **kwargs)


def ssd_300_resnet50_v1(classes=20, **kwargs):
    return SSD('resnet50_v1b', classes=classes, **kwargs)


class SSDMultiBoxLoss:
    """symbol_builder.py training loss: softmax CE over anchors with ignore label (-1), normalised by
    the valid anchors, plus smooth-L1 on masked location offsets normalised by the positives."""

    def __init__(self, negative_mining_ratio=3.0, overlap_threshold=0.5, negative_mining_thresh=0.5,
                 variances=(0.1, 0.1, 0.2, 0.2), lambd=1.0):
        self.ratio = negative_mining_ratio
        self.thr = overlap_threshold
        self.neg_thresh = negative_mining_thresh
        self.variances = variances
        self.lambd = lambd

    def targets(self, anchors, labels, cls_preds):
        with autograd.pause():
            cp = cls_preds.detach().transpose((0, 2, 1))
            return nd.contrib.MultiBoxTarget(anchors, labels, cp, overlap_threshold=self.thr,
                                             negative_mining_ratio=self.ratio,
                                             negative_mining_thresh=self.neg_thresh, variances=self.variances)

    def __call__(self, cls_preds, loc_preds, anchors, labels):
        loc_t, loc_m, cls_t = self.targets(anchors, labels, cls_preds)
        if cls_preds.context.device_type == 'gpu':
            # one fused kernel pass for the loss and one for both gradients (detection.hip ssd_loss_*)
            return nd.contrib.ssd_multibox_loss(cls_preds, loc_preds, cls_t, loc_t, loc_m, lambd=self.lambd)
        logp = nd.log_softmax(cls_preds.astype('float32'), axis=-1)
        valid = cls_t >= 0
        ce = -nd.pick(logp, nd.maximum(cls_t, 0), axis=-1) * valid
        nvalid = nd.maximum(valid.sum(), 1)
        npos = nd.maximum((cls_t > 0).sum(), 1)
        diff = (loc_preds.astype('float32') - loc_t) * loc_m
        loc_l = nd.smooth_l1(diff, scalar=1.0)
        return ce.sum() / nvalid + self.lambd * loc_l.sum() / npos


class SSDTrainStep:
    """One SSD training step (forward, target assignment, loss, backward, optimizer update)."""

    def __init__(self, net, trainer, data_shape, loss=None):
        self.net = net
        self.trainer = trainer
        self.data_shape = data_shape
        self.loss = loss or SSDMultiBoxLoss()

    def __call__(self, x, labels, batch_size):
        anchors = self.net.anchors(self.data_shape, x.context)
        with autograd.record():
            cls, loc = self.net(x)
            L = self.loss(cls, loc, anchors, labels)
        L.backward()
        self.trainer.step(batch_size)
        return L
