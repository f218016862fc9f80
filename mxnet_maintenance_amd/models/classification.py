"""Image-classification training harness (the flagship workload).

Parity: example/image-classification/train_imagenet.py + common/fit.py in the
reference (model from the zoo, multi-precision SGD with momentum, kvstore
gradient reduction, fixed loss scaling for fp16).  MI355X design: NHWC
activations end-to-end, fp16/bf16 compute with fp32 master weights held by the
fused multi-tensor optimizer, the hybridized graph running our HIP
conv/BN/pool kernels, and gradient buckets all-reduced over RCCL while the
backward pass is still running.
"""
import torch

from .. import autograd, gluon, nd
from .. import initializer as init

__all__ = ['ClassificationTrainer']


class ClassificationTrainer:
    """Owns net + Trainer + loss; ``step(x, y)`` is one full training step."""

    def __init__(self, model='resnet50_v1b', ctx=None, dtype='float16', classes=1000, layout='NHWC', fuse=True,
                 lr=0.1, momentum=0.9, wd=1e-4, loss_scale=None, kvstore='device', hybridize=True):
        from .. import context
        self.ctx = ctx or context.current_context()
        self.dtype = dtype
        self.net = gluon.model_zoo.vision.get_model(model, layout=layout, fuse=fuse, classes=classes)
        self.net.initialize(init.Xavier(rnd_type='gaussian', factor_type='in', magnitude=2), ctx=self.ctx)
        if dtype != 'float32':
            self.net.cast(dtype)
        if hybridize:
            self.net.hybridize(static_alloc=True, static_shape=True)
        self.loss_scale = loss_scale if loss_scale is not None else (128.0 if dtype == 'float16' else 1.0)
        self.trainer = gluon.Trainer(self.net.collect_params(), 'sgd',
                                     {'learning_rate': lr, 'momentum': momentum, 'wd': wd,
                                      'multi_precision': dtype != 'float32', 'rescale_grad': 1.0 / self.loss_scale},
                                     kvstore=kvstore)
        self.loss_fn = gluon.loss.SoftmaxCrossEntropyLoss()

    def synthetic_batch(self, batch, image_size=224, layout='NHWC'):
        shape = (batch, image_size, image_size, 3) if layout == 'NHWC' else (batch, 3, image_size, image_size)
        x = nd.random.uniform(-1, 1, shape=shape, ctx=self.ctx).astype(self.dtype)
        y = nd.array(torch.randint(0, 1000, (batch,)).numpy(), ctx=self.ctx)
        return x, y

    def step(self, x, y):
        with autograd.record():
            loss = self.loss_fn(self.net(x), y)
            if self.loss_scale != 1.0:
                loss = loss * self.loss_scale
        loss.backward()
        self.trainer.step(x.shape[0])
        return loss

    def loss_value(self, loss):
        return float(loss.mean().asscalar()) / self.loss_scale
