"""Where do the plain device copies / fills / adds of a training step come from?  Runs eager SSD-512
(`ssd`, default) or ResNet-50 (`resnet`) steps with torch's copy / contiguous / clone / zeros / add entry points wrapped, and
prints the framework call sites by count (tensor sizes summed).  Diagnostic only."""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
hits = collections.Counter()
bytes_ = collections.Counter()
active = [False]


def site():
    for fr in reversed(traceback.extract_stack()[:-2]):
        if fr.filename.startswith(REPO) and 'copy_sources_probe' not in fr.filename:
            return '%s:%d %s' % (os.path.relpath(fr.filename, REPO), fr.lineno, fr.name)
    return '?'


def wrap(owner, name):
    orig = getattr(owner, name)

    def f(*a, **k):
        r = orig(*a, **k)
        same = (name in ('contiguous', 'to', 'float') and a and isinstance(a[0], torch.Tensor)
                and isinstance(r, torch.Tensor) and r.data_ptr() == a[0].data_ptr())
        if active[0] and isinstance(r, torch.Tensor) and r.is_cuda and not same:
            key = '%-10s %s' % (name, site())
            hits[key] += 1
            bytes_[key] += r.numel() * r.element_size()
        return r
    setattr(owner, name, f)


for n in ('copy_', 'contiguous', 'clone', 'add', '__add__', 'add_', 'to', 'float', 'zero_'):
    wrap(torch.Tensor, n)
for n in ('zeros', 'zeros_like', 'cat', 'add'):
    wrap(torch, n)
torch.nn.functional.pad = (lambda orig: (lambda *a, **k: (hits.update(['pad        ' + site()]) if active[0] else None,
                                                          orig(*a, **k))[1]))(torch.nn.functional.pad)

import mxnet_maintenance_amd as mx  # noqa: E402
from mxnet_maintenance_amd import autograd, gluon, nd  # noqa: E402

ctx = mx.gpu(0)
MODEL = sys.argv[1] if len(sys.argv) > 1 else 'ssd'
if MODEL == 'ssd':
    from mxnet_maintenance_amd.models import ssd  # noqa: E402
    B, S = 32, 512
    net = ssd.ssd_512_resnet50_v1(classes=20, layout='NHWC', fuse=True, deformable=True)
    net.initialize(mx.init.Xavier(magnitude=2), ctx=ctx)
    net.cast('float16')
    net.hybridize(static_alloc=True, static_shape=True)
    trainer = gluon.Trainer(net.collect_params(), 'sgd', {'learning_rate': 1e-3, 'momentum': 0.9, 'wd': 5e-4,
                                                          'multi_precision': True}, kvstore='device')
    step_fn = ssd.SSDTrainStep(net, trainer, (S, S))
    x = nd.random.uniform(-1, 1, shape=(B, S, S, 3), ctx=ctx).astype('float16')
    sys.path.insert(0, os.path.join(REPO, 'tools'))
    from bench_ssd import synthetic_labels  # noqa: E402
    labels = nd.array(synthetic_labels(B, 16, 20, torch.Generator().manual_seed(11)).numpy(), ctx=ctx)

    def step():
        step_fn(x, labels, 1)
else:
    # the bench.py ResNet-50 v1b fp16 b256 NHWC step, eager
    B = 256
    net = gluon.model_zoo.vision.get_model('resnet50_v1b', layout='NHWC', fuse=True, classes=1000)
    net.initialize(mx.init.Xavier(rnd_type='gaussian', factor_type='in', magnitude=2), ctx=ctx)
    net.cast('float16')
    net.hybridize(static_alloc=True, static_shape=True)
    trainer = gluon.Trainer(net.collect_params(), 'sgd', {'learning_rate': 0.1, 'momentum': 0.9, 'wd': 1e-4,
                                                          'multi_precision': True, 'rescale_grad': 1 / 128.},
                            kvstore='device')
    loss_fn = gluon.loss.SoftmaxCrossEntropyLoss()
    x = nd.random.uniform(-1, 1, shape=(B, 224, 224, 3), ctx=ctx).astype('float16')
    y = nd.array(torch.randint(0, 1000, (B,)).numpy(), ctx=ctx)

    def step():
        with autograd.record():
            loss = loss_fn(net(x), y) * 128.0
        loss.backward()
        trainer.step(B)
for _ in range(3):
    step()
torch.cuda.synchronize()
active[0] = True
step()
torch.cuda.synchronize()
active[0] = False
for k, v in hits.most_common(45):
    print('%4d  %8.1f MB  %s' % (v, bytes_[k] / 1e6, k))
