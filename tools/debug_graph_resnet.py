"""Eager vs GraphStep on ResNet (NHWC fp16, mp-SGD): per-step loss and parameter drift (debug aid)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import mxnet_maintenance_amd as mx
from mxnet_maintenance_amd import gluon, autograd, nd


def run(graph, model='resnet50_v1b', B=32, S=112, steps=6, lr=0.001):
    mx.random.seed(3)
    torch.manual_seed(3)
    ctx = mx.gpu(0)
    net = gluon.model_zoo.vision.get_model(model, layout='NHWC', fuse=True, classes=1000)
    net.initialize(mx.init.Xavier(rnd_type='gaussian', factor_type='in', magnitude=2), ctx=ctx)
    net.cast('float16')
    net.hybridize(static_alloc=True, static_shape=True)
    tr = gluon.Trainer(net.collect_params(), 'sgd', {'learning_rate': lr, 'momentum': 0.9, 'wd': 1e-4,
                                                      'multi_precision': True, 'rescale_grad': 1.0 / 128})
    lf = gluon.loss.SoftmaxCrossEntropyLoss()
    g = torch.Generator().manual_seed(0)
    x = nd.array((torch.rand((B, S, S, 3), generator=g) * 2 - 1).numpy(), ctx=ctx).astype('float16')
    y = nd.array(torch.randint(0, 1000, (B,), generator=g).numpy(), ctx=ctx)

    def step():
        with autograd.record():
            loss = lf(net(x), y) * 128.0
        loss.backward()
        tr.step(B)
        return loss

    f = gluon.GraphStep(step, tr, warmup=2) if graph else step
    out = []
    for _ in range(steps):
        l = f()
        ps = [p.data().asnumpy().astype(np.float32) for p in net.collect_params().values()]
        out.append((float(l.mean().asscalar()) / 128, ps))
    return out


if __name__ == '__main__':
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument('--lr', type=float, default=0.001)
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--size', type=int, default=112)
    ap.add_argument('--steps', type=int, default=6)
    a = ap.parse_args()
    kw = dict(B=a.batch, S=a.size, steps=a.steps, lr=a.lr)
    e0 = run(False, **kw)      # autotunes
    e = run(False, **kw)       # same kernels as the graph run
    g = run(True, **kw)
    for i, ((le0, pe0), (le, pe), (lg, pg)) in enumerate(zip(e0, e, g)):
        d_ee = max(float(np.abs(a - b).max()) for a, b in zip(pe0, pe))
        d = max(float(np.abs(a - b).max()) for a, b in zip(pe, pg))
        print('step %d eager %.5f eager2 %.5f graph %.5f  eager-vs-eager %.3g  eager-vs-graph %.3g'
              % (i, le0, le, lg, d_ee, d), flush=True)
