"""Training-correctness diagnostic on the headline bench config.

ResNet-50 v1b, NHWC, fp16 + fp32 master weights, mp-SGD lr 0.1 momentum 0.9
wd 1e-4, static loss scale 128, one fixed synthetic batch.  Runs the step
eagerly twice and through gluon.GraphStep once (same process, so the autotuned
kernel choices are shared) and prints the per-step loss of each run plus the
relative weight distance at the end.

    python tools/diag_train_bench.py [--batch 64] [--steps 30] [--modes eager,eager,graph]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(mode, args):
    import torch
    import mxnet_maintenance_amd as mx
    from mxnet_maintenance_amd import gluon, autograd, nd
    mx.random.seed(7)
    torch.manual_seed(7)
    ctx = mx.gpu(0)
    net = gluon.model_zoo.vision.get_model(args.model, layout='NHWC', fuse=True, classes=1000)
    net.initialize(mx.init.Xavier(rnd_type='gaussian', factor_type='in', magnitude=2), ctx=ctx)
    net.cast('float16')
    net.hybridize(static_alloc=True, static_shape=True)
    tr = gluon.Trainer(net.collect_params(), 'sgd', {'learning_rate': args.lr, 'momentum': 0.9, 'wd': 1e-4,
                                                      'multi_precision': True, 'rescale_grad': 1.0 / 128})
    lf = gluon.loss.SoftmaxCrossEntropyLoss()
    g = torch.Generator().manual_seed(0)
    B, S = args.batch, args.size
    x = nd.array((torch.rand((B, S, S, 3), generator=g) * 2 - 1).numpy(), ctx=ctx).astype('float16')
    y = nd.array(torch.randint(0, 1000, (B,), generator=g).numpy(), ctx=ctx)

    def step():
        with autograd.record():
            loss = lf(net(x), y) * 128.0
        loss.backward()
        tr.step(B)
        return loss

    f = gluon.GraphStep(step, tr, warmup=args.graph_warmup) if mode == 'graph' else step
    losses = []
    t0 = time.time()
    for _ in range(args.steps):
        losses.append(float(f().mean().asscalar()) / 128)
    dt = time.time() - t0
    ws = [p.data().asnumpy().astype(np.float32).ravel() for p in net.collect_params().values()]
    return np.asarray(losses), np.concatenate(ws), dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--model', default='resnet50_v1b')
    ap.add_argument('--batch', type=int, default=64)
    ap.add_argument('--size', type=int, default=224)
    ap.add_argument('--steps', type=int, default=30)
    ap.add_argument('--lr', type=float, default=0.1)
    ap.add_argument('--graph-warmup', type=int, default=4)
    ap.add_argument('--modes', default='eager,eager,graph')
    args = ap.parse_args()
    res = []
    for m in args.modes.split(','):
        l, w, dt = run(m, args)
        res.append((m, l, w))
        print('%-6s %5.1fs losses %s' % (m, dt, np.array2string(l, precision=4, max_line_width=400)), flush=True)
    m0, l0, w0 = res[0]
    for m, l, w in res[1:]:
        print('%s vs %s: max |dloss| %.3g (first step differing: %s), weight rel dist %.3g' % (
            m, m0, float(np.abs(l - l0).max()),
            int(np.argmax(np.abs(l - l0) > 0)) if np.any(l != l0) else None,
            float(np.linalg.norm(w - w0) / np.linalg.norm(w0))), flush=True)


if __name__ == '__main__':
    main()
