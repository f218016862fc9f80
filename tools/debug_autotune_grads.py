"""Does the first (autotuning) backward of a hybridized NHWC fp16 ResNet give the same gradients as
later ones?  Prints per-parameter relative error of pass 1 and pass 2 against pass 3.

    python tools/debug_autotune_grads.py [resnet18_v1|resnet50_v1b] [--nofuse]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mxnet_maintenance_amd as mx  # noqa: E402
from mxnet_maintenance_amd import autograd, gluon, nd  # noqa: E402
from mxnet_maintenance_amd.ops import kernel_fns as KF  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith('--') else 'resnet18_v1'
    if '--nofuse' in sys.argv:
        KF._BN_BWD_FUSE[0] = False
    rs = np.random.RandomState(0)
    x = nd.array(rs.uniform(-1, 1, (16, 64, 64, 3)), ctx=mx.gpu(0), dtype='float16')
    y = nd.array(rs.randint(0, 10, (16,)), ctx=mx.gpu(0))
    loss_fn = gluon.loss.SoftmaxCrossEntropyLoss()
    grads = []
    names = None
    for p in range(3):
        mx.random.seed(5)
        net = gluon.model_zoo.vision.get_model(name, layout='NHWC', fuse=True, classes=10)
        net.initialize(mx.init.Xavier(rnd_type='gaussian', factor_type='in', magnitude=2), ctx=mx.gpu(0))
        net.cast('float16')
        net.hybridize(static_alloc=True, static_shape=True)
        with autograd.record():
            loss = loss_fn(net(x), y).mean() * 128
        loss.backward()
        ps = [(k, v) for k, v in net.collect_params().items() if v.grad_req != 'null']
        names = [k for k, _ in ps]
        grads.append([v.grad().asnumpy().astype(np.float32) for _, v in ps])
        print('pass', p, 'loss', float(loss.asscalar()), 'algos', len(KF._ALGO), flush=True)
    for i, n in enumerate(names):
        ref = grads[2][i]
        d = np.linalg.norm(ref) + 1e-6
        e1 = np.linalg.norm(grads[0][i] - ref) / d
        e2 = np.linalg.norm(grads[1][i] - ref) / d
        print('%-60s pass1 %.2e  pass2 %.2e  %s' % (n, e1, e2, '<<' if max(e1, e2) > 1e-2 else ''))
    for k, v in sorted(KF._ALGO.items(), key=lambda kv: str(kv[0])):
        print('ALGO', k, v)


if __name__ == '__main__':
    main()
