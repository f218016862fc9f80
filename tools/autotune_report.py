"""Per-shape autotune report for the ResNet-50 training step: which candidate won each conv / GEMM
key and how far the best in-tree kernel is from a winning vendor kernel (MIOpen / hipBLASLt)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mxnet_maintenance_amd as mx  # noqa: E402
from mxnet_maintenance_amd import gluon, autograd, nd  # noqa: E402
from mxnet_maintenance_amd.ops import kernel_fns as KF  # noqa: E402


def main(batch=256):
    ctx = mx.gpu(0)
    net = gluon.model_zoo.vision.resnet50_v1b(layout='NHWC', fuse=True, classes=1000)
    net.initialize(mx.init.Xavier(), ctx=ctx)
    net.cast('float16')
    net.hybridize(static_alloc=True, static_shape=True)
    tr = gluon.Trainer(net.collect_params(), 'sgd', {'learning_rate': 0.01, 'momentum': 0.9,
                                                      'multi_precision': True})
    lf = gluon.loss.SoftmaxCrossEntropyLoss()
    x = nd.random.uniform(shape=(batch, 224, 224, 3), ctx=ctx).astype('float16')
    y = nd.array(torch.randint(0, 1000, (batch,)).numpy(), ctx=ctx)
    for _ in range(3):
        with autograd.record():
            loss = lf(net(x), y)
        loss.backward()
        tr.step(batch)
    torch.cuda.synchronize()
    vendor = ('mm', 'miopen')
    tot_gap = 0.0
    for key, times in sorted(KF._TIMES.items(), key=lambda kv: -min(kv[1].values())):
        win = KF._ALGO.get(key)
        ours = {k: v for k, v in times.items() if k not in vendor}
        best_ours = min(ours.items(), key=lambda kv: kv[1]) if ours else (None, float('nan'))
        gap = (best_ours[1] - times[win]) if win in vendor and ours else 0.0
        tot_gap += gap
        print('%-8s %-70s win=%-8s %.3f ms | best in-tree %s %.3f ms | gap %.3f' % (
            'VENDOR' if win in vendor else 'ours', str(key)[:70], win, times[win], best_ours[0], best_ours[1], gap),
            flush=True)
    print('rejected:', KF._REJECTED)
    print('total in-tree deficit on vendor-won keys: %.3f ms per call set' % tot_gap)


if __name__ == '__main__':
    main()
