"""Per-shape autotune report for the ResNet-50 training step: which candidate won each conv / GEMM
key and how far the best in-tree kernel is from a winning vendor kernel (MIOpen / hipBLASLt)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import mxnet_maintenance_amd as mx  # noqa: E402
from mxnet_maintenance_amd import gluon, autograd, nd  # noqa: E402
from mxnet_maintenance_amd.ops import kernel_fns as KF  # noqa: E402


PEAK_TF = 2300.0     # dense fp16 MFMA, sustained clock (TF/s)
PEAK_TB = 5.3        # achievable HBM stream bandwidth (TB/s)


def _cost(key):
    """(GFLOP, minimal HBM GB) of one conv pass: every operand read once, the output written once."""
    kind = key[0]
    x = key[1]
    w = key[2]
    N, H, W, C = x
    K, R, S = w[0], w[1], w[2]
    if kind == 'teedgrad':
        Ho, Wo, st = H, W, 1
    else:
        st = key[3][0]
        pad = key[4][0]
        Ho = (H + 2 * pad - R) // st + 1
        Wo = (W + 2 * pad - S) // st + 1
    M = N * Ho * Wo
    flop = 2.0 * M * K * R * S * C / 1e9
    act_in, act_out, wt = N * H * W * C * 2, M * K * 2, K * R * S * C * 2
    by = (act_in + act_out + wt) / 1e9
    if kind == 'teedgrad':
        by += act_in / 1e9      # the shortcut gradient read as the addend
    if kind == 'wgrad':
        by = (act_in + act_out + wt * 2) / 1e9
    return flop, by


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
    tot_t = tot_bound = 0.0
    for key, times in sorted(KF._TIMES.items(), key=lambda kv: -min(kv[1].values())):
        try:
            fl, by = _cost(key)
            t = times[KF._ALGO.get(key)]
            bound = max(fl / PEAK_TF, by / PEAK_TB)      # ms: GFLOP / (TF/s) = ms
            tot_t += t
            tot_bound += bound
            print('   roofline %-9s %7.1f GF %6.3f GB | %6.0f TF/s %5.2f TB/s | bound %.3f ms (%s) eff %3.0f%%' % (
                key[0], fl, by, fl / t, by / t, bound, 'mem' if by / PEAK_TB > fl / PEAK_TF else 'mfma',
                100 * bound / t))
        except Exception as e:  # noqa: BLE001
            print('   roofline n/a', e)
        win = KF._ALGO.get(key)
        ours = {k: v for k, v in times.items() if k not in vendor}
        best_ours = min(ours.items(), key=lambda kv: kv[1]) if ours else (None, float('nan'))
        gap = (best_ours[1] - times[win]) if win in vendor and ours else 0.0
        tot_gap += gap
        print('%-8s %-70s win=%-8s %.3f ms | best in-tree %s %.3f ms | gap %.3f' % (
            'VENDOR' if win in vendor else 'ours', str(key)[:70], win, times[win], best_ours[0], best_ours[1], gap),
            flush=True)
    print('rejected:', KF._REJECTED)
    print('sum of chosen per-key times %.3f ms, roofline bound %.3f ms (%.0f%%)' % (tot_t, tot_bound,
                                                                                  100 * tot_bound / max(tot_t, 1e-9)))
    print('total in-tree deficit on vendor-won keys: %.3f ms per call set' % tot_gap)


if __name__ == '__main__':
    main()
