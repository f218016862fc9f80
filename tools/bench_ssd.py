#!/usr/bin/env python
"""SSD-ResNet50 512x512 training throughput (BASELINE.json config 5).

ResNet-50 v1b backbone (NHWC, fused BN, fp16 compute, fp32 master weights via
multi-precision SGD), reference SSD head layout (example/ssd/symbol/symbol_factory.py
'resnet50'), 20 VOC classes, MultiBoxTarget with 3:1 hard-negative mining on the
GPU, softmax-CE + smooth-L1 loss.  Synthetic images and random ground-truth boxes
(random-init weights).  Launch like bench.py: N>1 through torch.distributed.run,
one process per GPU, RCCL all-reduce of the gradients (KVStore 'device').

Usage: python tools/bench_ssd.py [--batch 32] [--steps 20] [--warmup 5] [--size 512]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def synthetic_labels(B, max_obj, classes, gen):
    import torch
    lab = torch.full((B, max_obj, 5), -1.0)
    for b in range(B):
        n = int(torch.randint(1, max_obj + 1, (1,), generator=gen))
        xy = torch.rand(n, 2, generator=gen) * 0.7
        wh = 0.05 + torch.rand(n, 2, generator=gen) * 0.3
        lab[b, :n, 0] = torch.randint(0, classes, (n,), generator=gen).float()
        lab[b, :n, 1:3] = xy
        lab[b, :n, 3:5] = torch.clamp(xy + wh, max=1.0)
    return lab


def _load_launcher():
    """parallel/launch.py by path (no package import, so no GPU initialisation before the fork)."""
    import importlib.util
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        'mxnet_maintenance_amd', 'parallel', 'launch.py')
    spec = importlib.util.spec_from_file_location('_mxamd_launch', path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=32, help='per-GPU batch')
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--size', type=int, default=512)
    ap.add_argument('--classes', type=int, default=20)
    ap.add_argument('--dtype', default='float16', choices=['float16', 'bfloat16', 'float32'])
    ap.add_argument('--gpus', type=int, default=1, help='worker processes (one per GPU)')
    ap.add_argument('--deformable', type=int, default=1,
                    help='deformable 3x3 convs in the extra feature layers (the config\'s deformable/im2col conv)')
    ap.add_argument('--graph', type=int, default=1,
                    help='capture the whole step (forward, MultiBoxTarget, loss, backward, update) in one HIP graph '
                         '(gluon.GraphStep; eager fallback if capture fails)')
    args = ap.parse_args()
    launch = _load_launcher()
    if launch.needs_launch(args.gpus):
        sys.exit(launch.relaunch_self(args.gpus))

    import torch
    import mxnet_maintenance_amd as mx
    from mxnet_maintenance_amd import gluon, nd
    from mxnet_maintenance_amd.models import ssd
    from mxnet_maintenance_amd.parallel import dist

    if int(os.environ.get('WORLD_SIZE', '1')) > 1:
        dist.init()
    rank, n = dist.rank(), dist.world_size()
    gpu = torch.cuda.is_available()
    dev = dist.local_rank() % max(1, torch.cuda.device_count()) if gpu else 0
    if gpu:
        torch.cuda.set_device(dev)
    ctx = mx.gpu(dev) if gpu else mx.cpu()
    mx.random.seed(7 + rank)

    B, S = args.batch, args.size
    net = ssd.ssd_512_resnet50_v1(classes=args.classes, layout='NHWC', fuse=True, deformable=bool(args.deformable))
    net.initialize(mx.init.Xavier(magnitude=2), ctx=ctx)
    if args.dtype != 'float32':
        net.cast(args.dtype)
    net.hybridize(static_alloc=True, static_shape=True)
    trainer = gluon.Trainer(net.collect_params(), 'sgd', {'learning_rate': 1e-3, 'momentum': 0.9, 'wd': 5e-4,
                                                          'multi_precision': args.dtype != 'float32'},
                            kvstore='device')
    step = ssd.SSDTrainStep(net, trainer, (S, S))
    use_graph = bool(args.graph) and gpu
    if use_graph:
        step = gluon.GraphStep(step, trainer, warmup=max(1, args.warmup - 1), fallback=True)
    gen = torch.Generator().manual_seed(11 + rank)
    x = nd.random.uniform(-1, 1, shape=(B, S, S, 3), ctx=ctx).astype(args.dtype)
    labels = nd.array(synthetic_labels(B, 16, args.classes, gen).numpy(), ctx=ctx)

    def sync():
        if gpu:
            torch.cuda.synchronize()
        dist.barrier()

    for _ in range(args.warmup):
        L = step(x, labels, n)        # loss is already a per-rank mean; RCCL sums the ranks
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        L = step(x, labels, n)
    sync()
    dt = time.perf_counter() - t0
    if n > 1:
        t = torch.tensor([dt], dtype=torch.float64, device='cuda' if gpu else 'cpu')
        dist.all_reduce(t, op='max')
        dt = float(t.item())
    if rank == 0:
        print(json.dumps({
            'metric': 'images/sec (whole node) SSD-ResNet50 512x512 training', 'value': round(B * n * args.steps / dt, 2),
            'unit': 'images/sec', 'n_gpus': n, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': round(dt / args.steps * 1000, 3), 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': {'float16': 'fp16', 'bfloat16': 'bf16', 'float32': 'fp32'}[args.dtype],
            'data': 'synthetic (random-init weights, uniform images, random gt boxes)',
            'config': {'model': 'SSD-ResNet50 v1b', 'image_size': S, 'per_gpu_batch': B, 'global_batch': B * n,
                       'classes': args.classes, 'anchors': int(net.anchors((S, S), ctx).shape[1]),
                       'parallelism': 'dp%d' % n, 'final_loss': round(float(L.asscalar()), 4),
                       'deformable_extras': bool(args.deformable),
                       'hip_graph': bool(use_graph and getattr(step, 'captured', False))},
        }), flush=True)
    if os.environ.get('MXAMD_BENCH_VERBOSE', '0') == '1' and rank == 0:
        # per-shape autotune winners and candidate times (conv, GEMM, deformable GEMM keys)
        from mxnet_maintenance_amd.ops import kernel_fns
        times = kernel_fns.conv_algo_times()
        for k, v in sorted(kernel_fns.conv_algos().items(), key=str):
            t = ' '.join('%s=%.3f' % (nm, ms) for nm, ms in sorted(times.get(k, {}).items(), key=lambda z: z[1]))
            print('conv-algo', v, k, t, file=sys.stderr)
    if n > 1:
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
