#!/usr/bin/env python
"""Headline benchmark: ResNet-50 v1b training throughput (images/sec, whole node).

Config (BASELINE.json): ResNet-50 v1b, fp16 compute with fp32 master weights
(multi-precision SGD, momentum 0.9), batch 256 per GPU, 224x224, synthetic
data / random-init weights, hybridized Gluon model, KVStore('device') RCCL
all-reduce for N > 1 (one process per GPU, launched by torch.distributed.run).

Timing: W untimed warm-up steps, then exactly K steps bracketed by a barrier +
device synchronisation on both sides; the max over ranks is reported.  Each
step = forward + loss + backward + gradient all-reduce + optimizer update.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
"""
import argparse
import json
import os
import sys
import time

BASELINE_IMG_S = 363.69   # reference's published ResNet-50 training number (V100, perf.md)
# Fixed lr warm-up (steps), deliberately NOT tied to --warmup: the driver's short runs
# (--warmup 5 --steps 20) must follow the same optimisation trajectory as long ones.
LR_WARMUP_STEPS = 40


def _load_launcher():
    """parallel/launch.py loaded by path: importing the package would import torch + HIP extensions."""
    import importlib.util
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'mxnet_maintenance_amd', 'parallel', 'launch.py')
    spec = importlib.util.spec_from_file_location('_mxamd_launch', path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=None,
                    help='GPUs (ranks) of this node; default: WORLD_SIZE under a launcher, else 1')
    ap.add_argument('--steps', type=int, default=30)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--batch', type=int, default=256, help='per-GPU batch size')
    ap.add_argument('--dtype', default='float16', choices=['float16', 'bfloat16', 'float32'])
    ap.add_argument('--model', default='resnet50_v1b')
    ap.add_argument('--no-fuse', action='store_true')
    ap.add_argument('--image-size', type=int, default=224)
    ap.add_argument('--layout', default='NHWC', choices=['NHWC', 'NCHW'],
                    help='model layout (NCHW = default Gluon layout, executed channels-last on the HIP kernels)')
    ap.add_argument('--lr-warmup', type=int, default=LR_WARMUP_STEPS,
                    help='linear learning-rate warm-up steps from 0 to 0.1, independent of --warmup (lr 0.1 '
                         'from random init on one fixed batch overshoots before it fits it)')
    ap.add_argument('--graph', default='auto', choices=['auto', 'on', 'off'],
                    help='capture the whole training step in one HIP graph (gluon.GraphStep); with N>1 the bucketed '
                         'RCCL all-reduces are captured too; auto = on for 1 GPU, eager for N>1 until measured')
    args = ap.parse_args()
    gpus_given = args.gpus is not None
    if args.gpus is None:
        args.gpus = int(os.environ.get('WORLD_SIZE', '1'))

    # `bench.py --gpus N` without a launcher: start N fresh worker processes (one per GPU) and exit
    # with their status.  This happens before anything in this process touches the GPU.
    launch = _load_launcher()
    if launch.needs_launch(args.gpus):
        sys.exit(launch.relaunch_self(args.gpus))

    import torch
    import mxnet_maintenance_amd as mx
    from mxnet_maintenance_amd import gluon, autograd, nd
    from mxnet_maintenance_amd.parallel import dist

    world = int(os.environ.get('WORLD_SIZE', '1'))
    if world > 1:
        dist.init()
    if gpus_given and dist.world_size() != args.gpus:
        raise SystemExit('bench.py: --gpus %d but the process group has %d ranks' % (args.gpus, dist.world_size()))
    rank = dist.rank()
    local_rank = dist.local_rank()
    # one process per GPU; ranks beyond the visible devices share them (single-GPU rehearsals)
    dev = local_rank % max(1, torch.cuda.device_count()) if torch.cuda.is_available() else 0
    ctx = mx.gpu(dev) if torch.cuda.is_available() else mx.cpu()
    if torch.cuda.is_available():
        torch.cuda.set_device(dev)
    mx.random.seed(1234 + rank)

    B = args.batch
    S = args.image_size
    net = gluon.model_zoo.vision.get_model(args.model, layout=args.layout, fuse=not args.no_fuse, classes=1000)
    net.initialize(mx.init.Xavier(rnd_type='gaussian', factor_type='in', magnitude=2), ctx=ctx)
    if args.dtype != 'float32':
        net.cast(args.dtype)
    net.hybridize(static_alloc=True, static_shape=True)

    loss_scale = 128.0 if args.dtype == 'float16' else 1.0
    warm = args.lr_warmup
    # constant 0.1 after a linear ramp; the schedule is device-staged per HIP-graph replay
    sched = mx.lr_scheduler.FactorScheduler(step=1 << 30, factor=1.0, base_lr=0.1, warmup_steps=warm,
                                            warmup_begin_lr=0.0) if warm > 0 else None
    trainer = gluon.Trainer(net.collect_params(), 'sgd',
                            {'learning_rate': 0.1, 'momentum': 0.9, 'wd': 1e-4, 'lr_scheduler': sched,
                             'multi_precision': args.dtype != 'float32',
                             'rescale_grad': 1.0 / loss_scale},
                            kvstore='device')
    loss_fn = gluon.loss.SoftmaxCrossEntropyLoss()

    shape = (B, S, S, 3) if args.layout == 'NHWC' else (B, 3, S, S)
    x = nd.random.uniform(-1, 1, shape=shape, ctx=ctx).astype(args.dtype)
    y = nd.array(torch.randint(0, 1000, (B,)).numpy(), ctx=ctx)

    n_ranks = dist.world_size()

    def step():
        with autograd.record():
            out = net(x)
            loss = loss_fn(out, y)
            if loss_scale != 1.0:
                loss = loss * loss_scale
        loss.backward()
        # gradients are summed over ranks by the RCCL all-reduce: normalise by the GLOBAL batch so
        # N-GPU data parallelism is the same optimisation as one GPU at batch B*N
        trainer.step(B * n_ranks)
        return loss

    def sync():
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        dist.barrier()

    use_graph = args.graph == 'on' or (args.graph == 'auto' and dist.world_size() == 1 and torch.cuda.is_available())
    if use_graph:
        # forward + backward + fused mp-SGD replayed as one graph; the first warm-up calls run eagerly
        # (kernel autotuning, arena construction) and the last one captures
        step = gluon.GraphStep(step, trainer, warmup=max(1, args.warmup - 1), fallback=args.graph == 'auto')
    first_loss = None
    trace = os.environ.get('MXAMD_BENCH_VERBOSE', '0') == '1'
    for i in range(args.warmup):
        out = step()
        if i == 0 or trace:
            v = float(out.mean().asscalar()) / loss_scale     # host read: outside the timed region
            first_loss = v if first_loss is None else first_loss
            if trace and rank == 0:
                print('warmup step %d loss %.4f' % (i, v), file=sys.stderr, flush=True)
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        last = step()
    sync()
    dt = time.perf_counter() - t0
    if dist.world_size() > 1:
        t = torch.tensor([dt], dtype=torch.float64, device='cuda' if torch.cuda.is_available() else 'cpu')
        dist.all_reduce(t, op='max')
        dt = float(t.item())
    ms = dt / args.steps * 1000.0
    n = dist.world_size()
    value = B * n * args.steps / dt
    if rank == 0:
        loss_val = float(last.mean().asscalar()) / loss_scale
        print(json.dumps({
            'metric': 'images/sec (whole node) ResNet-50 fp16 batch 256/GPU at 1/2/4/8 MI355X',
            'value': round(value, 2), 'unit': 'images/sec', 'n_gpus': n, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(ms, 3), 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': round(value / BASELINE_IMG_S, 3), 'dtype': {'float16': 'fp16', 'bfloat16': 'bf16',
                                                                         'float32': 'fp32'}[args.dtype],
            'data': 'synthetic (random-init weights, uniform images, random labels)',
            # the reference publishes no fp16 ResNet-50 *training* number: vs_baseline divides by its best
            # published training number, 1x V100 fp32 batch 128 -- not a same-config ratio
            'baseline': {'value': BASELINE_IMG_S, 'source': 'reference perf.md, 1x V100, fp32, batch 128, training',
                         'same_config': False},
            'config': {'model': args.model.replace('resnet50_v1b', 'ResNet-50 v1b'), 'global_batch': B * n,
                       'per_gpu_batch': B, 'seq_len': None, 'image_size': S, 'parallelism': 'dp%d' % n,
                       'layout': args.layout, 'optimizer': 'mp-SGD momentum 0.9, lr 0.1 (linear warm-up %d steps)' % warm,
                       'first_loss': None if first_loss is None else round(first_loss, 4),
                       'final_loss': round(loss_val, 4),
                       'hip_graph': bool(use_graph and getattr(step, 'captured', False))},
        }), flush=True)
    if os.environ.get('MXAMD_BENCH_VERBOSE', '0') == '1' and rank == 0:
        try:
            from mxnet_maintenance_amd.ops import kernel_fns
            times = kernel_fns.conv_algo_times()
            for k, v in sorted(kernel_fns.conv_algos().items(), key=str):
                t = ' '.join('%s=%.3f' % (n, ms) for n, ms in sorted(times.get(k, {}).items(), key=lambda z: z[1]))
                print('conv-algo', v, k, t, file=sys.stderr)
        except Exception as e:  # pragma: no cover
            print('conv-algo unavailable:', e, file=sys.stderr)
    if dist.world_size() > 1:
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    main()
