#!/usr/bin/env python
"""BERT pre-training throughput (BASELINE.json config 4: BERT-base, seq 128, bf16).

One step = embeddings + 12 encoder layers (fused QKV projection, SDPA attention,
LayerNorm / GELU / dropout HIP kernels) + MLM (20 masked positions per
sequence, tied decoder) + NSP heads, softmax-CE losses, backward, bucketed
gradient all-reduce (N > 1, torch.distributed.run) and a fused flat-arena
LAMB (default) or AdamW update.  Synthetic token ids / random-init weights.

Usage: python tools/bench_bert.py [--batch 32] [--seq 128] [--steps 20] [--warmup 5]
       [--model bert_12_768_12] [--optimizer lamb|adamw] [--dtype bfloat16] [--graph]
Prints one JSON line (tokens/s and sequences/s for the whole job).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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
    ap.add_argument('--batch', type=int, default=32, help='per-GPU sequences')
    ap.add_argument('--seq', type=int, default=128)
    ap.add_argument('--masked', type=int, default=20)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--model', default='bert_12_768_12')
    ap.add_argument('--optimizer', default='lamb', choices=['lamb', 'adamw', 'adam'])
    ap.add_argument('--dtype', default='bfloat16', choices=['bfloat16', 'float16', 'float32'])
    ap.add_argument('--vocab', type=int, default=30528, help='30522 padded to a multiple of 64')
    ap.add_argument('--gpus', type=int, default=1, help='worker processes (one per GPU)')
    ap.add_argument('--graph', action='store_true', help='capture the whole step in a HIP graph (GraphStep)')
    ap.add_argument('--trace-loss', action='store_true', help='print every step\'s loss (debugging; syncs)')
    ap.add_argument('--gemm-table', default=os.path.join(os.path.dirname(os.path.abspath(__file__)), 'tunableop',
                                                          'bert_base_b32_s128_bf16_gfx950.csv'),
                    help='hipBLASLt/rocBLAS solution table (PyTorch TunableOp CSV) for the library GEMMs; '
                         '"none" keeps the library heuristics, "tune" measures a new one')
    args = ap.parse_args()
    launch = _load_launcher()
    if launch.needs_launch(args.gpus):
        sys.exit(launch.relaunch_self(args.gpus))

    import torch
    if os.environ.get('MXAMD_FILL_UNINIT'):
        # debugging: torch.empty returns NaN-filled memory, exposing reads of unwritten buffers
        torch.use_deterministic_algorithms(True, warn_only=True)
        torch.utils.deterministic.fill_uninitialized_memory = True
    if args.gemm_table != 'none' and torch.cuda.is_available():
        # per-shape library GEMM solutions measured on gfx950 (tools/tunableop/; +2-3 % here): the table
        # is read, not re-tuned, unless --gemm-table tune; shapes it lacks keep the default heuristics
        import torch.cuda.tunable as tunable
        tunable.enable(True)
        if args.gemm_table == 'tune':
            tunable.tuning_enable(True)
        elif os.path.exists(args.gemm_table) and (args.batch, args.seq) == (32, 128):
            import tempfile
            tunable.tuning_enable(False)
            # results the run writes at exit go to a scratch file, never over the committed table
            tunable.set_filename(os.path.join(tempfile.gettempdir(), 'mxamd_tunableop_%d.csv' % os.getpid()))
            tunable.read_file(args.gemm_table)
        else:
            tunable.enable(False)
    import mxnet_maintenance_amd as mx
    from mxnet_maintenance_amd import gluon, autograd, nd
    from mxnet_maintenance_amd.models import bert as bert_mod
    from mxnet_maintenance_amd.parallel import dist

    if int(os.environ.get('WORLD_SIZE', '1')) > 1:
        dist.init()
    rank = dist.rank()
    # one process per GPU; ranks beyond the visible devices share them (single-GPU rehearsals)
    dev = dist.local_rank() % max(1, torch.cuda.device_count()) if torch.cuda.is_available() else 0
    ctx = mx.gpu(dev) if torch.cuda.is_available() else mx.cpu()
    if torch.cuda.is_available():
        torch.cuda.set_device(dev)
    mx.random.seed(4321 + rank)
    B, S, P = args.batch, args.seq, args.masked
    net = bert_mod.get_bert_model(args.model, vocab_size=args.vocab)
    net.initialize(mx.init.Normal(0.02), ctx=ctx)
    if args.dtype != 'float32':
        net.cast(args.dtype)
    net.hybridize(static_alloc=True, static_shape=True)
    opt_params = {'learning_rate': 1e-4, 'wd': 0.01, 'multi_precision': args.dtype != 'float32'}
    trainer = gluon.Trainer(net.collect_params(), args.optimizer, opt_params, kvstore='device')
    ce = gluon.loss.SoftmaxCrossEntropyLoss()

    g = torch.Generator().manual_seed(rank)
    tokens = nd.array(torch.randint(0, args.vocab, (B, S), generator=g).numpy(), ctx=ctx)
    types = nd.array(torch.randint(0, 2, (B, S), generator=g).numpy(), ctx=ctx)
    valid = nd.array(torch.full((B,), S).numpy(), ctx=ctx)
    pos = nd.array(torch.stack([torch.randperm(S, generator=g)[:P] for _ in range(B)]).numpy(), ctx=ctx)
    mlm_label = nd.array(torch.randint(0, args.vocab, (B, P), generator=g).numpy(), ctx=ctx)
    nsp_label = nd.array(torch.randint(0, 2, (B,), generator=g).numpy(), ctx=ctx)

    def step():
        with autograd.record():
            _seq, _pooled, nsp, mlm = net(tokens, types, valid, pos)
            loss = ce(mlm.reshape((-1, args.vocab)), mlm_label.reshape((-1,))).mean() + ce(nsp, nsp_label).mean()
        loss.backward()
        trainer.step(dist.world_size())   # per-rank mean loss; RCCL sums the ranks
        return loss

    def sync():
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        dist.barrier()

    if args.graph:
        step = gluon.GraphStep(step, trainer, warmup=max(1, args.warmup - 1))
    for i in range(args.warmup):
        r = step()
        if args.trace_loss:
            print('warmup step %d loss %.5f' % (i, float(r.asscalar())), flush=True)
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        last = step()
        if args.trace_loss:
            print('step %d loss %.5f' % (i, float(last.asscalar())), flush=True)
    sync()
    dt = time.perf_counter() - t0
    if dist.world_size() > 1:
        t = torch.tensor([dt], dtype=torch.float64, device='cuda' if torch.cuda.is_available() else 'cpu')
        dist.all_reduce(t, op='max')
        dt = float(t.item())
    n = dist.world_size()
    if rank == 0:
        print(json.dumps({
            'metric': 'BERT pre-training tokens/sec (whole job)', 'value': round(B * S * n * args.steps / dt, 1),
            'unit': 'tokens/sec', 'sequences_per_sec': round(B * n * args.steps / dt, 2), 'n_gpus': n,
            'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(dt / args.steps * 1000, 3),
            'dtype': {'bfloat16': 'bf16', 'float16': 'fp16', 'float32': 'fp32'}[args.dtype],
            'data': 'synthetic token ids, random-init weights',
            'config': {'model': args.model, 'per_gpu_batch': B, 'seq_len': S, 'masked_positions': P,
                       'optimizer': args.optimizer, 'parallelism': 'dp%d' % n, 'hip_graph': args.graph,
                       'final_loss': round(float(last.asscalar()), 4)}}), flush=True)
    if args.trace_loss or os.environ.get('MXAMD_BENCH_VERBOSE', '0') == '1':
        from mxnet_maintenance_amd.ops import kernel_fns
        times = kernel_fns.conv_algo_times()
        for k, v in sorted(kernel_fns._ALGO.items(), key=str):
            t = ' '.join('%s=%.3f' % (n, ms) for n, ms in sorted(times.get(k, {}).items(), key=lambda z: z[1]))
            print('algo', v, k, t, file=sys.stderr)
    if dist.world_size() > 1:
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
