#!/usr/bin/env python
"""LSTM word language model training throughput (reference example/gluon/word_language_model).

standard_lstm_lm_650 (2x650 LSTM, embedding 650, vocab 10k), batch 32, BPTT 35, synthetic but
learnable token ids (every column walks one fixed random cycle through the vocabulary and the target
is the next token, so the loss falls from ln(vocab) as the model trains), SGD with gradient clipping -- one step = forward, softmax-CE over the vocabulary, backward
(BPTT through the in-tree recurrent kernels), clip, update.  MXAMD_RNN_VENDOR=1 runs the same
model on torch's fused (MIOpen) RNN for an A/B.

Usage: python tools/bench_lstm_lm.py [--steps 20] [--warmup 5] [--batch 32] [--bptt 35] [--dtype float32]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--bptt', type=int, default=35)
    ap.add_argument('--hidden', type=int, default=650)
    ap.add_argument('--vocab', type=int, default=10000)
    ap.add_argument('--dtype', default='float32', choices=['float32', 'float16', 'bfloat16'])
    ap.add_argument('--lr', type=float, default=20.0)
    args = ap.parse_args()
    import torch
    import mxnet_maintenance_amd as mx
    from mxnet_maintenance_amd import gluon, autograd, nd
    from mxnet_maintenance_amd.models import language_model as lm
    ctx = mx.gpu(0) if torch.cuda.is_available() else mx.cpu()
    mx.random.seed(3)
    net = lm.RNNModel('lstm', args.vocab, args.hidden, args.hidden, 2, 0.5)
    net.initialize(mx.init.Xavier(), ctx=ctx)
    if args.dtype != 'float32':
        net.cast(args.dtype)
    net.hybridize()
    # lr 20 with clipping at 0.25 per token, as the reference example trains this model
    trainer = gluon.Trainer(net.collect_params(), 'sgd', {'learning_rate': args.lr, 'momentum': 0.0,
                                                          'multi_precision': args.dtype != 'float32'})
    loss_fn = gluon.loss.SoftmaxCrossEntropyLoss()
    T, B = args.bptt, args.batch
    g = torch.Generator().manual_seed(7)
    cycle = torch.randperm(args.vocab, generator=g)
    pos = (torch.arange(T)[:, None] + 37 * torch.arange(B)[None, :]) % args.vocab
    data = nd.array(cycle[pos].numpy(), ctx=ctx)
    target = nd.array(cycle[(pos + 1) % args.vocab].numpy(), ctx=ctx)
    hidden = net.begin_state(batch_size=B, ctx=ctx, dtype=args.dtype)
    params = [p for p in net.collect_params().values() if p.grad_req != 'null']

    def step(hidden):
        hidden = lm.detach(hidden)
        with autograd.record():
            out, hidden = net(data, *hidden)
            L = loss_fn(out.reshape((-1, args.vocab)), target.reshape((-1,)))
        L.backward()
        grads = [p.grad(ctx) for p in params]
        gluon.utils.clip_global_norm(grads, 0.25 * T * B)
        trainer.step(T * B)
        return hidden, L

    first = None
    for i in range(args.warmup):
        hidden, L = step(hidden)
        if i == 0:
            first = float(L.astype('float32').mean().asscalar())
    nd.waitall()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        hidden, L = step(hidden)
    nd.waitall()
    dt = time.perf_counter() - t0
    print(json.dumps({'metric': 'LSTM LM training tokens/sec', 'value': round(T * B * args.steps / dt, 1),
                      'ms_per_step': round(dt / args.steps * 1e3, 3), 'steps': args.steps, 'dtype': args.dtype,
                      'rnn_path': 'torch-fused (MIOpen)' if os.environ.get('MXAMD_RNN_VENDOR') == '1'
                      else 'in-tree rnn.hip',
                      'rnn_dispatch': __import__('mxnet_maintenance_amd.ops.rnn_fns', fromlist=['x']).DISPATCH,
                      'config': {'model': 'standard_lstm_lm_%d' % args.hidden, 'batch': B, 'bptt': T,
                                 'vocab': args.vocab, 'first_loss': round(first, 4),
                                 'final_loss': round(float(L.astype('float32').mean().asscalar()), 4)}}), flush=True)


if __name__ == '__main__':
    main()
