"""Eager vs GraphStep on a small bf16 BERT (dropout 0): per-step loss and parameter drift (debug aid)."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import mxnet_maintenance_amd as mx
from mxnet_maintenance_amd import gluon, autograd, nd
from mxnet_maintenance_amd.models import bert as bert_mod


def run(graph, opt, steps=6, dtype='bfloat16', layers=2, units=256, V=1024, dropout=0.0, lr=1e-3, max_length=128):
    mx.random.seed(7)
    torch.manual_seed(7)
    B, S, P = 8, 64, 8
    net = bert_mod.BERTModel(vocab_size=V, units=units, hidden_size=4 * units, num_layers=layers,
                             num_heads=units // 64, max_length=max_length, dropout=dropout)
    net.initialize(mx.init.Normal(0.02), ctx=mx.gpu(0))
    net.cast(dtype)
    net.hybridize(static_alloc=True, static_shape=True)
    tr = gluon.Trainer(net.collect_params(), opt, {'learning_rate': lr, 'wd': 0.01, 'multi_precision': True})
    ce = gluon.loss.SoftmaxCrossEntropyLoss()
    g = torch.Generator().manual_seed(0)
    ctx = mx.gpu(0)
    tok = nd.array(torch.randint(0, V, (B, S), generator=g).numpy(), ctx=ctx)
    typ = nd.array(torch.randint(0, 2, (B, S), generator=g).numpy(), ctx=ctx)
    vl = nd.array(np.full((B,), S), ctx=ctx)
    pos = nd.array(torch.stack([torch.randperm(S, generator=g)[:P] for _ in range(B)]).numpy(), ctx=ctx)
    ml = nd.array(torch.randint(0, V, (B, P), generator=g).numpy(), ctx=ctx)
    nl = nd.array(torch.randint(0, 2, (B,), generator=g).numpy(), ctx=ctx)

    def step():
        with autograd.record():
            _s, _p, nsp, mlm = net(tok, typ, vl, pos)
            loss = ce(mlm.reshape((-1, V)), ml.reshape((-1,))).mean() + ce(nsp, nl).mean()
        loss.backward()
        tr.step(1)
        return loss

    f = gluon.GraphStep(step, tr, warmup=2) if graph else step
    out = []
    for i in range(steps):
        loss = f()
        if os.environ.get('NO_READ'):
            out.append((float(loss.asscalar()), [], None))
            continue
        torch.cuda.synchronize()
        ps = [(k.split('_', 1)[1], p.data().asnumpy().astype(np.float32)) for k, p in net.collect_params().items()]
        hp = tr._hyper.cpu().numpy().tolist() if getattr(tr, '_hyper', None) is not None else None
        out.append((float(loss.asscalar()), ps, hp))
    return out


if __name__ == '__main__':
    opt = sys.argv[1] if len(sys.argv) > 1 else 'lamb'
    kw = dict(layers=int(sys.argv[2]), units=int(sys.argv[3]), V=int(sys.argv[4]), dropout=float(sys.argv[5]),
              lr=float(sys.argv[6]), max_length=int(sys.argv[7]) if len(sys.argv) > 7 else 128) if len(sys.argv) > 6 else {}
    if os.environ.get('GRAPH_ONLY'):
        for i, (lg, _p, hp) in enumerate(run(True, opt, **kw)):
            print('step %d graph %.5f hp %s' % (i, lg, hp), flush=True)
        sys.exit(0)
    e = run(False, opt, **kw)
    g = run(True, opt, **kw)
    for i, ((le, pe, _), (lg, pg, hp)) in enumerate(zip(e, g)):
        worst = max(((k, float(np.abs(a - b).max())) for (k, a), (_, b) in zip(pe, pg)), key=lambda kv: kv[1])
        print('step %d eager %.5f graph %.5f  worst param diff %s %.3g  hp %s' % (i, le, lg, worst[0], worst[1], hp),
              flush=True)
