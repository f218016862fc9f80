"""Model families beyond the vision zoo: BERT (transformer contrib ops), RNN language model.
Parity: tests/python/unittest/test_operator.py::test_multihead_attention_selfatt / encdec,
example/gluon/word_language_model."""
import numpy as onp
import torch

import mxnet_maintenance_amd as mx
from mxnet_maintenance_amd import nd, autograd, gluon, models


def _mha_reference(qkv, heads):
    """Plain fp32 multi-head self-attention on the interleaved (S,B,H*3*D) layout."""
    S, B, C = qkv.shape
    D = C // (3 * heads)
    t = torch.as_tensor(qkv).reshape(S, B, heads, 3, D)
    q, k, v = [t[:, :, :, i].permute(1, 2, 0, 3) for i in range(3)]           # (B,H,S,D)
    att = torch.softmax(q @ k.transpose(-1, -2) / D ** 0.5, -1)
    return (att @ v).permute(2, 0, 1, 3).reshape(S, B, heads * D).numpy(), att


def test_interleaved_selfatt_ops_match_reference():
    S, B, H, D = 6, 2, 3, 4
    x = onp.random.RandomState(0).randn(S, B, H * 3 * D).astype('float32')
    X = nd.array(x)
    X.attach_grad()
    with autograd.record():
        sc = nd.contrib.interleaved_matmul_selfatt_qk(X, heads=H)
        att = nd.softmax(sc, axis=-1)
        out = nd.contrib.interleaved_matmul_selfatt_valatt(X, att, heads=H)
    out.backward(nd.ones_like(out))
    ref, ref_att = _mha_reference(x, H)
    onp.testing.assert_allclose(out.asnumpy(), ref, rtol=1e-5, atol=1e-5)
    onp.testing.assert_allclose(att.asnumpy(), ref_att.reshape(B * H, S, S).numpy(), rtol=1e-5, atol=1e-6)
    t = torch.tensor(x, requires_grad=True)
    S_, B_, C_ = t.shape
    tt = t.reshape(S, B, H, 3, D)
    q, k, v = [tt[:, :, :, i].permute(1, 2, 0, 3) for i in range(3)]
    o = (torch.softmax(q @ k.transpose(-1, -2) / D ** 0.5, -1) @ v).permute(2, 0, 1, 3).reshape(S, B, H * D)
    o.sum().backward()
    onp.testing.assert_allclose(X.grad.asnumpy(), t.grad.numpy(), rtol=1e-4, atol=1e-5)
    fused = nd.contrib.sdp_attention(X, heads=H)
    onp.testing.assert_allclose(fused.asnumpy(), ref, rtol=1e-5, atol=1e-5)


def test_encdec_ops():
    Sq, Sk, B, H, D = 3, 5, 2, 2, 4
    rng = onp.random.RandomState(1)
    q = rng.randn(Sq, B, H * D).astype('float32')
    kv = rng.randn(Sk, B, H * 2 * D).astype('float32')
    sc = nd.contrib.interleaved_matmul_encdec_qk(nd.array(q), nd.array(kv), heads=H)
    assert sc.shape == (B * H, Sq, Sk)
    qt = torch.tensor(q).reshape(Sq, B, H, D).permute(1, 2, 0, 3)
    kvt = torch.tensor(kv).reshape(Sk, B, H, 2, D)
    kt, vt = kvt[:, :, :, 0].permute(1, 2, 0, 3), kvt[:, :, :, 1].permute(1, 2, 0, 3)
    ref = (qt @ kt.transpose(-1, -2) / D ** 0.5).reshape(B * H, Sq, Sk)
    onp.testing.assert_allclose(sc.asnumpy(), ref.numpy(), rtol=1e-5, atol=1e-5)
    att = nd.softmax(sc, axis=-1)
    o = nd.contrib.interleaved_matmul_encdec_valatt(nd.array(kv), att, heads=H)
    ro = (torch.tensor(att.asnumpy()).reshape(B, H, Sq, Sk) @ vt).permute(2, 0, 1, 3).reshape(Sq, B, H * D)
    onp.testing.assert_allclose(o.asnumpy(), ro.numpy(), rtol=1e-5, atol=1e-5)


def test_bert_forward_backward_hybridize():
    net = models.get_bert_model('bert_12_768_12', vocab_size=100, num_layers=2, units=64, hidden_size=128,
                                num_heads=4, max_length=32)
    net.initialize()
    B, S = 2, 8
    rng = onp.random.RandomState(0)
    inp = nd.array(rng.randint(0, 100, (B, S)))
    tt = nd.zeros((B, S))
    vl = nd.array([5, 8])
    mp = nd.array([[1, 2], [3, 4]])
    seq, pooled, nsp, mlm = net(inp, tt, vl, mp)
    assert seq.shape == (B, S, 64) and pooled.shape == (B, 64) and nsp.shape == (B, 2) and mlm.shape == (B, 2, 100)
    # padding positions do not influence valid positions
    inp2 = inp.copy()
    inp2[0, 6] = (int(inp2[0, 6].asscalar()) + 1) % 100
    seq2 = net(inp2, tt, vl, mp)[0]
    onp.testing.assert_allclose(seq2[0, :5].asnumpy(), seq[0, :5].asnumpy(), rtol=1e-5, atol=1e-5)
    net.hybridize()
    h = net(inp, tt, vl, mp)
    onp.testing.assert_allclose(h[3].asnumpy(), mlm.asnumpy(), rtol=1e-5, atol=1e-5)
    tr = gluon.Trainer(net.collect_params(), 'adam', {'learning_rate': 1e-3})
    lossf = gluon.loss.SoftmaxCrossEntropyLoss()
    labels = nd.array(rng.randint(0, 100, (B, 2)))
    first = None
    for _ in range(5):
        with autograd.record():
            out = net(inp, tt, vl, mp)
            loss = lossf(out[3], labels).mean() + lossf(out[2], nd.array([0, 1])).mean()
        loss.backward()
        tr.step(1)
        first = first if first is not None else float(loss.asscalar())
    assert float(loss.asscalar()) < first


def test_rnn_language_model_trains():
    lm = models.RNNModel('lstm', vocab_size=20, num_embed=16, num_hidden=16, num_layers=1, dropout=0.0,
                         tie_weights=True)
    lm.initialize(mx.init.Xavier())
    tr = gluon.Trainer(lm.collect_params(), 'adam', {'learning_rate': 0.02})
    assert lm.decoder.weight is lm.encoder.weight   # tied decoder shares the embedding matrix
    seq = onp.tile(onp.arange(10), 8)
    data = nd.array(seq[:-1].reshape(-1, 1)[:70])
    target = nd.array(seq[1:].reshape(-1, 1)[:70])
    lossf = gluon.loss.SoftmaxCrossEntropyLoss()
    losses = []
    for _ in range(60):
        states = lm.begin_state(batch_size=1)
        with autograd.record():
            out, states = lm(data, *states)
            loss = lossf(out.reshape((-1, 20)), target.reshape((-1,))).mean()
        loss.backward()
        gluon.utils.clip_global_norm([p.grad() for p in lm.collect_params().values()], 1.0)
        tr.step(1)
        losses.append(float(loss.asscalar()))
    assert losses[-1] < 0.5 * losses[0]
    assert models.language_model.detach(states)[0].shape == (1, 1, 16)


def test_lenet5_synthetic_mnist_cpu_kvstore_local():
    """BASELINE.json config 1: LeNet-5 on synthetic MNIST through Gluon imperative mode on mx.cpu()
    with KVStore('local'); training must reduce the loss and fit the (learnable) synthetic labels."""
    import numpy as np
    import mxnet_maintenance_amd as mx
    from mxnet_maintenance_amd import gluon, autograd, nd
    mx.random.seed(0)
    rs = np.random.RandomState(0)
    protos = rs.rand(10, 1, 28, 28).astype('float32')
    y = rs.randint(0, 10, size=256)
    x = protos[y] + 0.1 * rs.randn(256, 1, 28, 28).astype('float32')
    net = gluon.nn.Sequential()
    net.add(gluon.nn.Conv2D(6, 5, padding=2, activation='tanh'), gluon.nn.AvgPool2D(2, 2),
            gluon.nn.Conv2D(16, 5, activation='tanh'), gluon.nn.AvgPool2D(2, 2), gluon.nn.Flatten(),
            gluon.nn.Dense(120, activation='tanh'), gluon.nn.Dense(84, activation='tanh'), gluon.nn.Dense(10))
    net.initialize(mx.init.Xavier(), ctx=mx.cpu())
    kv = mx.kv.create('local')
    trainer = gluon.Trainer(net.collect_params(), 'adam', {'learning_rate': 0.003}, kvstore=kv)
    loss_fn = gluon.loss.SoftmaxCrossEntropyLoss()
    data = gluon.data.DataLoader(gluon.data.ArrayDataset(x, y.astype('float32')), batch_size=32, shuffle=True)
    first = last = None
    for epoch in range(4):
        tot = 0.0
        for xb, yb in data:
            with autograd.record():
                loss = loss_fn(net(xb), yb)
            loss.backward()
            trainer.step(xb.shape[0])
            tot += float(loss.mean().asscalar())
        first = tot if first is None else first
        last = tot
    acc = mx.metric.Accuracy()
    acc.update([nd.array(y)], [net(nd.array(x))])
    assert last < first * 0.5 and acc.get()[1] > 0.9, (first, last, acc.get())
