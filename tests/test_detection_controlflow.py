"""Detection operators and control-flow ops (parity: tests/python/unittest/test_contrib_operator.py,
test_operator.py::test_multibox_*, test_contrib_control_flow.py)."""
import numpy as np
import torch

import mxnet_maintenance_amd as mx
from mxnet_maintenance_amd import nd, autograd


def test_multibox_prior_layout():
    a = nd.contrib.MultiBoxPrior(nd.zeros((1, 3, 2, 2)), sizes=[0.5, 0.25], ratios=[1, 4])
    assert a.shape == (1, 2 * 2 * 3, 4)
    b = a.asnumpy()[0]
    # first pixel centre (0.25, 0.25): size 0.5 ratio 1, size 0.25 ratio 1, size 0.5 ratio 4
    np.testing.assert_allclose(b[0], [0, 0, 0.5, 0.5], atol=1e-6)
    np.testing.assert_allclose(b[1], [0.125, 0.125, 0.375, 0.375], atol=1e-6)
    np.testing.assert_allclose(b[2], [-0.25, 0.125, 0.75, 0.375], atol=1e-6)
    assert nd.contrib.MultiBoxPrior(nd.zeros((1, 3, 2, 2)), sizes=[0.9], clip=True).asnumpy().min() >= 0


def test_multibox_target_and_detection_roundtrip():
    anchors = nd.array([[[0.1, 0.1, 0.4, 0.4], [0.5, 0.5, 0.9, 0.9], [0.0, 0.6, 0.3, 0.9], [0.6, 0.0, 0.9, 0.3]]])
    label = nd.array([[[2, 0.12, 0.1, 0.42, 0.38], [-1, -1, -1, -1, -1]]])
    cls = nd.zeros((1, 4, 4))
    lt, lm, ct = nd.contrib.MultiBoxTarget(anchors, label, cls)
    np.testing.assert_array_equal(ct.asnumpy(), [[3, 0, 0, 0]])
    np.testing.assert_array_equal(lm.asnumpy()[0, :4], [1, 1, 1, 1])
    assert lm.asnumpy()[0, 4:].sum() == 0
    # decoding the loc target against its anchor recovers the ground-truth box
    probs = nd.array(np.array([[[0.1, 0.9, 0.9, 0.9], [0, 0, 0, 0], [0, 0.05, 0.05, 0.05], [0.9, 0.05, 0.05, 0.05]]],
                              dtype='float32'))
    det = nd.contrib.MultiBoxDetection(probs, lt, anchors, threshold=0.5, clip=False)
    d = det.asnumpy()[0]
    assert d[0, 0] == 2 and abs(d[0, 1] - 0.9) < 1e-6
    np.testing.assert_allclose(d[0, 2:], [0.12, 0.1, 0.42, 0.38], atol=1e-5)
    assert (d[1:, 0] == -1).all()


def test_multibox_target_negative_mining():
    a = nd.contrib.MultiBoxPrior(nd.zeros((1, 3, 4, 4)), sizes=[0.5, 0.25], ratios=[1, 2, 0.5])
    lab = nd.array([[[0, 0.1, 0.1, 0.4, 0.4], [1, 0.5, 0.5, 0.9, 0.9]]])
    cls = nd.random.uniform(shape=(1, 3, a.shape[1]))
    _, lm, ct = nd.contrib.MultiBoxTarget(a, lab, cls, negative_mining_ratio=3)
    c = ct.asnumpy()
    npos = (c > 0).sum()
    assert npos >= 2 and (c == 0).sum() == 3 * npos and (c == -1).sum() == c.size - 4 * npos
    assert lm.asnumpy().sum() == 4 * npos


def test_box_nms_iou_matching():
    data = nd.array([[[0, 0.9, 0, 0, 1, 1], [0, 0.8, 0.05, 0.05, 1, 1], [1, 0.7, 0, 0, 1, 1], [0, 0.6, 2, 2, 3, 3]]])
    out = nd.contrib.box_nms(data, overlap_thresh=0.5, id_index=0).asnumpy()[0]
    np.testing.assert_allclose(out[:, 1], [0.9, 0.7, 0.6, -1])
    out2 = nd.contrib.box_nms(data, overlap_thresh=0.5, id_index=0, force_suppress=True).asnumpy()[0]
    np.testing.assert_allclose(out2[:, 1], [0.9, 0.6, -1, -1])
    out3 = nd.contrib.box_nms(data, overlap_thresh=0.5, topk=1, coord_start=2, score_index=1).asnumpy()[0]
    assert out3[0, 1] == np.float32(0.9) and (out3[1:] == -1).all()
    iou = nd.contrib.box_iou(nd.array([[0, 0, 1, 1]]), nd.array([[0, 0, 1, 1], [0.5, 0, 1.5, 1], [2, 2, 3, 3]]))
    np.testing.assert_allclose(iou.asnumpy(), [[1, 1 / 3, 0]], atol=1e-6)
    iouc = nd.contrib.box_iou(nd.array([[0.5, 0.5, 1, 1]]), nd.array([[0, 0, 1, 1]]), format='center')
    np.testing.assert_allclose(iouc.asnumpy(), [[1 / 7]], atol=1e-6)
    r, c = nd.contrib.bipartite_matching(nd.array([[0.5, 0.6], [0.1, 0.9], [0.3, 0.2]]), threshold=0.01)
    np.testing.assert_array_equal(r.asnumpy(), [0, 1, -1])
    np.testing.assert_array_equal(c.asnumpy(), [0, 1])


def test_box_encode_decode_inverse():
    anchors = nd.array([[[0.1, 0.1, 0.5, 0.5], [0.2, 0.3, 0.6, 0.9]]])
    refs = nd.array([[[0.15, 0.1, 0.45, 0.6], [0.3, 0.3, 0.7, 0.8]]])
    t, m = nd.contrib.box_encode(nd.array([[1, 1]]), nd.array([[0, 1]]), anchors, refs,
                                 nd.array([0, 0, 0, 0]), nd.array([0.1, 0.1, 0.2, 0.2]))
    assert m.asnumpy().min() == 1
    dec = nd.contrib.box_decode(t, anchors, 0.1, 0.1, 0.2, 0.2, format='corner')
    np.testing.assert_allclose(dec.asnumpy(), refs.asnumpy(), atol=1e-5)


def test_roi_align_matches_bilinear_average():
    feat = np.arange(2 * 6 * 6, dtype='float32').reshape(2, 1, 6, 6)
    out = nd.contrib.ROIAlign(nd.array(feat), nd.array([[1, 0, 0, 3, 3]]), pooled_size=(2, 2), spatial_scale=1.0,
                              sample_ratio=2).asnumpy()
    # plane is linear (v = 36 + 6y + x) so each bin is the value at its sample centroid
    np.testing.assert_allclose(out[0, 0], [[36 + 6 * 0.75 + 0.75, 36 + 6 * 0.75 + 2.25],
                                           [36 + 6 * 2.25 + 0.75, 36 + 6 * 2.25 + 2.25]], atol=1e-4)
    x = nd.array(np.random.rand(1, 4, 8, 8).astype('float32'))
    x.attach_grad()
    with autograd.record():
        y = nd.contrib.ROIAlign(x, nd.array([[0, 1, 1, 6, 6]]), pooled_size=(2, 2), spatial_scale=1.0)
    y.backward()
    assert y.shape == (1, 4, 2, 2) and x.grad.asnumpy().sum() > 0


def test_multi_proposal_shapes():
    A = 12
    p = nd.contrib.MultiProposal(nd.random.uniform(shape=(2, 2 * A, 5, 5)),
                                 nd.random.normal(0, 0.1, shape=(2, 4 * A, 5, 5)), nd.array([[80, 80, 1]] * 2),
                                 rpn_pre_nms_top_n=50, rpn_post_nms_top_n=10, rpn_min_size=2, output_score=True)
    rois, scores = p
    assert rois.shape == (20, 5) and scores.shape == (20, 1)
    r = rois.asnumpy()
    assert set(r[:, 0].tolist()) == {0.0, 1.0} and (r[:, 1:] >= 0).all() and (r[:, 1:] <= 79).all()


def test_foreach_imperative_and_symbolic():
    def step(x, states):
        s = states[0] + x
        return s * 2, [s]
    data = nd.array([[0, 1], [2, 3], [4, 5]])
    outs, st = nd.contrib.foreach(step, data, [nd.zeros((2,))])
    np.testing.assert_allclose(outs.asnumpy(), [[0, 2], [4, 8], [12, 18]])
    np.testing.assert_allclose(st[0].asnumpy(), [6, 9])
    d = mx.sym.var('d')
    w = mx.sym.var('w')
    s0 = mx.sym.var('s0')

    def body(x, states):
        s = states[0] + x * w
        return s, [s]
    o, _ = mx.sym.contrib.foreach(body, d, [s0])
    g = mx.sym.load_json(o.tojson())
    ex = g.simple_bind(mx.cpu(), d=(3, 2), w=(2,), s0=(2,))
    ex.arg_dict['d'][:] = data
    ex.arg_dict['w'][:] = nd.array([1, 1])
    ex.arg_dict['s0'][:] = 0
    out = ex.forward(is_train=True)[0]
    np.testing.assert_allclose(out.asnumpy(), [[0, 1], [2, 4], [6, 9]])
    ex.backward(nd.ones((3, 2)))
    # d(sum over t of cumulative sums)/dw = sum_t (T - t) * d_t
    np.testing.assert_allclose(ex.grad_dict['w'].asnumpy(), [3 * 0 + 2 * 2 + 1 * 4, 3 * 1 + 2 * 3 + 1 * 5])


def test_while_loop_and_cond():
    outs, (i, acc) = nd.contrib.while_loop(lambda i, a: i < 5, lambda i, a: (a + i, (i + 1, a + i)),
                                           (nd.array([0]), nd.array([0])), max_iterations=8)
    assert outs.shape[0] == 8 and int(i.asscalar()) == 5 and int(acc.asscalar()) == 10
    np.testing.assert_allclose(outs.asnumpy()[:5, 0], [0, 1, 3, 6, 10])
    a, b = nd.array([3.0]), nd.array([4.0])
    r = nd.contrib.cond(a < b, lambda: a * 2, lambda: b * 2)
    assert float(r.asscalar()) == 6.0
    r2 = nd.contrib.cond(a > b, lambda: a * 2, lambda: b * 2)
    assert float(r2.asscalar()) == 8.0
    x = mx.sym.var('x')
    y = mx.sym.var('y')
    c = mx.sym.contrib.cond(x < y, lambda: x + y, lambda: x - y)
    ex = c.bind(mx.cpu(), {'x': nd.array([1.0]), 'y': nd.array([5.0])})
    assert float(ex.forward()[0].asscalar()) == 6.0
