"""Data pipeline: mx.io iterators, mx.image, gluon.data (parity: test_io.py, test_image.py,
test_gluon_data.py, test_gluon_data_vision.py)."""
import io as _io
import os
import tempfile

import numpy as np
import pytest

import mxnet_maintenance_amd as mx
from mxnet_maintenance_amd import nd, recordio
from mxnet_maintenance_amd.gluon import data as gdata
from mxnet_maintenance_amd.gluon.data.vision import transforms as T


def _png(a):
    from PIL import Image
    b = _io.BytesIO()
    Image.fromarray(a).save(b, format='PNG')
    return b.getvalue()


def test_ndarrayiter_pad_discard_rollover():
    data = np.arange(10 * 2).reshape(10, 2).astype(np.float32)
    label = np.arange(10).astype(np.float32)
    it = mx.io.NDArrayIter(data, label, batch_size=4, last_batch_handle='pad')
    batches = list(it)
    assert len(batches) == 3 and batches[-1].pad == 2
    np.testing.assert_array_equal(batches[-1].label[0].asnumpy(), [8, 9, 0, 1])
    assert it.provide_data[0].name == 'data' and it.provide_data[0].shape == (4, 2)
    assert it.provide_label[0].name == 'softmax_label'
    it = mx.io.NDArrayIter(data, label, batch_size=4, last_batch_handle='discard')
    assert len(list(it)) == 2
    it = mx.io.NDArrayIter(data, label, batch_size=4, last_batch_handle='roll_over')
    assert len(list(it)) == 2
    it.reset()
    first = next(it)
    np.testing.assert_array_equal(first.label[0].asnumpy(), [8, 9, 0, 1])
    assert first.pad == 2
    it = mx.io.NDArrayIter({'a': data, 'b': data}, batch_size=5, shuffle=True)
    assert sorted(d.name for d in it.provide_data) == ['a', 'b']
    b = next(it)
    np.testing.assert_array_equal(b.data[0].asnumpy(), b.data[1].asnumpy())


def test_resize_and_prefetching_iter():
    data = np.random.rand(12, 3).astype(np.float32)
    it = mx.io.NDArrayIter(data, np.zeros(12), batch_size=4)
    r = mx.io.ResizeIter(it, 5)
    assert len(list(r)) == 5
    p = mx.io.PrefetchingIter(mx.io.NDArrayIter(data, np.zeros(12), batch_size=4))
    assert len(list(p)) == 3
    p.reset()
    assert len(list(p)) == 3


def test_csv_and_libsvm_iter():
    with tempfile.TemporaryDirectory() as d:
        f = os.path.join(d, 'x.csv')
        np.savetxt(f, np.arange(24).reshape(6, 4), delimiter=',')
        lf = os.path.join(d, 'y.csv')
        np.savetxt(lf, np.arange(6), delimiter=',')
        it = mx.io.CSVIter(data_csv=f, data_shape=(2, 2), label_csv=lf, batch_size=4)
        bs = list(it)
        assert bs[0].data[0].shape == (4, 2, 2) and bs[1].pad == 2
        np.testing.assert_array_equal(bs[0].label[0].asnumpy(), [0, 1, 2, 3])
        s = os.path.join(d, 'x.svm')
        with open(s, 'w') as fo:
            fo.write('1 0:1.5 3:2\n0 1:1\n1 2:3\n')
        it = mx.io.LibSVMIter(data_libsvm=s, data_shape=(4,), batch_size=2)
        b = next(it)
        assert b.data[0].stype == 'csr'
        np.testing.assert_allclose(b.data[0].asnumpy()[0], [1.5, 0, 0, 2])


def test_mnist_iter():
    import gzip
    import struct
    with tempfile.TemporaryDirectory() as d:
        imgs = (np.random.rand(20, 28, 28) * 255).astype(np.uint8)
        labs = np.arange(20).astype(np.uint8) % 10
        with gzip.open(os.path.join(d, 'img.gz'), 'wb') as f:
            f.write(struct.pack('>IIII', 2051, 20, 28, 28) + imgs.tobytes())
        with gzip.open(os.path.join(d, 'lab.gz'), 'wb') as f:
            f.write(struct.pack('>II', 2049, 20) + labs.tobytes())
        it = mx.io.MNISTIter(image=os.path.join(d, 'img.gz'), label=os.path.join(d, 'lab.gz'), batch_size=8,
                             shuffle=False, flat=True)
        b = next(it)
        assert b.data[0].shape == (8, 784)
        np.testing.assert_allclose(b.data[0].asnumpy()[0], imgs[0].reshape(-1) / 255.0, rtol=1e-6)


def _make_image_rec(d, n=6, size=(24, 32)):
    rec, idx = os.path.join(d, 'im.rec'), os.path.join(d, 'im.idx')
    w = recordio.MXIndexedRecordIO(idx, rec, 'w')
    imgs = []
    for i in range(n):
        a = (np.random.rand(size[0], size[1], 3) * 255).astype(np.uint8)
        imgs.append(a)
        w.write_idx(i, recordio.pack(recordio.IRHeader(0, float(i), i, 0), _png(a)))
    w.close()
    return rec, idx, imgs


def test_image_record_iter_and_image_iter():
    with tempfile.TemporaryDirectory() as d:
        rec, idx, imgs = _make_image_rec(d)
        it = mx.io.ImageRecordIter(path_imgrec=rec, data_shape=(3, 16, 16), batch_size=4, mean_r=10, std_r=2)
        b = next(it)
        assert b.data[0].shape == (4, 3, 16, 16)
        np.testing.assert_array_equal(b.label[0].asnumpy(), [0, 1, 2, 3])
        crop = imgs[0][4:20, 8:24].astype(np.float32).transpose(2, 0, 1)
        crop[0] = (crop[0] - 10) / 2
        np.testing.assert_allclose(b.data[0].asnumpy()[0], crop, atol=1e-4)
        b2 = next(it)
        assert b2.pad == 2
        with pytest.raises(StopIteration):
            next(it)
        ii = mx.image.ImageIter(batch_size=3, data_shape=(3, 16, 16), path_imgrec=rec, path_imgidx=idx,
                                shuffle=True, rand_crop=True, rand_mirror=True)
        b = next(ii)
        assert b.data[0].shape == (3, 3, 16, 16)
        assert sorted(b.label[0].asnumpy().tolist()) == sorted(set(b.label[0].asnumpy().tolist()))
        ds = gdata.vision.ImageRecordDataset(rec)
        x, y = ds[2]
        assert x.shape == (24, 32, 3) and y == 2.0
        np.testing.assert_array_equal(x.asnumpy(), imgs[2])


def test_image_functions_and_augmenters():
    a = (np.random.rand(40, 60, 3) * 255).astype(np.uint8)
    img = mx.image.imdecode(_png(a))
    np.testing.assert_array_equal(img.asnumpy(), a)
    assert mx.image.resize_short(img, 20).shape == (20, 30, 3)
    out, box = mx.image.center_crop(img, (16, 20))
    assert out.shape == (20, 16, 3) and box == (22, 10, 16, 20)
    out, _ = mx.image.random_size_crop(img, (10, 10), 0.3, (0.75, 1.33))
    assert out.shape == (10, 10, 3)
    bgr = mx.image.imdecode(_png(a), to_rgb=0)
    np.testing.assert_array_equal(bgr.asnumpy(), a[:, :, ::-1])
    augs = mx.image.CreateAugmenter((3, 24, 24), resize=30, rand_crop=True, rand_resize=True, rand_mirror=True,
                                    mean=True, std=True, brightness=.1, contrast=.1, saturation=.1, hue=.1,
                                    pca_noise=.1, rand_gray=.1)
    x = img
    for t in augs:
        x = t(x)
        t.dumps()
    assert x.shape == (24, 24, 3)
    rot = mx.image.imrotate(nd.ones((1, 3, 8, 8)), 90)
    assert rot.shape == (1, 3, 8, 8)


def test_detection_augmenters():
    img = nd.array((np.random.rand(50, 60, 3) * 255).astype(np.uint8), dtype='uint8')
    label = np.array([[0, 0.1, 0.1, 0.5, 0.6], [1, 0.4, 0.3, 0.9, 0.9]], dtype=np.float32)
    augs = mx.image.CreateDetAugmenter((3, 32, 32), rand_crop=1, rand_pad=1, rand_mirror=True, mean=True,
                                       std=True, brightness=0.1)
    for _ in range(5):
        x, lab = img, label.copy()
        for a in augs:
            x, lab = a(x, lab)
        assert x.shape == (32, 32, 3)
        assert lab.shape[1] == 5 and (lab[:, 1:] >= 0).all() and (lab[:, 1:] <= 1).all()
    f = mx.image.DetHorizontalFlipAug(1.0)
    _, l2 = f(img, label.copy())
    np.testing.assert_allclose(l2[0, 1:5:2], [0.5, 0.9])


def test_gluon_dataset_sampler_loader():
    ds = gdata.ArrayDataset(np.random.rand(10, 4).astype('float32'), np.arange(10))
    assert len(ds.shard(3, 0)) == 4 and len(ds.shard(3, 2)) == 3
    assert len(ds.take(4)) == 4
    assert len(ds.filter(lambda s: s[1] % 2 == 0)) == 5
    assert ds.transform_first(lambda x: x * 2)[1][1] == 1
    bs = gdata.BatchSampler(gdata.SequentialSampler(10), 3, 'rollover')
    assert [len(b) for b in bs] == [3, 3, 3]
    assert list(bs)[0] == [9, 0, 1]
    assert list(gdata.IntervalSampler(6, 3)) == [0, 3, 1, 4, 2, 5]
    for kw in [{}, {'num_workers': 2}, {'num_workers': 2, 'thread_pool': True}]:
        dl = gdata.DataLoader(ds, batch_size=4, **kw)
        got = [(x.shape, y.asnumpy().tolist()) for x, y in dl]
        assert got[0][1] == [0, 1, 2, 3] and got[-1][0] == (2, 4), kw
        assert len(dl) == 3


def test_vision_transforms():
    img = nd.array((np.random.rand(32, 40, 3) * 255).astype('uint8'), dtype='uint8')
    t = T.Compose([T.Resize(20), T.CenterCrop(16), T.RandomFlipLeftRight(), T.RandomColorJitter(.1, .1, .1, .1),
                   T.RandomLighting(.1), T.ToTensor(), T.Normalize(0.5, 0.2)])
    y = t(img)
    assert y.shape == (3, 16, 16) and str(y.dtype) == 'float32' or y.dtype == np.float32
    x = T.ToTensor()(img)
    np.testing.assert_allclose(x.asnumpy(), img.asnumpy().transpose(2, 0, 1) / 255.0, rtol=1e-6)
    n = T.Normalize((0.1, 0.2, 0.3), (1, 2, 3))(x)
    np.testing.assert_allclose(n.asnumpy()[1], (x.asnumpy()[1] - 0.2) / 2, rtol=1e-5)
    assert T.RandomResizedCrop(12)(img).shape == (12, 12, 3)
    assert T.CropResize(0, 0, 10, 10, 5)(img).shape == (5, 5, 3)
    assert T.RandomCrop(30, pad=2)(img).shape == (30, 30, 3)
    assert T.Rotate(10)(x).shape == (3, 32, 40)


def test_image_record_iter_decodes_on_engine_and_propagates_errors():
    from mxnet_maintenance_amd import engine
    with tempfile.TemporaryDirectory() as d:
        rec, idx, imgs = _make_image_rec(d)
        before = getattr(engine.get(), 'executed', 0)
        it = mx.io.ImageRecordIter(path_imgrec=rec, data_shape=(3, 16, 16), batch_size=2)
        batches = list(it)
        assert len(batches) == 3
        if engine.native_available():
            assert engine.get().executed - before >= 6      # one engine task per decoded image
        # a record that is not an image: the worker's exception surfaces in next()
        bad = os.path.join(d, 'bad.rec')
        w = recordio.MXRecordIO(bad, 'w')
        for i in range(2):
            w.write(recordio.pack(recordio.IRHeader(0, float(i), i, 0), b'not an image'))
        w.close()
        it = mx.io.ImageRecordIter(path_imgrec=bad, data_shape=(3, 16, 16), batch_size=2)
        with pytest.raises(Exception):
            next(it)
