"""Vision datasets (parity: python/mxnet/gluon/data/vision/datasets.py).

There is no network access on the target nodes, so the download step of the
reference is replaced by a clear error when the expected files are absent;
file formats (MNIST idx, CIFAR binary batches, RecordIO, image folders/lists)
are read exactly as the reference reads them.
"""
import gzip
import os
import struct
import warnings

import numpy as np

from ..dataset import Dataset, _DownloadedDataset, RecordFileDataset
from .... import image, recordio
from .... import ndarray as nd
from ....base import MXNetError

__all__ = ['MNIST', 'FashionMNIST', 'CIFAR10', 'CIFAR100', 'ImageRecordDataset', 'ImageFolderDataset',
           'ImageListDataset']


def _data_dir():
    return os.environ.get('MXNET_HOME', os.path.join(os.path.expanduser('~'), '.mxnet'))


def _find(root, names):
    for n in names:
        p = os.path.join(root, n)
        if os.path.exists(p):
            return p
    raise MXNetError('dataset file %s not found under %s (no network: place the files there)' % (names[0], root))


def _open(path):
    return gzip.open(path, 'rb') if path.endswith('.gz') else open(path, 'rb')


class MNIST(_DownloadedDataset):
    """MNIST handwritten digits: (28, 28, 1) uint8 images, int32 labels."""

    _files = {True: ('train-images-idx3-ubyte', 'train-labels-idx1-ubyte'),
              False: ('t10k-images-idx3-ubyte', 't10k-labels-idx1-ubyte')}

    def __init__(self, root=os.path.join(_data_dir(), 'datasets', 'mnist'), train=True, transform=None):
        self._train = train
        super().__init__(root, transform)

    def _get_data(self):
        img_name, lab_name = self._files[self._train]
        from .... import test_utils
        if type(self) is MNIST and test_utils._synthetic_enabled() and not any(
                os.path.exists(os.path.join(self._root, n + e)) for n in (lab_name,) for e in ('', '.gz')):
            # MXNET_TEST_SYNTHETIC_DATA=1 (reference-test harness only): random-pixel idx files
            test_utils.get_mnist_ubyte(self._root)
        lab_path = _find(self._root, [lab_name + '.gz', lab_name])
        img_path = _find(self._root, [img_name + '.gz', img_name])
        with _open(lab_path) as fin:
            struct.unpack('>II', fin.read(8))
            label = np.frombuffer(fin.read(), dtype=np.uint8).astype(np.int32)
        with _open(img_path) as fin:
            struct.unpack('>IIII', fin.read(16))
            data = np.frombuffer(fin.read(), dtype=np.uint8).reshape(len(label), 28, 28, 1)
        self._data = nd.array(data, dtype=data.dtype)
        self._label = label


class FashionMNIST(MNIST):
    def __init__(self, root=os.path.join(_data_dir(), 'datasets', 'fashion-mnist'), train=True, transform=None):
        super().__init__(root, train, transform)


class CIFAR10(_DownloadedDataset):
    """CIFAR-10 binary version: (32, 32, 3) uint8 images."""

    def __init__(self, root=os.path.join(_data_dir(), 'datasets', 'cifar10'), train=True, transform=None):
        self._train = train
        super().__init__(root, transform)

    def _read_batch(self, filename):
        with open(filename, 'rb') as fin:
            data = np.frombuffer(fin.read(), dtype=np.uint8).reshape(-1, 3072 + 1)
        return data[:, 1:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1), data[:, 0].astype(np.int32)

    def _files(self):
        sub = 'cifar-10-batches-bin'
        base = os.path.join(self._root, sub) if os.path.isdir(os.path.join(self._root, sub)) else self._root
        if self._train:
            return [_find(base, ['data_batch_%d.bin' % i]) for i in range(1, 6)]
        return [_find(base, ['test_batch.bin'])]

    def _get_data(self):
        data, label = zip(*(self._read_batch(f) for f in self._files()))
        data = np.concatenate(data)
        self._data = nd.array(data, dtype=data.dtype)
        self._label = np.concatenate(label)


class CIFAR100(CIFAR10):
    """CIFAR-100 binary version; ``fine_label`` selects the 100-class labels."""

    def __init__(self, root=os.path.join(_data_dir(), 'datasets', 'cifar100'), fine_label=False, train=True,
                 transform=None):
        self._fine_label = fine_label
        super().__init__(root, train, transform)

    def _read_batch(self, filename):
        with open(filename, 'rb') as fin:
            data = np.frombuffer(fin.read(), dtype=np.uint8).reshape(-1, 3072 + 2)
        return data[:, 2:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1), \
            data[:, 0 + self._fine_label].astype(np.int32)

    def _files(self):
        sub = 'cifar-100-binary'
        base = os.path.join(self._root, sub) if os.path.isdir(os.path.join(self._root, sub)) else self._root
        return [_find(base, ['train.bin' if self._train else 'test.bin'])]


class ImageRecordDataset(RecordFileDataset):
    """Images + labels stored in a RecordIO file (``im2rec`` output)."""

    def __init__(self, filename, flag=1, transform=None):
        super().__init__(filename)
        self._flag = flag
        self._transform = transform

    def __getitem__(self, idx):
        record = super().__getitem__(idx)
        header, img = recordio.unpack(record)
        if self._transform is not None:
            return self._transform(image.imdecode(img, self._flag), header.label)
        return image.imdecode(img, self._flag), header.label


class ImageFolderDataset(Dataset):
    """``root/<class>/<image>`` folder layout; labels are sorted class indices."""

    def __init__(self, root, flag=1, transform=None):
        self._root = os.path.expanduser(root)
        self._flag = flag
        self._transform = transform
        self._exts = ['.jpg', '.jpeg', '.png']
        self._list_images(self._root)

    def _list_images(self, root):
        self.synsets = []
        self.items = []
        for folder in sorted(os.listdir(root)):
            path = os.path.join(root, folder)
            if not os.path.isdir(path):
                warnings.warn('Ignoring %s, which is not a directory.' % path, stacklevel=3)
                continue
            label = len(self.synsets)
            self.synsets.append(folder)
            for filename in sorted(os.listdir(path)):
                filename = os.path.join(path, filename)
                ext = os.path.splitext(filename)[1]
                if ext.lower() not in self._exts:
                    warnings.warn('Ignoring %s of type %s. Only support %s' % (filename, ext, ', '.join(self._exts)))
                    continue
                self.items.append((filename, label))

    def __getitem__(self, idx):
        img = image.imread(self.items[idx][0], self._flag)
        label = self.items[idx][1]
        if self._transform is not None:
            return self._transform(img, label)
        return img, label

    def __len__(self):
        return len(self.items)


class ImageListDataset(Dataset):
    """Images listed in a ``.lst`` file (``idx\\tlabel...\\tpath``) or a python list of ``[label, path]``."""

    def __init__(self, root='.', imglist=None, flag=1):
        self._root = root
        self._flag = flag
        self.items = []
        if isinstance(imglist, str):
            with open(imglist) as fin:
                for line in fin:
                    parts = line.strip().split('\t')
                    if len(parts) < 3:
                        continue
                    label = np.array([float(x) for x in parts[1:-1]], dtype=np.float32)
                    self.items.append((parts[-1], label[0] if label.size == 1 else label))
        elif imglist is not None:
            for item in imglist:
                label, path = item[:-1], item[-1]
                label = np.array(label, dtype=np.float32).reshape(-1)
                self.items.append((path, label[0] if label.size == 1 else label))

    def __getitem__(self, idx):
        path, label = self.items[idx]
        return image.imread(os.path.join(self._root, path), self._flag), label

    def __len__(self):
        return len(self.items)
