"""Detection augmenters and ImageDetIter.

Parity: python/mxnet/image/detection.py (DetAugmenter, DetBorrowAug,
DetRandomSelectAug, DetHorizontalFlipAug, DetRandomCropAug, DetRandomPadAug,
CreateMultiRandCropAugmenter, CreateDetAugmenter, ImageDetIter).  Labels are
(num_objects, 5+) arrays ``[cls, xmin, ymin, xmax, ymax, ...]`` with
coordinates normalised to [0, 1]; raw record labels carry the
``[header_width, obj_width, ...header..., objects...]`` prefix.
"""
import json
import logging
import random

import numpy as np

from .. import ndarray as nd
from ..ndarray.ndarray import NDArray
from .. import io as mxio
from .image import (Augmenter, ImageIter, ResizeAug, ForceResizeAug, CastAug, ColorJitterAug, HueJitterAug,
                    LightingAug, RandomGrayAug, ColorNormalizeAug, fixed_crop, copyMakeBorder)

__all__ = ['DetAugmenter', 'DetBorrowAug', 'DetRandomSelectAug', 'DetHorizontalFlipAug', 'DetRandomCropAug',
           'DetRandomPadAug', 'CreateMultiRandCropAugmenter', 'CreateDetAugmenter', 'ImageDetIter']


class DetAugmenter:
    """Base class: ``__call__(src, label) -> (src, label)``."""

    def __init__(self, **kwargs):
        self._kwargs = {}
        for k, v in kwargs.items():
            if isinstance(v, NDArray):
                v = v.asnumpy()
            if isinstance(v, np.ndarray):
                v = v.tolist()
            self._kwargs[k] = v

    def dumps(self):
        return json.dumps([self.__class__.__name__.lower(), self._kwargs])

    def __call__(self, src, label):
        raise NotImplementedError('Must override implementation.')


class DetBorrowAug(DetAugmenter):
    """Apply a classification augmenter that does not move pixels (label untouched)."""

    def __init__(self, augmenter):
        if not isinstance(augmenter, Augmenter):
            raise TypeError('Borrowing from invalid Augmenter')
        super().__init__(augmenter=augmenter.dumps())
        self.augmenter = augmenter

    def dumps(self):
        return [self.__class__.__name__.lower(), self.augmenter.dumps()]

    def __call__(self, src, label):
        return self.augmenter(src), label


class DetRandomSelectAug(DetAugmenter):
    """Apply one randomly chosen augmenter of ``aug_list`` (or none with prob ``skip_prob``)."""

    def __init__(self, aug_list, skip_prob=0):
        super().__init__(skip_prob=skip_prob)
        if not isinstance(aug_list, (list, tuple)):
            aug_list = [aug_list]
        for aug in aug_list:
            if not isinstance(aug, DetAugmenter):
                raise ValueError('Allow DetAugmenter in list only')
        self.aug_list = list(aug_list)
        self.skip_prob = 1 if not aug_list else skip_prob

    def dumps(self):
        return [self.__class__.__name__.lower(), [x.dumps() for x in self.aug_list]]

    def __call__(self, src, label):
        if random.random() < self.skip_prob:
            return src, label
        return random.choice(self.aug_list)(src, label)


class DetHorizontalFlipAug(DetAugmenter):
    def __init__(self, p):
        super().__init__(p=p)
        self.p = p

    def __call__(self, src, label):
        if random.random() < self.p:
            src = nd.flip(src, axis=1)
            xmin = 1.0 - label[:, 3]
            label[:, 3] = 1.0 - label[:, 1]
            label[:, 1] = xmin
        return src, label


def _box_areas(b):
    return np.clip(b[:, 2] - b[:, 0], 0, None) * np.clip(b[:, 3] - b[:, 1], 0, None)


def _intersect(boxes, x0, y0, x1, y1):
    ix0 = np.maximum(boxes[:, 0], x0)
    iy0 = np.maximum(boxes[:, 1], y0)
    ix1 = np.minimum(boxes[:, 2], x1)
    iy1 = np.minimum(boxes[:, 3], y1)
    return np.stack([ix0, iy0, ix1, iy1], 1)


class DetRandomCropAug(DetAugmenter):
    """Random crop whose window covers >= ``min_object_covered`` of at least one object.

    Objects whose remaining visible fraction falls below ``min_eject_coverage``
    are dropped; the rest are clipped and re-normalised to the crop.
    """

    def __init__(self, min_object_covered=0.1, aspect_ratio_range=(0.75, 1.33), area_range=(0.05, 1.0),
                 min_eject_coverage=0.3, max_attempts=50):
        if not isinstance(aspect_ratio_range, (tuple, list)):
            aspect_ratio_range = (1 - aspect_ratio_range, 1 + aspect_ratio_range)
        if not isinstance(area_range, (tuple, list)):
            area_range = (1 - area_range, 1 + area_range)
        super().__init__(min_object_covered=min_object_covered, aspect_ratio_range=aspect_ratio_range,
                         area_range=area_range, min_eject_coverage=min_eject_coverage, max_attempts=max_attempts)
        self.min_object_covered = min_object_covered
        self.min_eject_coverage = min_eject_coverage
        self.max_attempts = max_attempts
        self.aspect_ratio_range = aspect_ratio_range
        self.area_range = area_range
        self.enabled = (area_range[1] > 0 and area_range[0] <= area_range[1] and aspect_ratio_range[0] > 0 and
                        aspect_ratio_range[0] <= aspect_ratio_range[1])
        if area_range[1] <= 0 or area_range[0] > area_range[1]:
            logging.warning('Skip DetRandomCropAug due to invalid area_range: %s', area_range)
        if aspect_ratio_range[0] <= 0 or aspect_ratio_range[0] > aspect_ratio_range[1]:
            logging.warning('Skip DetRandomCropAug due to invalid aspect_ratio_range: %s', aspect_ratio_range)

    def __call__(self, src, label):
        h, w = src.shape[0], src.shape[1]
        crop = self._propose(label, h, w)
        if crop:
            x, y, cw, ch, label = crop
            src = fixed_crop(src, x, y, cw, ch, None)
        return src, label

    def _satisfied(self, label, x0, y0, x1, y1):
        boxes = label[:, 1:5]
        areas = _box_areas(boxes)
        inter = _box_areas(_intersect(boxes, x0, y0, x1, y1))
        cov = inter / np.maximum(areas, 1e-12)
        return bool((cov[areas > 0] >= self.min_object_covered).any())

    def _update(self, label, box):
        x0, y0, x1, y1 = box
        out = label.copy()
        b = _intersect(out[:, 1:5], x0, y0, x1, y1)
        areas = _box_areas(out[:, 1:5])
        cov = _box_areas(b) / np.maximum(areas, 1e-12)
        keep = cov >= self.min_eject_coverage
        cw, ch = x1 - x0, y1 - y0
        b[:, (0, 2)] = (b[:, (0, 2)] - x0) / cw
        b[:, (1, 3)] = (b[:, (1, 3)] - y0) / ch
        out[:, 1:5] = np.clip(b, 0, 1)
        out = out[keep]
        return out if out.shape[0] else None

    def _propose(self, label, height, width):
        if not self.enabled or height <= 0 or width <= 0:
            return ()
        min_area = self.area_range[0] * height * width
        max_area = self.area_range[1] * height * width
        for _ in range(self.max_attempts):
            ratio = random.uniform(*self.aspect_ratio_range)
            if ratio <= 0:
                continue
            h = int(round(np.sqrt(min_area / ratio)))
            max_h = int(round(np.sqrt(max_area / ratio)))
            if round(max_h * ratio) > width:
                max_h = int((width + 0.4999999) / ratio)
            max_h = min(max_h, height)
            h = min(h, max_h)
            if h < max_h:
                h = random.randint(h, max_h)
            w = int(round(h * ratio))
            if w <= 0 or h <= 0 or w * h < min_area or w * h > max_area or w > width or h > height:
                continue
            y = random.randint(0, max(0, height - h))
            x = random.randint(0, max(0, width - w))
            box = (x / width, y / height, (x + w) / width, (y + h) / height)
            if self._satisfied(label, *box):
                new_label = self._update(label, box)
                if new_label is not None:
                    return x, y, w, h, new_label
        return ()


class DetRandomPadAug(DetAugmenter):
    """Random expansion: place the image inside a larger ``pad_val`` canvas."""

    def __init__(self, aspect_ratio_range=(0.75, 1.33), area_range=(1.0, 3.0), max_attempts=50,
                 pad_val=(128, 128, 128)):
        if not isinstance(pad_val, (list, tuple)):
            pad_val = (pad_val,)
        if not isinstance(aspect_ratio_range, (list, tuple)):
            aspect_ratio_range = (1 - aspect_ratio_range, 1 + aspect_ratio_range)
        if not isinstance(area_range, (list, tuple)):
            area_range = (1 - area_range, 1 + area_range)
        super().__init__(aspect_ratio_range=aspect_ratio_range, area_range=area_range, max_attempts=max_attempts,
                         pad_val=pad_val)
        self.pad_val = pad_val
        self.aspect_ratio_range = aspect_ratio_range
        self.area_range = area_range
        self.max_attempts = max_attempts
        self.enabled = area_range[1] > 1.0 and area_range[0] <= area_range[1] and aspect_ratio_range[0] > 0

    def __call__(self, src, label):
        height, width = src.shape[0], src.shape[1]
        pad = self._propose(label, height, width)
        if pad:
            x, y, w, h, label = pad
            src = copyMakeBorder(src, y, h - y - height, x, w - x - width, 0, values=self.pad_val)
        return src, label

    def _propose(self, label, height, width):
        if not self.enabled or height <= 0 or width <= 0:
            return ()
        min_area = self.area_range[0] * height * width
        max_area = self.area_range[1] * height * width
        for _ in range(self.max_attempts):
            ratio = random.uniform(*self.aspect_ratio_range)
            if ratio <= 0:
                continue
            h = int(round(np.sqrt(min_area / ratio)))
            max_h = int(round(np.sqrt(max_area / ratio)))
            if round(h * ratio) < width:
                h = int((width + 0.499999) / ratio)
            h = max(h, height)
            if h < max_h:
                h = random.randint(h, max_h)
            w = int(round(h * ratio))
            if (h - height) < 2 or (w - width) < 2:
                continue
            y = random.randint(0, max(0, h - height))
            x = random.randint(0, max(0, w - width))
            out = label.copy()
            out[:, (1, 3)] = (out[:, (1, 3)] * width + x) / w
            out[:, (2, 4)] = (out[:, (2, 4)] * height + y) / h
            return x, y, w, h, out
        return ()


def CreateMultiRandCropAugmenter(min_object_covered=0.1, aspect_ratio_range=(0.75, 1.33), area_range=(0.05, 1.0),
                                 min_eject_coverage=0.3, max_attempts=50, skip_prob=0):
    """Several DetRandomCropAug with (broadcast) parameter lists, one chosen at random per image."""
    def align(params):
        lens = [len(p) for p in params if isinstance(p, list)]
        n = max(lens) if lens else 1
        out = []
        for p in params:
            if not isinstance(p, list):
                p = [p] * n
            assert len(p) == n, 'Number of parameters mismatch'
            out.append(p)
        return out
    aligned = align([min_object_covered, aspect_ratio_range, area_range, min_eject_coverage, max_attempts])
    augs = [DetRandomCropAug(min_object_covered=moc, aspect_ratio_range=arr, area_range=ar,
                             min_eject_coverage=mec, max_attempts=ma) for moc, arr, ar, mec, ma in zip(*aligned)]
    return DetRandomSelectAug(augs, skip_prob=skip_prob)


def CreateDetAugmenter(data_shape, resize=0, rand_crop=0, rand_pad=0, rand_gray=0, rand_mirror=False, mean=None,
                       std=None, brightness=0, contrast=0, saturation=0, pca_noise=0, hue=0, inter_method=2,
                       min_object_covered=0.1, aspect_ratio_range=(0.75, 1.33), area_range=(0.05, 3.0),
                       min_eject_coverage=0.3, max_attempts=50, pad_val=(127, 127, 127)):
    """Standard detection augmenter pipeline."""
    auglist = []
    if resize > 0:
        auglist.append(DetBorrowAug(ResizeAug(resize, inter_method)))
    if rand_crop > 0:
        crop_augs = CreateMultiRandCropAugmenter(min_object_covered, aspect_ratio_range,
                                                 (area_range[0], min(1.0, area_range[1])), min_eject_coverage,
                                                 max_attempts, skip_prob=(1 - rand_crop))
        auglist.append(crop_augs)
    if rand_mirror > 0:
        auglist.append(DetHorizontalFlipAug(0.5))
    if rand_pad > 0:
        pad_aug = DetRandomPadAug(aspect_ratio_range, (1.0, area_range[1]), max_attempts, pad_val)
        auglist.append(DetRandomSelectAug([pad_aug], 1 - rand_pad))
    auglist.append(DetBorrowAug(ForceResizeAug((data_shape[2], data_shape[1]), inter_method)))
    auglist.append(DetBorrowAug(CastAug()))
    if brightness or contrast or saturation:
        auglist.append(DetBorrowAug(ColorJitterAug(brightness, contrast, saturation)))
    if hue:
        auglist.append(DetBorrowAug(HueJitterAug(hue)))
    if pca_noise > 0:
        eigval = np.array([55.46, 4.794, 1.148])
        eigvec = np.array([[-0.5675, 0.7192, 0.4009], [-0.5808, -0.0045, -0.8140], [-0.5836, -0.6948, 0.4203]])
        auglist.append(DetBorrowAug(LightingAug(pca_noise, eigval, eigvec)))
    if rand_gray > 0:
        auglist.append(DetBorrowAug(RandomGrayAug(rand_gray)))
    if mean is True:
        mean = np.array([123.68, 116.28, 103.53])
    if std is True:
        std = np.array([58.395, 57.12, 57.375])
    if mean is not None or std is not None:
        auglist.append(DetBorrowAug(ColorNormalizeAug(mean, std)))
    return auglist


class ImageDetIter(ImageIter):
    """ImageIter for detection: labels become (batch, max_objects, obj_width) padded with -1."""

    def __init__(self, batch_size, data_shape, path_imgrec=None, path_imglist=None, path_root=None,
                 path_imgidx=None, shuffle=False, part_index=0, num_parts=1, aug_list=None, imglist=None,
                 data_name='data', label_name='label', last_batch_handle='pad', **kwargs):
        super().__init__(batch_size=batch_size, data_shape=data_shape, path_imgrec=path_imgrec,
                         path_imglist=path_imglist, path_root=path_root, path_imgidx=path_imgidx, shuffle=shuffle,
                         part_index=part_index, num_parts=num_parts, aug_list=[], imglist=imglist,
                         data_name=data_name, label_name=label_name, last_batch_handle=last_batch_handle)
        self.auglist = CreateDetAugmenter(data_shape, **kwargs) if aug_list is None else aug_list
        label_shape = self._estimate_label_shape()
        self.provide_label = [(label_name, (self.batch_size, label_shape[0], label_shape[1]))]
        self.label_shape = label_shape

    def _check_valid_label(self, label):
        if len(label.shape) != 2 or label.shape[1] < 5:
            raise RuntimeError('Label with shape (1+, 5+) required, %s received.' % str(label))
        valid = np.where(np.logical_and(label[:, 0] >= 0, np.logical_and(label[:, 3] > label[:, 1],
                                                                         label[:, 4] > label[:, 2])))[0]
        if valid.size < 1:
            raise RuntimeError('Invalid label occurs.')

    def _estimate_label_shape(self):
        max_count, width = 0, 5
        self.reset()
        try:
            while True:
                label, _ = self.next_sample()
                label = self._parse_label(label)
                max_count = max(max_count, label.shape[0])
                width = label.shape[1]
        except StopIteration:
            pass
        self.reset()
        return (max_count, width)

    def _parse_label(self, label):
        if isinstance(label, NDArray):
            label = label.asnumpy()
        raw = np.asarray(label, dtype=np.float32).ravel()
        if raw.size < 7:
            raise RuntimeError('Label shape is invalid: ' + str(raw.shape))
        header_width, obj_width = int(raw[0]), int(raw[1])
        if (raw.size - header_width) % obj_width != 0:
            raise RuntimeError('Label shape %s inconsistent with annotation width %d.' % (str(raw.shape), obj_width))
        out = np.reshape(raw[header_width:], (-1, obj_width))
        valid = np.where(np.logical_and(out[:, 3] > out[:, 1], out[:, 4] > out[:, 2]))[0]
        if valid.size < 1:
            raise RuntimeError('Encounter sample with no valid label.')
        return out[valid, :]

    def reshape(self, data_shape=None, label_shape=None):
        if data_shape is not None:
            self.check_data_shape(data_shape)
            self.provide_data = [(self.provide_data[0][0], (self.batch_size,) + tuple(data_shape))]
            self.data_shape = tuple(data_shape)
        if label_shape is not None:
            self.check_label_shape(label_shape)
            self.provide_label = [(self.provide_label[0][0], (self.batch_size,) + tuple(label_shape))]
            self.label_shape = tuple(label_shape)

    def check_label_shape(self, label_shape):
        if not len(label_shape) == 2:
            raise ValueError('label_shape should have length 2')
        if label_shape[0] < self.label_shape[0]:
            raise ValueError('Attempts to reduce label count from %d to %d, not allowed.'
                             % (self.label_shape[0], label_shape[0]))
        if label_shape[1] != self.provide_label[0][1][2]:
            raise ValueError('label_shape object width inconsistent: %d vs %d.'
                             % (self.provide_label[0][1][2], label_shape[1]))

    def _batchify(self, batch_data, batch_label, start=0):
        i = start
        try:
            while i < self.batch_size:
                label, s = self.next_sample()
                data = self.imdecode(s)
                try:
                    self.check_valid_image([data])
                    label = self._parse_label(label)
                    data, label = self.augmentation_transform(data, label)
                    self._check_valid_label(label)
                except RuntimeError as e:
                    logging.debug('Invalid image, skipping:  %s', str(e))
                    continue
                batch_data[i] = self.postprocess_data(data)
                lab = np.full(batch_label.shape[1:], -1.0, dtype=np.float32)
                n = min(label.shape[0], lab.shape[0])
                lab[:n] = label[:n]
                batch_label[i] = nd.array(lab)
                i += 1
        except StopIteration:
            if not i:
                raise StopIteration
        return i

    def next(self):
        c, h, w = self.data_shape
        if self._cache_data is not None:
            batch_data, batch_label, i = self._cache_data, self._cache_label, self._cache_idx
        else:
            batch_data = nd.zeros((self.batch_size, c, h, w))
            batch_label = nd.full(self.provide_label[0][1], -1.0)
            i = self._batchify(batch_data, batch_label)
        pad = self.batch_size - i
        if pad != 0:
            if self.last_batch_handle == 'discard':
                raise StopIteration
            if self.last_batch_handle == 'roll_over' and self._cache_data is None:
                self._cache_data, self._cache_label, self._cache_idx = batch_data, batch_label, i
                raise StopIteration
            self._batchify(batch_data, batch_label, i)
            if self.last_batch_handle == 'pad':
                self._allow_read = False
            else:
                self._cache_data = self._cache_label = self._cache_idx = None
        return mxio.DataBatch([batch_data], [batch_label], pad=pad)

    def augmentation_transform(self, data, label):  # pylint: disable=arguments-differ
        for aug in self.auglist:
            data, label = aug(data, label)
        return data, label

    def sync_label_shape(self, it, verbose=False):
        assert isinstance(it, ImageDetIter), 'Synchronize with invalid iterator.'
        train_label_shape = self.label_shape
        val_label_shape = it.label_shape
        assert train_label_shape[1] == val_label_shape[1], 'object width mismatch.'
        max_count = max(train_label_shape[0], val_label_shape[0])
        if max_count > train_label_shape[0]:
            self.reshape(None, (max_count, train_label_shape[1]))
        if max_count > val_label_shape[0]:
            it.reshape(None, (max_count, val_label_shape[1]))
        if verbose and max_count > min(train_label_shape[0], val_label_shape[0]):
            logging.info('Resized label_shape to (%d, %d).', max_count, train_label_shape[1])
        return it
