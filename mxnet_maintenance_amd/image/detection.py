"""Detection augmenters and ``ImageDetIter`` (mx.image).

Behavioural parity with python/mxnet/image/detection.py (DetAugmenter :40, DetBorrowAug :60,
DetRandomSelectAug :90, DetHorizontalFlipAug :130, DetRandomCropAug :150 with its constraint
check :236 / label update :253 / proposal :275, DetRandomPadAug :324, CreateMultiRandCropAugmenter
:420, CreateDetAugmenter :480, ImageDetIter :640).

A detection label is a float32 ``(num_objects, width >= 5)`` array of rows
``[class, xmin, ymin, xmax, ymax, extra...]`` with coordinates normalised to [0, 1].  A raw record
label is flat: ``[header_width, object_width, header..., objects...]``.  Every augmenter maps
``(image, label) -> (image, label)``; the batch assembly (``last_batch_handle``, roll-over carry)
is ``ImageIter``'s, with labels padded to a fixed object count by -1 rows.
"""
import logging
import math
import random as _rand

import numpy as np

from .. import ndarray as nd
from ..ndarray.ndarray import NDArray
from .image import (Augmenter, ImageIter, ResizeAug, ForceResizeAug, CastAug, ColorJitterAug, HueJitterAug,
                    LightingAug, RandomGrayAug, ColorNormalizeAug, fixed_crop, copyMakeBorder,
                    _PCA_EIGVAL, _PCA_EIGVEC, _IMAGENET_MEAN, _IMAGENET_STD)

__all__ = ['DetAugmenter', 'DetBorrowAug', 'DetRandomSelectAug', 'DetHorizontalFlipAug', 'DetRandomCropAug',
           'DetRandomPadAug', 'CreateMultiRandCropAugmenter', 'CreateDetAugmenter', 'ImageDetIter']


class DetAugmenter:
    """Callable ``(src, label) -> (src, label)``; keyword parameters are recorded for ``dumps``."""

    __init__ = Augmenter.__init__
    dumps = Augmenter.dumps

    def __call__(self, src, label):
        raise NotImplementedError('Must override implementation.')


class DetBorrowAug(DetAugmenter):
    """Run a classification ``Augmenter`` that keeps geometry (the label passes through)."""

    def __init__(self, augmenter):
        if not isinstance(augmenter, Augmenter):
            raise TypeError('Borrowing from invalid Augmenter')
        super().__init__(augmenter=augmenter.dumps())
        self.augmenter = augmenter

    def dumps(self):
        return [type(self).__name__.lower(), self.augmenter.dumps()]

    def __call__(self, src, label):
        return self.augmenter(src), label


class DetRandomSelectAug(DetAugmenter):
    """Apply one augmenter drawn from ``aug_list``, or none with probability ``skip_prob``."""

    def __init__(self, aug_list, skip_prob=0):
        choices = list(aug_list) if isinstance(aug_list, (list, tuple)) else [aug_list]
        if any(not isinstance(a, DetAugmenter) for a in choices):
            raise ValueError('Allow DetAugmenter in list only')
        super().__init__(skip_prob=skip_prob)
        self.aug_list = choices
        self.skip_prob = skip_prob if choices else 1

    def dumps(self):
        return [type(self).__name__.lower(), [a.dumps() for a in self.aug_list]]

    def __call__(self, src, label):
        if _rand.random() < self.skip_prob:
            return src, label
        return _rand.choice(self.aug_list)(src, label)


class DetHorizontalFlipAug(DetAugmenter):
    """Mirror image and boxes left-right with probability ``p``."""

    def __init__(self, p):
        super().__init__(p=p)

    def __call__(self, src, label):
        if _rand.random() < self.p:
            src = nd.flip(src, axis=1)
            label[:, (1, 3)] = 1.0 - label[:, (3, 1)]
        return src, label


# ---------------------------------------------------------------------------- box arithmetic
# ``boxes`` below are (n, 4) arrays [xmin, ymin, xmax, ymax] in normalised coordinates.
def _areas(boxes):
    return np.maximum(0, boxes[:, 2] - boxes[:, 0]) * np.maximum(0, boxes[:, 3] - boxes[:, 1])


def _clip_to(boxes, window):
    """Intersection of every box with ``window``; empty intersections become all-zero rows."""
    lo = np.maximum(boxes[:, :2], window[:2])
    hi = np.minimum(boxes[:, 2:4], window[2:])
    inter = np.concatenate([lo, hi], axis=1)
    inter[(lo >= hi).any(axis=1)] = 0
    return inter


def _as_range(val):
    """A scalar ``r`` means the fixed range (r, r)."""
    return tuple(val) if isinstance(val, (list, tuple)) else (val, val)


def _draw_height(lo, hi):
    """Uniform integer in [lo, hi]; ``hi`` when the range is empty (clamped like the reference)."""
    return _rand.randint(lo, hi) if lo < hi else hi


class DetRandomCropAug(DetAugmenter):
    """Random crop (SSD-style) constrained by object coverage.

    A window of area fraction in ``area_range`` and aspect ``w / h`` in ``aspect_ratio_range`` is
    accepted when every object it touches keeps more than ``min_object_covered`` of its area;
    objects keeping at most ``min_eject_coverage`` are then dropped and the rest re-normalised.
    """

    def __init__(self, min_object_covered=0.1, aspect_ratio_range=(0.75, 1.33), area_range=(0.05, 1.0),
                 min_eject_coverage=0.3, max_attempts=50):
        aspect_ratio_range, area_range = _as_range(aspect_ratio_range), _as_range(area_range)
        super().__init__(min_object_covered=min_object_covered, aspect_ratio_range=aspect_ratio_range,
                         area_range=area_range, min_eject_coverage=min_eject_coverage, max_attempts=max_attempts)
        area_ok = 0 < area_range[1] and area_range[0] <= area_range[1]
        ratio_ok = 0 < aspect_ratio_range[0] <= aspect_ratio_range[1]
        if not area_ok:
            logging.warning('Skip DetRandomCropAug due to invalid area_range: %s', area_range)
        if not ratio_ok:
            logging.warning('Skip DetRandomCropAug due to invalid aspect_ratio_range: %s', aspect_ratio_range)
        self.enabled = area_ok and ratio_ok

    def __call__(self, src, label):
        proposal = self._random_crop_proposal(label, src.shape[0], src.shape[1])
        if proposal:
            x, y, w, h, label = proposal
            src = fixed_crop(src, x, y, w, h, None)
        return src, label

    def _check_satisfy_constraints(self, label, xmin, ymin, xmax, ymax, width, height):
        if (xmax - xmin) * (ymax - ymin) < 2:
            return False                        # a one-pixel window
        window = np.array([xmin / width, ymin / height, xmax / width, ymax / height], dtype=np.float64)
        areas = _areas(label[:, 1:5])
        big = areas * width * height > 2
        if not big.any():
            return False
        kept = _areas(_clip_to(label[big, 1:5], window)) / areas[big]
        touched = kept[kept > 0]
        return touched.size > 0 and touched.min() > self.min_object_covered

    def _update_labels(self, label, crop_box, height, width):
        x, y, w, h = crop_box
        fx, fy = w / width, h / height
        out = label.copy()
        out[:, (1, 3)] = (out[:, (1, 3)] - x / width) / fx
        out[:, (2, 4)] = (out[:, (2, 4)] - y / height) / fy
        out[:, 1:5] = np.clip(out[:, 1:5], 0, 1)
        kept = _areas(out[:, 1:5]) * fx * fy / _areas(label[:, 1:5])
        ok = (out[:, 3] > out[:, 1]) & (out[:, 4] > out[:, 2]) & (kept > self.min_eject_coverage)
        return out[ok] if ok.any() else None

    def _random_crop_proposal(self, label, height, width):
        if not self.enabled or height <= 0 or width <= 0:
            return ()
        area_lo, area_hi = (f * height * width for f in self.area_range)
        for _ in range(self.max_attempts):
            ratio = _rand.uniform(*self.aspect_ratio_range)
            if ratio <= 0:
                continue
            h_hi = int(round(math.sqrt(area_hi / ratio)))
            if round(h_hi * ratio) > width:
                h_hi = int((width + 0.4999999) / ratio)     # largest h whose width still fits
            h_hi = min(h_hi, height)
            h = _draw_height(min(int(round(math.sqrt(area_lo / ratio))), h_hi), h_hi)
            w = int(round(h * ratio))
            # nudge by one row when rounding pushed the area out of range
            if w * h < area_lo:
                h += 1
                w = int(round(h * ratio))
            if w * h > area_hi:
                h -= 1
                w = int(round(h * ratio))
            if not (area_lo <= w * h <= area_hi and 0 <= w <= width and 0 <= h <= height):
                continue
            y = _rand.randint(0, max(0, height - h))
            x = _rand.randint(0, max(0, width - w))
            if self._check_satisfy_constraints(label, x, y, x + w, y + h, width, height):
                moved = self._update_labels(label, (x, y, w, h), height, width)
                if moved is not None:
                    return x, y, w, h, moved
        return ()


class DetRandomPadAug(DetAugmenter):
    """Random expansion: paste the image into a larger ``pad_val`` canvas (area factor in
    ``area_range``, canvas aspect in ``aspect_ratio_range``) and shift the boxes accordingly."""

    def __init__(self, aspect_ratio_range=(0.75, 1.33), area_range=(1.0, 3.0), max_attempts=50,
                 pad_val=(128, 128, 128)):
        pad_val = tuple(pad_val) if isinstance(pad_val, (list, tuple)) else (pad_val,)
        aspect_ratio_range, area_range = _as_range(aspect_ratio_range), _as_range(area_range)
        super().__init__(aspect_ratio_range=aspect_ratio_range, area_range=area_range, max_attempts=max_attempts,
                         pad_val=pad_val)
        area_ok = area_range[1] > 1.0 and area_range[0] <= area_range[1]
        ratio_ok = 0 < aspect_ratio_range[0] <= aspect_ratio_range[1]
        if not area_ok:
            logging.warning('Skip DetRandomPadAug due to invalid parameters: %s', area_range)
        if not ratio_ok:
            logging.warning('Skip DetRandomPadAug due to invalid aspect_ratio_range: %s', aspect_ratio_range)
        self.enabled = area_ok and ratio_ok

    def __call__(self, src, label):
        height, width = src.shape[0], src.shape[1]
        proposal = self._random_pad_proposal(label, height, width)
        if proposal:
            x, y, w, h, label = proposal
            src = copyMakeBorder(src, y, h - y - height, x, w - x - width, 0, values=self.pad_val)
        return src, label

    def _update_labels(self, label, pad_box, height, width):
        x, y, w, h = pad_box
        out = label.copy()
        out[:, (1, 3)] = (out[:, (1, 3)] * width + x) / w
        out[:, (2, 4)] = (out[:, (2, 4)] * height + y) / h
        return out

    def _random_pad_proposal(self, label, height, width):
        if not self.enabled or height <= 0 or width <= 0:
            return ()
        area_lo, area_hi = (f * height * width for f in self.area_range)
        for _ in range(self.max_attempts):
            ratio = _rand.uniform(*self.aspect_ratio_range)
            if ratio <= 0:
                continue
            h = int(round(math.sqrt(area_lo / ratio)))
            if round(h * ratio) < width:
                h = int((width + 0.499999) / ratio)          # canvas at least as wide as the image
            h = _draw_height(max(h, height), int(round(math.sqrt(area_hi / ratio))))
            w = int(round(h * ratio))
            if h - height < 2 or w - width < 2:
                continue                                       # not a real expansion
            y = _rand.randint(0, max(0, h - height))
            x = _rand.randint(0, max(0, w - width))
            return x, y, w, h, self._update_labels(label, (x, y, w, h), height, width)
        return ()


def CreateMultiRandCropAugmenter(min_object_covered=0.1, aspect_ratio_range=(0.75, 1.33), area_range=(0.05, 1.0),
                                 min_eject_coverage=0.3, max_attempts=50, skip_prob=0):
    """One ``DetRandomCropAug`` per entry of the (list-valued, broadcast) parameters, picked at random."""
    params = [min_object_covered, aspect_ratio_range, area_range, min_eject_coverage, max_attempts]
    count = max([len(p) for p in params if isinstance(p, list)] or [1])
    columns = []
    for p in params:
        col = p if isinstance(p, list) else [p] * count
        assert len(col) == count, 'Number of parameters mismatch'
        columns.append(col)
    crops = [DetRandomCropAug(min_object_covered=moc, aspect_ratio_range=arr, area_range=ar,
                              min_eject_coverage=mec, max_attempts=ma) for moc, arr, ar, mec, ma in zip(*columns)]
    return DetRandomSelectAug(crops, skip_prob=skip_prob)


def CreateDetAugmenter(data_shape, resize=0, rand_crop=0, rand_pad=0, rand_gray=0, rand_mirror=False, mean=None,
                       std=None, brightness=0, contrast=0, saturation=0, pca_noise=0, hue=0, inter_method=2,
                       min_object_covered=0.1, aspect_ratio_range=(0.75, 1.33), area_range=(0.05, 3.0),
                       min_eject_coverage=0.3, max_attempts=50, pad_val=(127, 127, 127)):
    """The standard detection pipeline: resize, random crop / mirror / pad, force-resize to
    ``data_shape``, cast, colour jitter, lighting, grey, normalise."""
    borrow = DetBorrowAug
    mean = np.array(_IMAGENET_MEAN) if mean is True else mean
    std = np.array(_IMAGENET_STD) if std is True else std
    stages = [
        (resize > 0, lambda: borrow(ResizeAug(resize, inter_method))),
        (rand_crop > 0, lambda: CreateMultiRandCropAugmenter(
            min_object_covered, aspect_ratio_range, (area_range[0], min(1.0, area_range[1])),
            min_eject_coverage, max_attempts, skip_prob=(1 - rand_crop))),
        (rand_mirror > 0, lambda: DetHorizontalFlipAug(0.5)),
        (rand_pad > 0, lambda: DetRandomSelectAug(
            [DetRandomPadAug(aspect_ratio_range, (1.0, area_range[1]), max_attempts, pad_val)], 1 - rand_pad)),
        (True, lambda: borrow(ForceResizeAug((data_shape[2], data_shape[1]), inter_method))),
        (True, lambda: borrow(CastAug())),
        (brightness or contrast or saturation, lambda: borrow(ColorJitterAug(brightness, contrast, saturation))),
        (hue, lambda: borrow(HueJitterAug(hue))),
        (pca_noise > 0, lambda: borrow(LightingAug(pca_noise, _PCA_EIGVAL, _PCA_EIGVEC))),
        (rand_gray > 0, lambda: borrow(RandomGrayAug(rand_gray))),
        (mean is not None or std is not None, lambda: borrow(ColorNormalizeAug(mean, std))),
    ]
    return [make() for wanted, make in stages if wanted]


class ImageDetIter(ImageIter):
    """``ImageIter`` for detection: labels are ``(batch, max_objects, object_width)``, -1 padded.

    ``max_objects`` is estimated by one pass over the labels at construction; ``reshape`` /
    ``sync_label_shape`` grow it (e.g. to share one shape between train and validation iterators).
    """

    def __init__(self, batch_size, data_shape, path_imgrec=None, path_imglist=None, path_root=None,
                 path_imgidx=None, shuffle=False, part_index=0, num_parts=1, aug_list=None, imglist=None,
                 data_name='data', label_name='label', last_batch_handle='pad', **kwargs):
        super().__init__(batch_size=batch_size, data_shape=data_shape, path_imgrec=path_imgrec,
                         path_imglist=path_imglist, path_root=path_root, path_imgidx=path_imgidx, shuffle=shuffle,
                         part_index=part_index, num_parts=num_parts, aug_list=[], imglist=imglist,
                         data_name=data_name, label_name=label_name, last_batch_handle=last_batch_handle)
        self.auglist = CreateDetAugmenter(data_shape, **kwargs) if aug_list is None else aug_list
        self.label_shape = self._estimate_label_shape()
        self.provide_label = [(label_name, (self.batch_size,) + self.label_shape)]

    # ---------------------------------------------------------------- labels
    def _parse_label(self, label):
        """Flat record label -> (num_valid_objects, object_width) float32 array."""
        flat = np.asarray(label.asnumpy() if isinstance(label, NDArray) else label, dtype=np.float32).ravel()
        if flat.size < 7:
            raise RuntimeError('Label shape is invalid: ' + str(flat.shape))
        header, width = int(flat[0]), int(flat[1])
        if (flat.size - header) % width:
            raise RuntimeError('Label shape %s inconsistent with annotation width %d.' % (str(flat.shape), width))
        objs = flat[header:].reshape(-1, width)
        ok = (objs[:, 3] > objs[:, 1]) & (objs[:, 4] > objs[:, 2])
        if not ok.any():
            raise RuntimeError('Encounter sample with no valid label.')
        return objs[ok]

    def _check_valid_label(self, label):
        if label.ndim != 2 or label.shape[1] < 5:
            raise RuntimeError('Label with shape (1+, 5+) required, %s received.' % str(label))
        ok = (label[:, 0] >= 0) & (label[:, 3] > label[:, 1]) & (label[:, 4] > label[:, 2])
        if not ok.any():
            raise RuntimeError('Invalid label occurs.')

    def _estimate_label_shape(self):
        most, width = 0, 5
        self.reset()
        try:
            while True:
                objs = self._parse_label(self.next_sample()[0])
                most, width = max(most, objs.shape[0]), objs.shape[1]
        except StopIteration:
            pass
        self.reset()
        return (most, width)

    def reshape(self, data_shape=None, label_shape=None):
        """Change the batch data shape and / or grow the label shape."""
        if data_shape is not None:
            self.check_data_shape(data_shape)
            self.data_shape = tuple(data_shape)
            self.provide_data = [(self.provide_data[0][0], (self.batch_size,) + self.data_shape)]
        if label_shape is not None:
            self.check_label_shape(label_shape)
            self.label_shape = tuple(label_shape)
            self.provide_label = [(self.provide_label[0][0], (self.batch_size,) + self.label_shape)]

    def check_label_shape(self, label_shape):
        if len(label_shape) != 2:
            raise ValueError('label_shape should have length 2')
        if label_shape[0] < self.label_shape[0]:
            raise ValueError('Attempts to reduce label count from %d to %d, not allowed.'
                             % (self.label_shape[0], label_shape[0]))
        if label_shape[1] != self.provide_label[0][1][2]:
            raise ValueError('label_shape object width inconsistent: %d vs %d.'
                             % (self.provide_label[0][1][2], label_shape[1]))

    def sync_label_shape(self, it, verbose=False):
        """Give ``self`` and ``it`` the same (larger) max-object count; returns ``it``."""
        assert isinstance(it, ImageDetIter), 'Synchronize with invalid iterator.'
        mine, theirs = self.label_shape, it.label_shape
        assert mine[1] == theirs[1], 'object width mismatch.'
        most = max(mine[0], theirs[0])
        for target, shape in ((self, mine), (it, theirs)):
            if shape[0] < most:
                target.reshape(None, (most, shape[1]))
        if verbose and most > min(mine[0], theirs[0]):
            logging.info('Resized label_shape to (%d, %d).', most, mine[1])
        return it

    # ---------------------------------------------------------------- samples / batches
    def augmentation_transform(self, data, label):  # pylint: disable=arguments-differ
        for aug in self.auglist:
            data, label = aug(data, label)
        return data, label

    def _load_one(self, label, raw):
        img = self.imdecode(raw)
        self.check_valid_image([img])
        img, objs = self.augmentation_transform(img, self._parse_label(label))
        self._check_valid_label(objs)
        padded = np.full(self.provide_label[0][1][1:], -1.0, dtype=np.float32)
        keep = min(objs.shape[0], padded.shape[0])
        padded[:keep] = objs[:keep]
        return self.postprocess_data(img), nd.array(padded)

    def _empty_label_batch(self):
        return nd.full(self.provide_label[0][1], -1.0)
