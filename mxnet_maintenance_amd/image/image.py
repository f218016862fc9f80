"""Image decoding, transforms, augmenters and ImageIter (mx.image).

Parity: python/mxnet/image/image.py (imread/imdecode/imresize/resize_short/
crops/color_normalize/random_size_crop/imrotate, the Augmenter family,
CreateAugmenter, ImageIter).  The reference decodes with OpenCV in C++;
here decoding is PIL (libjpeg-turbo, releases the GIL so ImageIter's thread
pool scales) and images are HWC NDArrays exactly like the reference.
"""
import io as _io
import json
import logging
import math
import os
import random as _pyrandom

import numpy as np

from ..base import MXNetError
from .. import ndarray as nd
from ..ndarray.ndarray import NDArray
from .. import io as mxio
from .. import recordio

__all__ = ['imread', 'imdecode', 'imdecode_np', 'imresize', 'scale_down', 'copyMakeBorder', 'resize_short',
           'fixed_crop', 'random_crop', 'center_crop', 'color_normalize', 'random_size_crop', 'imrotate',
           'random_rotate', 'Augmenter', 'SequentialAug', 'ResizeAug', 'ForceResizeAug', 'RandomCropAug',
           'RandomSizedCropAug', 'CenterCropAug', 'RandomOrderAug', 'BrightnessJitterAug', 'ContrastJitterAug',
           'SaturationJitterAug', 'HueJitterAug', 'ColorJitterAug', 'LightingAug', 'ColorNormalizeAug',
           'RandomGrayAug', 'HorizontalFlipAug', 'CastAug', 'CreateAugmenter', 'ImageIter']

_GRAY = np.array([0.299, 0.587, 0.114], dtype=np.float32)


def _np(src):
    return src.asnumpy() if isinstance(src, NDArray) else np.asarray(src)


def _wrap(a, like):
    return nd.array(a, dtype=a.dtype) if isinstance(like, NDArray) or like is None else a


def imdecode_np(buf, flag=1, to_rgb=True):
    """Decode an encoded image (bytes) to a HWC uint8 numpy array (RGB, or BGR with to_rgb=False)."""
    from PIL import Image
    if isinstance(buf, NDArray):
        buf = buf.asnumpy().astype(np.uint8).tobytes()
    elif isinstance(buf, np.ndarray):
        buf = buf.tobytes()
    try:
        im = Image.open(_io.BytesIO(buf))
        im = im.convert('RGB' if flag else 'L')
    except Exception as e:
        raise MXNetError('Decoding failed. Invalid image file: %s' % e)
    a = np.asarray(im)
    if not flag:
        return a[:, :, None]
    if not to_rgb:
        a = a[:, :, ::-1]
    return np.ascontiguousarray(a)


def imdecode(buf, flag=1, to_rgb=1, out=None):
    """Decode an image to an NDArray (HWC, uint8)."""
    a = imdecode_np(buf, flag, bool(to_rgb))
    r = nd.array(a, dtype='uint8')
    if out is not None:
        out[:] = r
        return out
    return r


def imread(filename, flag=1, to_rgb=True, out=None):
    with open(filename, 'rb') as f:
        return imdecode(f.read(), flag, to_rgb, out)


_PIL_INTERP = None


def _interp(interp, sizes=()):
    from PIL import Image
    table = {0: Image.NEAREST, 1: Image.BILINEAR, 2: Image.BICUBIC, 3: Image.BOX, 4: Image.LANCZOS}
    if interp == 9:
        if sizes:
            oh, ow, nh, nw = sizes
            if nh > oh and nw > ow:
                return Image.BICUBIC
            if nh < oh and nw < ow:
                return Image.BOX
        return Image.BILINEAR
    if interp == 10:
        return table[_pyrandom.randint(0, 4)]
    return table.get(interp, Image.BILINEAR)


def _get_interp_method(interp, sizes=()):
    if interp == 9 and sizes:
        oh, ow, nh, nw = sizes
        if nh > oh and nw > ow:
            return 2
        if nh < oh and nw < ow:
            return 3
        return 1
    if interp == 10:
        return _pyrandom.randint(0, 4)
    if interp not in (0, 1, 2, 3, 4):
        raise ValueError('Unknown interp method %d' % interp)
    return interp


def _resize_np(a, w, h, interp=1):
    from PIL import Image
    mode = _interp(interp, (a.shape[0], a.shape[1], h, w))
    if a.dtype == np.uint8:
        if a.shape[2] == 1:
            return np.asarray(Image.fromarray(a[:, :, 0]).resize((w, h), mode))[:, :, None]
        return np.asarray(Image.fromarray(a).resize((w, h), mode))
    chans = [np.asarray(Image.fromarray(a[:, :, c].astype(np.float32), mode='F').resize((w, h), mode))
             for c in range(a.shape[2])]
    return np.stack(chans, axis=2).astype(a.dtype)


def imresize(src, w, h, interp=1, out=None):
    # OpenCV interpolation codes (src/io/image_io.cc: 0 nearest .. 4 lanczos, 9 auto, 10 random)
    if int(interp) not in (0, 1, 2, 3, 4, 9, 10):
        from ..base import MXNetError
        raise MXNetError('imresize: invalid interpolation method %r (OpenCV error: Bad flag)' % (interp,))
    r = _wrap(_resize_np(_np(src), int(w), int(h), interp), src)
    if out is not None:
        out[:] = r
        return out
    return r


def scale_down(src_size, size):
    w, h = size
    sw, sh = src_size
    if sh < h:
        w, h = float(w * sh) / h, sh
    if sw < w:
        w, h = sw, float(h * sw) / w
    return int(w), int(h)


def copyMakeBorder(src, top, bot, left, right, type=0, value=0, values=None, out=None):  # noqa: A002
    """Pad an image; type 0 = constant, 1 = replicate, 2 = reflect (cv2 BORDER_* codes)."""
    a = _np(src)
    pad = ((top, bot), (left, right), (0, 0))
    if type == 0:
        cval = values if values is not None else value
        if np.ndim(cval):
            r = np.stack([np.pad(a[:, :, c], pad[:2], constant_values=cval[c]) for c in range(a.shape[2])], 2)
        else:
            r = np.pad(a, pad, constant_values=cval)
    else:
        r = np.pad(a, pad, mode={1: 'edge', 2: 'symmetric', 4: 'reflect'}.get(type, 'edge'))
    r = _wrap(r, src)
    if out is not None:
        out[:] = r
        return out
    return r


def resize_short(src, size, interp=2):
    h, w = src.shape[0], src.shape[1]
    if h > w:
        new_h, new_w = size * h // w, size
    else:
        new_h, new_w = size, size * w // h
    return imresize(src, new_w, new_h, interp=_get_interp_method(interp, (h, w, new_h, new_w)))


def fixed_crop(src, x0, y0, w, h, size=None, interp=2):
    out = src[y0:y0 + h, x0:x0 + w]
    if size is not None and (w, h) != tuple(size):
        sizes = (h, w, size[1], size[0])
        out = imresize(out, *size, interp=_get_interp_method(interp, sizes))
    return out


def random_crop(src, size, interp=2):
    h, w = src.shape[0], src.shape[1]
    new_w, new_h = scale_down((w, h), size)
    x0 = _pyrandom.randint(0, w - new_w)
    y0 = _pyrandom.randint(0, h - new_h)
    out = fixed_crop(src, x0, y0, new_w, new_h, size, interp)
    return out, (x0, y0, new_w, new_h)


def center_crop(src, size, interp=2):
    h, w = src.shape[0], src.shape[1]
    new_w, new_h = scale_down((w, h), size)
    x0 = int((w - new_w) / 2)
    y0 = int((h - new_h) / 2)
    out = fixed_crop(src, x0, y0, new_w, new_h, size, interp)
    return out, (x0, y0, new_w, new_h)


def color_normalize(src, mean, std=None):
    if mean is not None:
        src = src - mean
    if std is not None:
        src = src / std
    return src


def random_size_crop(src, size, area, ratio, interp=2, **kwargs):
    h, w = src.shape[0], src.shape[1]
    src_area = h * w
    if 'min_area' in kwargs:
        area = kwargs.pop('min_area')
    if isinstance(area, (int, float)):
        area = (area, 1.0)
    for _ in range(10):
        target_area = _pyrandom.uniform(area[0], area[1]) * src_area
        log_ratio = (np.log(ratio[0]), np.log(ratio[1]))
        new_ratio = np.exp(_pyrandom.uniform(*log_ratio))
        new_w = int(round(np.sqrt(target_area * new_ratio)))
        new_h = int(round(np.sqrt(target_area / new_ratio)))
        if new_w <= w and new_h <= h:
            x0 = _pyrandom.randint(0, w - new_w)
            y0 = _pyrandom.randint(0, h - new_h)
            out = fixed_crop(src, x0, y0, new_w, new_h, size, interp)
            return out, (x0, y0, new_w, new_h)
    return center_crop(src, size, interp)


def imrotate(src, rotation_degrees, zoom_in=False, zoom_out=False):
    """Rotate CHW (or NCHW) float images by the given degrees (bilinear, zero fill)."""
    import torch
    import torch.nn.functional as F
    if zoom_in and zoom_out:
        raise ValueError('`zoom_in` and `zoom_out` cannot be both True')
    x = src._data if isinstance(src, NDArray) else torch.as_tensor(src)
    if x.dtype not in (torch.float32, torch.float64, torch.float16):
        raise TypeError('Only floating point types are supported')
    squeeze = x.dim() == 3
    if squeeze:
        x = x.unsqueeze(0)
    n, _, h, w = x.shape
    deg = rotation_degrees._data if isinstance(rotation_degrees, NDArray) else torch.as_tensor(rotation_degrees)
    deg = deg.to(x.dtype).reshape(-1).expand(n) if deg.numel() == 1 else deg.to(x.dtype).reshape(-1)
    rad = deg * math.pi / 180
    c, s = torch.cos(rad), torch.sin(rad)
    scale = torch.ones_like(c)
    if zoom_in or zoom_out:
        ar = w / h
        hw = (torch.abs(c) * w + torch.abs(s) * h) / w
        hh = (torch.abs(s) * w + torch.abs(c) * h) / h
        big = torch.maximum(hw, hh)
        scale = 1 / big if zoom_in else big
        del ar
    theta = torch.zeros(n, 2, 3, dtype=x.dtype)
    theta[:, 0, 0] = c * scale
    theta[:, 0, 1] = -s * scale * h / w
    theta[:, 1, 0] = s * scale * w / h
    theta[:, 1, 1] = c * scale
    grid = F.affine_grid(theta.to(x.device), list(x.shape), align_corners=False)
    y = F.grid_sample(x, grid, align_corners=False)
    if squeeze:
        y = y[0]
    return NDArray(y)


def random_rotate(src, angle_limits, zoom_in=False, zoom_out=False):
    n = src.shape[0] if src.ndim == 4 else 1
    ang = np.random.uniform(angle_limits[0], angle_limits[1], size=n)
    return imrotate(src, nd.array(ang), zoom_in, zoom_out)


class Augmenter:
    """Image augmenter base class (callable on HWC NDArrays)."""

    def __init__(self, **kwargs):
        self._kwargs = kwargs
        for k, v in self._kwargs.items():
            if isinstance(v, NDArray):
                v = v.asnumpy()
            if isinstance(v, np.ndarray):
                self._kwargs[k] = v.tolist()

    def dumps(self):
        return json.dumps([self.__class__.__name__.lower(), self._kwargs])

    def __call__(self, src):
        raise NotImplementedError


class SequentialAug(Augmenter):
    def __init__(self, ts):
        super().__init__()
        self.ts = ts

    def dumps(self):
        return [self.__class__.__name__.lower(), [x.dumps() for x in self.ts]]

    def __call__(self, src):
        for aug in self.ts:
            src = aug(src)
        return src


class ResizeAug(Augmenter):
    def __init__(self, size, interp=2):
        super().__init__(size=size, interp=interp)
        self.size, self.interp = size, interp

    def __call__(self, src):
        return resize_short(src, self.size, self.interp)


class ForceResizeAug(Augmenter):
    def __init__(self, size, interp=2):
        super().__init__(size=size, interp=interp)
        self.size, self.interp = size, interp

    def __call__(self, src):
        sizes = (src.shape[0], src.shape[1], self.size[1], self.size[0])
        return imresize(src, *self.size, interp=_get_interp_method(self.interp, sizes))


class RandomCropAug(Augmenter):
    def __init__(self, size, interp=2):
        super().__init__(size=size, interp=interp)
        self.size, self.interp = size, interp

    def __call__(self, src):
        return random_crop(src, self.size, self.interp)[0]


class RandomSizedCropAug(Augmenter):
    def __init__(self, size, area, ratio, interp=2, **kwargs):
        super().__init__(size=size, area=area, ratio=ratio, interp=interp)
        self.size, self.interp, self.ratio = size, interp, ratio
        self.area = kwargs.pop('min_area') if 'min_area' in kwargs else area

    def __call__(self, src):
        return random_size_crop(src, self.size, self.area, self.ratio, self.interp)[0]


class CenterCropAug(Augmenter):
    def __init__(self, size, interp=2):
        super().__init__(size=size, interp=interp)
        self.size, self.interp = size, interp

    def __call__(self, src):
        return center_crop(src, self.size, self.interp)[0]


class RandomOrderAug(Augmenter):
    def __init__(self, ts):
        super().__init__()
        self.ts = ts

    def dumps(self):
        return [self.__class__.__name__.lower(), [x.dumps() for x in self.ts]]

    def __call__(self, src):
        order = list(self.ts)
        _pyrandom.shuffle(order)
        for t in order:
            src = t(src)
        return src


class BrightnessJitterAug(Augmenter):
    def __init__(self, brightness):
        super().__init__(brightness=brightness)
        self.brightness = brightness

    def __call__(self, src):
        alpha = 1.0 + _pyrandom.uniform(-self.brightness, self.brightness)
        return src * alpha


class ContrastJitterAug(Augmenter):
    def __init__(self, contrast):
        super().__init__(contrast=contrast)
        self.contrast = contrast

    def __call__(self, src):
        alpha = 1.0 + _pyrandom.uniform(-self.contrast, self.contrast)
        a = _np(src).astype(np.float32)
        gray = (a * _GRAY).sum(axis=2)
        gray = (3.0 * (1.0 - alpha) / gray.size) * gray.sum()
        return _wrap((a * alpha + gray).astype(np.float32), src)


class SaturationJitterAug(Augmenter):
    def __init__(self, saturation):
        super().__init__(saturation=saturation)
        self.saturation = saturation

    def __call__(self, src):
        alpha = 1.0 + _pyrandom.uniform(-self.saturation, self.saturation)
        a = _np(src).astype(np.float32)
        gray = (a * _GRAY).sum(axis=2, keepdims=True) * (1.0 - alpha)
        return _wrap((a * alpha + gray).astype(np.float32), src)


class HueJitterAug(Augmenter):
    def __init__(self, hue):
        super().__init__(hue=hue)
        self.hue = hue
        self.tyiq = np.array([[0.299, 0.587, 0.114], [0.596, -0.274, -0.321], [0.211, -0.523, 0.311]])
        self.ityiq = np.array([[1.0, 0.956, 0.621], [1.0, -0.272, -0.647], [1.0, -1.107, 1.705]])

    def __call__(self, src):
        alpha = _pyrandom.uniform(-self.hue, self.hue)
        u, w = np.cos(alpha * np.pi), np.sin(alpha * np.pi)
        bt = np.array([[1.0, 0.0, 0.0], [0.0, u, -w], [0.0, w, u]])
        t = np.dot(np.dot(self.ityiq, bt), self.tyiq).T
        a = _np(src).astype(np.float32)
        return _wrap(np.dot(a, t.astype(np.float32)), src)


class ColorJitterAug(RandomOrderAug):
    def __init__(self, brightness, contrast, saturation):
        ts = []
        if brightness > 0:
            ts.append(BrightnessJitterAug(brightness))
        if contrast > 0:
            ts.append(ContrastJitterAug(contrast))
        if saturation > 0:
            ts.append(SaturationJitterAug(saturation))
        super().__init__(ts)


class LightingAug(Augmenter):
    def __init__(self, alphastd, eigval, eigvec):
        super().__init__(alphastd=alphastd, eigval=eigval, eigvec=eigvec)
        self.alphastd = alphastd
        self.eigval = np.asarray(eigval)
        self.eigvec = np.asarray(eigvec)

    def __call__(self, src):
        alpha = np.random.normal(0, self.alphastd, size=(3,))
        rgb = np.dot(self.eigvec * alpha, self.eigval)
        return src + nd.array(rgb.astype(np.float32)) if isinstance(src, NDArray) else src + rgb


class ColorNormalizeAug(Augmenter):
    def __init__(self, mean, std):
        super().__init__(mean=mean, std=std)
        self.mean = mean if mean is None or isinstance(mean, NDArray) else nd.array(mean)
        self.std = std if std is None or isinstance(std, NDArray) else nd.array(std)

    def __call__(self, src):
        return color_normalize(src, self.mean, self.std)


class RandomGrayAug(Augmenter):
    def __init__(self, p):
        super().__init__(p=p)
        self.p = p
        self.mat = np.array([[0.21, 0.21, 0.21], [0.72, 0.72, 0.72], [0.07, 0.07, 0.07]], dtype=np.float32)

    def __call__(self, src):
        if _pyrandom.random() < self.p:
            src = _wrap(np.dot(_np(src).astype(np.float32), self.mat), src)
        return src


class HorizontalFlipAug(Augmenter):
    def __init__(self, p):
        super().__init__(p=p)
        self.p = p

    def __call__(self, src):
        if _pyrandom.random() < self.p:
            src = nd.flip(src, axis=1)
        return src


class CastAug(Augmenter):
    def __init__(self, typ='float32'):
        super().__init__(type=typ)
        self.typ = typ

    def __call__(self, src):
        return src.astype(self.typ)


def CreateAugmenter(data_shape, resize=0, rand_crop=False, rand_resize=False, rand_mirror=False, mean=None,
                    std=None, brightness=0, contrast=0, saturation=0, hue=0, pca_noise=0, rand_gray=0,
                    inter_method=2):
    """Standard augmenter list (resize -> crop -> flip -> cast -> color -> normalize)."""
    auglist = []
    if resize > 0:
        auglist.append(ResizeAug(resize, inter_method))
    crop_size = (data_shape[2], data_shape[1])
    if rand_resize:
        assert rand_crop
        auglist.append(RandomSizedCropAug(crop_size, 0.08, (3.0 / 4.0, 4.0 / 3.0), inter_method))
    elif rand_crop:
        auglist.append(RandomCropAug(crop_size, inter_method))
    else:
        auglist.append(CenterCropAug(crop_size, inter_method))
    if rand_mirror:
        auglist.append(HorizontalFlipAug(0.5))
    auglist.append(CastAug())
    if brightness or contrast or saturation:
        auglist.append(ColorJitterAug(brightness, contrast, saturation))
    if hue:
        auglist.append(HueJitterAug(hue))
    if pca_noise > 0:
        eigval = np.array([55.46, 4.794, 1.148])
        eigvec = np.array([[-0.5675, 0.7192, 0.4009], [-0.5808, -0.0045, -0.8140], [-0.5836, -0.6948, 0.4203]])
        auglist.append(LightingAug(pca_noise, eigval, eigvec))
    if rand_gray > 0:
        auglist.append(RandomGrayAug(rand_gray))
    if mean is True:
        mean = nd.array([123.68, 116.28, 103.53])
    if std is True:
        std = nd.array([58.395, 57.12, 57.375])
    if mean is not None or std is not None:
        auglist.append(ColorNormalizeAug(mean, std))
    return auglist


class ImageIter(mxio.DataIter):
    """Image iterator over a .rec file, an image list file or an in-memory list, with augmenters.

    Decoding+augmentation of a batch runs on a thread pool of
    ``MXNET_CPU_WORKER_NTHREADS`` workers (PIL releases the GIL).
    """

    def __init__(self, batch_size, data_shape, label_width=1, path_imgrec=None, path_imglist=None, path_root=None,
                 path_imgidx=None, shuffle=False, part_index=0, num_parts=1, aug_list=None, imglist=None,
                 data_name='data', label_name='softmax_label', dtype='float32', last_batch_handle='pad',
                 **kwargs):
        super().__init__()
        assert path_imgrec or path_imglist or isinstance(imglist, list)
        assert dtype in ['int32', 'float32', 'int64', 'float64'], dtype + ' label not supported'
        if path_imgrec:
            if path_imgidx:
                self.imgrec = recordio.MXIndexedRecordIO(path_imgidx, path_imgrec, 'r')
                self.imgidx = list(self.imgrec.keys)
            else:
                self.imgrec = recordio.MXRecordIO(path_imgrec, 'r')
                self.imgidx = None
        else:
            self.imgrec = None
        imgkeys = []
        if path_imglist:
            with open(path_imglist) as fin:
                imglist_d = {}
                for line in fin:
                    line = line.strip().split('\t')
                    if len(line) < 2:
                        continue
                    label = nd.array([float(x) for x in line[1:-1]], dtype=dtype)
                    key = int(line[0])
                    imglist_d[key] = (label, line[-1])
                    imgkeys.append(key)
                self.imglist = imglist_d
        elif isinstance(imglist, list):
            result = {}
            for index, img in enumerate(imglist, 1):
                key = str(index)
                if len(img) > 2:
                    label = nd.array(img[:-1], dtype=dtype)
                elif isinstance(img[0], (int, float, np.number)):
                    label = nd.array([img[0]], dtype=dtype)
                else:
                    label = nd.array(img[0], dtype=dtype)
                result[key] = (label, img[-1])
                imgkeys.append(key)
            self.imglist = result
        else:
            self.imglist = None
        self.path_root = path_root
        self.check_data_shape(data_shape)
        self.provide_data = [(data_name, (batch_size,) + tuple(data_shape))]
        self.provide_label = [(label_name, (batch_size, label_width) if label_width > 1 else (batch_size,))]
        self.batch_size = batch_size
        self.data_shape = tuple(data_shape)
        self.label_width = label_width
        self.shuffle = shuffle
        self.dtype = dtype
        if self.imgrec is None:
            self.seq = imgkeys
        elif shuffle or num_parts > 1 or path_imgidx:
            assert self.imgidx is not None
            self.seq = self.imgidx
        else:
            self.seq = None
        if num_parts > 1:
            assert part_index < num_parts
            n = len(self.seq)
            c = n // num_parts
            self.seq = self.seq[part_index * c:(part_index + 1) * c]
        self.auglist = CreateAugmenter(data_shape, **kwargs) if aug_list is None else aug_list
        self.cur = 0
        self._allow_read = True
        self.last_batch_handle = last_batch_handle
        self.num_image = len(self.seq) if self.seq is not None else None
        self._cache_data = None
        self._cache_label = None
        self._cache_idx = None
        self.reset()

    def reset(self):
        if self.seq is not None and self.shuffle:
            _pyrandom.shuffle(self.seq)
        if self.last_batch_handle != 'roll_over' or self._cache_data is None:
            if self.imgrec is not None:
                self.imgrec.reset()
            self.cur = 0
            if self._allow_read is False:
                self._allow_read = True

    def hard_reset(self):
        if self.seq is not None and self.shuffle:
            _pyrandom.shuffle(self.seq)
        if self.imgrec is not None:
            self.imgrec.reset()
        self.cur = 0
        self._allow_read = True
        self._cache_data = None
        self._cache_label = None
        self._cache_idx = None

    def next_sample(self):
        if self._allow_read is False:
            raise StopIteration
        if self.seq is not None:
            if self.cur < self.num_image:
                idx = self.seq[self.cur]
            else:
                if self.last_batch_handle != 'discard':
                    self.cur = 0
                raise StopIteration
            self.cur += 1
            if self.imgrec is not None:
                s = self.imgrec.read_idx(idx)
                header, img = recordio.unpack(s)
                if self.imglist is None:
                    return header.label, img
                return self.imglist[idx][0], img
            label, fname = self.imglist[idx]
            return label, self.read_image(fname)
        s = self.imgrec.read()
        if s is None:
            if self.last_batch_handle != 'discard':
                self.imgrec.reset()
            raise StopIteration
        header, img = recordio.unpack(s)
        return header.label, img

    def _batchify(self, batch_data, batch_label, start=0):
        i = start
        batch_size = self.batch_size
        try:
            while i < batch_size:
                label, s = self.next_sample()
                data = self.imdecode(s)
                try:
                    self.check_valid_image(data)
                except RuntimeError as e:
                    logging.debug('Invalid image, skipping:  %s', str(e))
                    continue
                data = self.augmentation_transform(data)
                assert i < batch_size, 'Batch size must be multiples of augmenter output length'
                batch_data[i] = self.postprocess_data(data)
                batch_label[i] = label
                i += 1
        except StopIteration:
            if not i:
                raise StopIteration
        return i

    def next(self):
        batch_size = self.batch_size
        c, h, w = self.data_shape
        if self._cache_data is not None:
            assert self._cache_label is not None
            assert self._cache_idx is not None
            batch_data, batch_label, i = self._cache_data, self._cache_label, self._cache_idx
        else:
            batch_data = nd.zeros((batch_size, c, h, w))
            batch_label = nd.empty(self.provide_label[0][1])
            batch_label[:] = 0
            i = self._batchify(batch_data, batch_label)
        pad = batch_size - i
        if pad != 0:
            if self.last_batch_handle == 'discard':
                raise StopIteration
            if self.last_batch_handle == 'roll_over' and self._cache_data is None:
                self._cache_data, self._cache_label, self._cache_idx = batch_data, batch_label, i
                raise StopIteration
            _ = self._batchify(batch_data, batch_label, i)
            if self.last_batch_handle == 'pad':
                self._allow_read = False
            else:
                self._cache_data = self._cache_label = self._cache_idx = None
        return mxio.DataBatch([batch_data], [batch_label], pad=pad)

    def check_data_shape(self, data_shape):
        if not len(data_shape) == 3:
            raise ValueError('data_shape should have length 3, with dimensions CxHxW')
        if not data_shape[0] == 3:
            raise ValueError('This iterator expects inputs to have 3 channels.')

    def check_valid_image(self, data):
        if len(data[0].shape) == 0:
            raise RuntimeError('Data shape is wrong')

    def imdecode(self, s):
        def locate():
            if self.seq is not None:
                idx = self.seq[(self.cur % self.num_image) - 1]
            else:
                idx = (self.cur % self.num_image) - 1
            if self.imglist is not None:
                _, fname = self.imglist[idx]
                return 'Broken image filename: {}'.format(fname)
            return 'Broken image index: {}'.format(idx)
        try:
            img = imdecode(s)
        except Exception as e:
            raise RuntimeError('{}, {}'.format(locate(), e))
        return img

    def read_image(self, fname):
        with open(os.path.join(self.path_root or '', fname), 'rb') as fin:
            return fin.read()

    def augmentation_transform(self, data):
        for aug in self.auglist:
            data = aug(data)
        return data

    def postprocess_data(self, datum):
        return nd.transpose(datum, axes=(2, 0, 1))
