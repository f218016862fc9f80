"""mx.image: decoding, geometric / photometric transforms, augmenter pipelines and ``ImageIter``.

Behavioural parity with python/mxnet/image/image.py (reference: imdecode :85, imresize :301,
scale_down :406, copyMakeBorder :437, resize_short :523, fixed_crop :563, random_crop :594,
center_crop :640... imrotate :618, the Augmenter family :848-1240, CreateAugmenter :1180 and
ImageIter :1250).  The reference decodes and resizes with OpenCV inside its C++ operator library;
this module keeps the host-side work in numpy + PIL (libjpeg-turbo, GIL released while decoding)
and does the batched float work (rotation) with torch so it runs on the GPU when the input lives
there.  The high-throughput training input path is the native ``io.ImageRecordIter`` (C++ decode
pool + pinned ring, io/image_record.py); ``ImageIter`` is the flexible Python iterator.

Layout conventions follow the reference: single images are HWC (uint8 after decoding, float32
after ``CastAug``); ``imrotate`` works on CHW / NCHW float32.
"""
import io as _bytesio
import json
import logging
import math
import os
import random as _rand
from numbers import Number

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

# ITU-R 601 luma weights (RGB order), used by the contrast / saturation jitters
_LUMA = np.array([0.299, 0.587, 0.114], dtype=np.float32)
# ImageNet statistics used by CreateAugmenter(mean=True / std=True / pca_noise>0)
_IMAGENET_MEAN = (123.68, 116.28, 103.53)
_IMAGENET_STD = (58.395, 57.12, 57.375)
_PCA_EIGVAL = np.array([55.46, 4.794, 1.148])
_PCA_EIGVEC = np.array([[-0.5675, 0.7192, 0.4009],
                        [-0.5808, -0.0045, -0.8140],
                        [-0.5836, -0.6948, 0.4203]])


# --------------------------------------------------------------------------- array plumbing
def _host(img):
    """numpy view of an image argument (NDArray or array-like)."""
    return img.asnumpy() if isinstance(img, NDArray) else np.asarray(img)


def _like(arr, ref):
    """Return ``arr`` in the container type of ``ref`` (NDArray unless ``ref`` is a numpy array)."""
    if isinstance(ref, np.ndarray):
        return arr
    return nd.array(arr, dtype=arr.dtype)


def _emit(result, out):
    """Honour the reference's optional ``out=`` argument."""
    if out is None:
        return result
    out[:] = result
    return out


# --------------------------------------------------------------------------- decode
def _as_bytes(buf):
    if isinstance(buf, NDArray):
        return buf.asnumpy().astype(np.uint8).tobytes()
    if isinstance(buf, np.ndarray):
        return buf.tobytes()
    return bytes(buf)


def imdecode_np(buf, flag=1, to_rgb=True):
    """Decode encoded image bytes to a contiguous HWC uint8 numpy array.

    ``flag`` 1 = 3-channel colour, 0 = one grey channel; ``to_rgb=False`` gives OpenCV's BGR order.
    """
    from PIL import Image
    data = _as_bytes(buf)
    if not data:
        raise MXNetError('Decoding failed: empty image buffer')
    try:
        with Image.open(_bytesio.BytesIO(data)) as im:
            pixels = np.asarray(im.convert('RGB' if flag else 'L'))
    except Exception as err:       # PIL raises several unrelated exception types
        raise MXNetError('Decoding failed. Invalid image file: %s' % err)
    if pixels.ndim == 2:
        return np.ascontiguousarray(pixels[:, :, None])
    return np.ascontiguousarray(pixels if to_rgb else pixels[:, :, ::-1])


def imdecode(buf, flag=1, to_rgb=1, out=None):
    """Decode an image buffer into an HWC uint8 NDArray (RGB unless ``to_rgb`` is false)."""
    return _emit(nd.array(imdecode_np(buf, flag, bool(to_rgb)), dtype='uint8'), out)


def imread(filename, flag=1, to_rgb=True, out=None):
    """Read and decode an image file (HWC uint8 NDArray)."""
    try:
        with open(filename, 'rb') as fh:
            payload = fh.read()
    except OSError as err:
        raise MXNetError('imread: cannot open %s (%s)' % (filename, err))
    return imdecode(payload, flag, to_rgb, out)


# --------------------------------------------------------------------------- resize
# OpenCV interpolation codes accepted by the reference (src/io/image_io.cc): 0 nearest, 1 bilinear,
# 2 bicubic, 3 area, 4 lanczos, 9 = pick by direction (cubic up / area down / linear), 10 = random.
_CONCRETE_INTERP = (0, 1, 2, 3, 4)


def _get_interp_method(interp, sizes=()):
    """Resolve the meta codes 9 / 10 into one of 0..4 for a resize ``sizes=(oh, ow, nh, nw)``."""
    if interp == 10:
        return _rand.randint(0, 4)
    if interp == 9:
        if not sizes:
            return 1
        old_h, old_w, new_h, new_w = sizes
        grow = new_h > old_h and new_w > old_w
        shrink = new_h < old_h and new_w < old_w
        return 2 if grow else (3 if shrink else 1)
    if interp not in _CONCRETE_INTERP:
        raise ValueError('Unknown interp method %d' % interp)
    return interp


def _pil_filter(code):
    from PIL import Image
    return (Image.NEAREST, Image.BILINEAR, Image.BICUBIC, Image.BOX, Image.LANCZOS)[code]


def _resize_np(pixels, w, h, interp=1):
    """Resize an HWC numpy image to (h, w); uint8 keeps PIL's fast path, floats go per channel."""
    from PIL import Image
    code = _get_interp_method(interp, (pixels.shape[0], pixels.shape[1], h, w))
    flt = _pil_filter(code)
    if pixels.dtype == np.uint8:
        if pixels.shape[2] == 1:
            return np.asarray(Image.fromarray(pixels[:, :, 0]).resize((w, h), flt))[:, :, None]
        return np.asarray(Image.fromarray(pixels).resize((w, h), flt))
    planes = []
    for ch in range(pixels.shape[2]):
        plane = Image.fromarray(np.ascontiguousarray(pixels[:, :, ch], dtype=np.float32), mode='F')
        planes.append(np.asarray(plane.resize((w, h), flt)))
    return np.stack(planes, axis=2).astype(pixels.dtype)


def imresize(src, w, h, interp=1, out=None):
    """Resize ``src`` (HWC) to exactly ``w`` x ``h``."""
    if int(interp) not in _CONCRETE_INTERP + (9, 10):
        raise MXNetError('imresize: invalid interpolation method %r (OpenCV error: Bad flag)' % (interp,))
    return _emit(_like(_resize_np(_host(src), int(w), int(h), interp), src), out)


def scale_down(src_size, size):
    """Shrink the crop ``size=(w, h)`` until it fits inside ``src_size=(w, h)``, keeping its aspect."""
    crop_w, crop_h = size
    img_w, img_h = src_size
    if img_h < crop_h:
        crop_w, crop_h = float(crop_w * img_h) / crop_h, img_h
    if img_w < crop_w:
        crop_w, crop_h = img_w, float(crop_h * img_w) / crop_w
    return int(crop_w), int(crop_h)


# cv2.BORDER_* -> numpy.pad mode (0 = constant is handled separately)
_BORDER_MODES = {1: 'edge', 2: 'symmetric', 3: 'wrap', 4: 'reflect'}


def copyMakeBorder(src, top, bot, left, right, type=0, value=0, values=None, out=None):  # noqa: A002
    """Pad an HWC image; ``type`` is an OpenCV border code (0 constant, 1 replicate, 2 reflect,
    3 wrap, 4 reflect-101)."""
    pixels = _host(src)
    spatial = ((top, bot), (left, right))
    if type == 0:
        fill = value if values is None else values
        if np.ndim(fill):
            padded = np.stack([np.pad(pixels[:, :, c], spatial, constant_values=fill[c])
                               for c in range(pixels.shape[2])], axis=2)
        else:
            padded = np.pad(pixels, spatial + ((0, 0),), constant_values=fill)
    else:
        if type not in _BORDER_MODES:
            raise MXNetError('copyMakeBorder: unsupported border type %r' % (type,))
        padded = np.pad(pixels, spatial + ((0, 0),), mode=_BORDER_MODES[type])
    return _emit(_like(padded, src), out)


def resize_short(src, size, interp=2):
    """Resize so the shorter edge becomes ``size`` (the longer keeps the aspect ratio)."""
    old_h, old_w = src.shape[0], src.shape[1]
    if old_h > old_w:
        new_w, new_h = size, size * old_h // old_w
    else:
        new_w, new_h = size * old_w // old_h, size
    code = _get_interp_method(interp, (old_h, old_w, new_h, new_w))
    return imresize(src, new_w, new_h, interp=code)


# --------------------------------------------------------------------------- crops
def fixed_crop(src, x0, y0, w, h, size=None, interp=2):
    """Crop the (x0, y0, w, h) window, then resize it to ``size=(w, h)`` when given."""
    window = src[y0:y0 + h, x0:x0 + w]
    if size is None or (w, h) == tuple(size):
        return window
    code = _get_interp_method(interp, (h, w, size[1], size[0]))
    return imresize(window, size[0], size[1], interp=code)


def _crop_at(src, box, size, interp):
    x0, y0, cw, ch = box
    return fixed_crop(src, x0, y0, cw, ch, size, interp), box


def random_crop(src, size, interp=2):
    """Random window of ``size`` (shrunk to fit); returns ``(image, (x0, y0, w, h))``."""
    img_h, img_w = src.shape[0], src.shape[1]
    cw, ch = scale_down((img_w, img_h), size)
    box = (_rand.randint(0, img_w - cw), _rand.randint(0, img_h - ch), cw, ch)
    return _crop_at(src, box, size, interp)


def center_crop(src, size, interp=2):
    """Central window of ``size`` (shrunk to fit); returns ``(image, (x0, y0, w, h))``."""
    img_h, img_w = src.shape[0], src.shape[1]
    cw, ch = scale_down((img_w, img_h), size)
    box = (int((img_w - cw) / 2), int((img_h - ch) / 2), cw, ch)
    return _crop_at(src, box, size, interp)


def random_size_crop(src, size, area, ratio, interp=2, **kwargs):
    """Inception-style crop: random area fraction in ``area`` and log-uniform aspect in ``ratio``
    (10 tries, then a centre crop).  ``min_area=`` is the deprecated spelling of ``area``."""
    img_h, img_w = src.shape[0], src.shape[1]
    area = kwargs.pop('min_area', area)
    lo_area, hi_area = (area, 1.0) if isinstance(area, Number) else area
    log_lo, log_hi = math.log(ratio[0]), math.log(ratio[1])
    for _ in range(10):
        target = _rand.uniform(lo_area, hi_area) * img_h * img_w
        aspect = math.exp(_rand.uniform(log_lo, log_hi))
        cw = int(round(math.sqrt(target * aspect)))
        ch = int(round(math.sqrt(target / aspect)))
        if cw <= img_w and ch <= img_h:
            box = (_rand.randint(0, img_w - cw), _rand.randint(0, img_h - ch), cw, ch)
            return _crop_at(src, box, size, interp)
    return center_crop(src, size, interp)


def color_normalize(src, mean, std=None):
    """``(src - mean) / std`` with either term optional."""
    shifted = src if mean is None else src - mean
    return shifted if std is None else shifted / std


# --------------------------------------------------------------------------- rotation
def imrotate(src, rotation_degrees, zoom_in=False, zoom_out=False):
    """Rotate CHW / NCHW float32 image(s) about their centre (bilinear, zero outside).

    ``rotation_degrees`` is a scalar or (for a batch) one angle per image.  ``zoom_in`` scales so
    no padding is visible, ``zoom_out`` so the whole rotated image fits.
    """
    import torch
    import torch.nn.functional as F
    if zoom_in and zoom_out:
        raise ValueError('`zoom_in` and `zoom_out` cannot be both True')
    if src.dtype != np.float32:
        raise TypeError('Only `float32` images are supported by this function')
    single = src.ndim == 3
    if single and not isinstance(rotation_degrees, Number):
        raise TypeError('When a single image is passed the rotation angle is required to be a scalar.')
    if src.ndim not in (3, 4):
        raise ValueError('Only 3D and 4D are supported by this function')
    imgs = src._data if isinstance(src, NDArray) else torch.as_tensor(src)
    if single:
        imgs = imgs.unsqueeze(0)
    n, _, h, w = imgs.shape
    if isinstance(rotation_degrees, Number):
        theta = torch.full((n,), float(rotation_degrees), dtype=torch.float32, device=imgs.device)
    else:
        raw = rotation_degrees._data if isinstance(rotation_degrees, NDArray) else torch.as_tensor(rotation_degrees)
        theta = raw.reshape(-1).to(device=imgs.device, dtype=torch.float32)
        if theta.numel() != n:
            raise ValueError('The number of images must be equal to the number of rotation angles')
    theta = theta * (math.pi / 180.0)
    cos_t, sin_t = torch.cos(theta).view(n, 1, 1), torch.sin(theta).view(n, 1, 1)
    # pixel-centred sampling grid, rotated in pixel units, then normalised (align_corners=True)
    cy, cx = (h - 1) / 2.0, (w - 1) / 2.0
    ys = (torch.arange(h, dtype=torch.float32, device=imgs.device) - cy).view(1, h, 1)
    xs = (torch.arange(w, dtype=torch.float32, device=imgs.device) - cx).view(1, 1, w)
    gx = (xs * cos_t - ys * sin_t) / cx
    gy = (xs * sin_t + ys * cos_t) / cy
    if zoom_in or zoom_out:
        ac, as_ = cos_t.abs(), sin_t.abs()
        fit = torch.maximum((ac * w + as_ * h) / w, (as_ * w + ac * h) / h)   # bounding box / image
        scale = fit if zoom_out else 1.0 / fit
        gx, gy = gx * scale, gy * scale
    grid = torch.stack([gx, gy], dim=-1)
    rotated = F.grid_sample(imgs, grid, mode='bilinear', padding_mode='zeros', align_corners=True)
    return NDArray(rotated[0] if single else rotated)


def random_rotate(src, angle_limits, zoom_in=False, zoom_out=False):
    """``imrotate`` by angle(s) drawn uniformly from ``angle_limits`` (one per image of a batch)."""
    if src.ndim == 3:
        return imrotate(src, float(np.random.uniform(*angle_limits)), zoom_in, zoom_out)
    angles = np.random.uniform(angle_limits[0], angle_limits[1], size=src.shape[0]).astype(np.float32)
    return imrotate(src, nd.array(angles), zoom_in, zoom_out)


# --------------------------------------------------------------------------- augmenters
class Augmenter:
    """Callable image transform.  Constructor keyword arguments are recorded (JSON-safe) for
    ``dumps`` and exposed as attributes, so subclasses only declare their parameters."""

    def __init__(self, **kwargs):
        self._kwargs = {}
        for key, val in kwargs.items():
            if isinstance(val, NDArray):
                val = val.asnumpy()
            self._kwargs[key] = val.tolist() if isinstance(val, np.ndarray) else val
            self.__dict__.setdefault(key, val)

    def dumps(self):
        """``[name, params]`` JSON description of this augmenter."""
        return json.dumps([type(self).__name__.lower(), self._kwargs])

    def __call__(self, src):
        raise NotImplementedError('Must override implementation.')


class _Composite(Augmenter):
    """Augmenter holding child augmenters (dumps them recursively)."""

    def __init__(self, ts):
        super().__init__()
        self.ts = list(ts)

    def dumps(self):
        return [type(self).__name__.lower(), [child.dumps() for child in self.ts]]

    def _run(self, src, order):
        for child in order:
            src = child(src)
        return src


class SequentialAug(_Composite):
    """Apply the children in order."""

    def __call__(self, src):
        return self._run(src, self.ts)


class RandomOrderAug(_Composite):
    """Apply the children in a freshly shuffled order."""

    def __call__(self, src):
        order = list(self.ts)
        _rand.shuffle(order)
        return self._run(src, order)


class ResizeAug(Augmenter):
    """Shorter edge to ``size``."""

    def __init__(self, size, interp=2):
        super().__init__(size=size, interp=interp)

    def __call__(self, src):
        return resize_short(src, self.size, self.interp)


class ForceResizeAug(Augmenter):
    """Resize to exactly ``size=(w, h)``, ignoring the aspect ratio."""

    def __init__(self, size, interp=2):
        super().__init__(size=size, interp=interp)

    def __call__(self, src):
        code = _get_interp_method(self.interp, (src.shape[0], src.shape[1], self.size[1], self.size[0]))
        return imresize(src, self.size[0], self.size[1], interp=code)


class RandomCropAug(Augmenter):
    """``random_crop`` to ``size``."""

    def __init__(self, size, interp=2):
        super().__init__(size=size, interp=interp)

    def __call__(self, src):
        return random_crop(src, self.size, self.interp)[0]


class RandomSizedCropAug(Augmenter):
    """``random_size_crop`` to ``size``."""

    def __init__(self, size, area, ratio, interp=2, **kwargs):
        area = kwargs.pop('min_area', area)
        super().__init__(size=size, area=area, ratio=ratio, interp=interp)

    def __call__(self, src):
        return random_size_crop(src, self.size, self.area, self.ratio, self.interp)[0]


class CenterCropAug(Augmenter):
    """``center_crop`` to ``size``."""

    def __init__(self, size, interp=2):
        super().__init__(size=size, interp=interp)

    def __call__(self, src):
        return center_crop(src, self.size, self.interp)[0]


def _blend(src, alpha, base):
    """``alpha * src + base`` in float32, keeping the container type of ``src``."""
    return _like((_host(src).astype(np.float32) * alpha + base).astype(np.float32), src)


class BrightnessJitterAug(Augmenter):
    """Scale intensities by ``1 + U(-brightness, brightness)``."""

    def __init__(self, brightness):
        super().__init__(brightness=brightness)

    def __call__(self, src):
        return src * (1.0 + _rand.uniform(-self.brightness, self.brightness))


class ContrastJitterAug(Augmenter):
    """Blend with the image's mean luma by ``1 + U(-contrast, contrast)``."""

    def __init__(self, contrast):
        super().__init__(contrast=contrast)

    def __call__(self, src):
        alpha = 1.0 + _rand.uniform(-self.contrast, self.contrast)
        luma = (_host(src).astype(np.float32) @ _LUMA).mean()
        return _blend(src, alpha, 3.0 * (1.0 - alpha) * luma)


class SaturationJitterAug(Augmenter):
    """Blend with the per-pixel luma by ``1 + U(-saturation, saturation)``."""

    def __init__(self, saturation):
        super().__init__(saturation=saturation)

    def __call__(self, src):
        alpha = 1.0 + _rand.uniform(-self.saturation, self.saturation)
        luma = (_host(src).astype(np.float32) @ _LUMA)[:, :, None]
        return _blend(src, alpha, (1.0 - alpha) * luma)


# RGB <-> YIQ; a hue shift is a rotation of the (I, Q) chroma plane
_RGB2YIQ = np.array([[0.299, 0.587, 0.114], [0.596, -0.274, -0.321], [0.211, -0.523, 0.311]])
_YIQ2RGB = np.array([[1.0, 0.956, 0.621], [1.0, -0.272, -0.647], [1.0, -1.107, 1.705]])


class HueJitterAug(Augmenter):
    """Rotate the chroma plane by ``U(-hue, hue) * pi``."""

    def __init__(self, hue):
        super().__init__(hue=hue)

    def __call__(self, src):
        ang = _rand.uniform(-self.hue, self.hue) * np.pi
        rot = np.array([[1.0, 0.0, 0.0], [0.0, np.cos(ang), -np.sin(ang)], [0.0, np.sin(ang), np.cos(ang)]])
        mix = (_YIQ2RGB @ rot @ _RGB2YIQ).T.astype(np.float32)
        return _like(_host(src).astype(np.float32) @ mix, src)


class ColorJitterAug(RandomOrderAug):
    """Brightness / contrast / saturation jitters (the non-zero ones) in random order."""

    def __init__(self, brightness, contrast, saturation):
        parts = [(brightness, BrightnessJitterAug), (contrast, ContrastJitterAug),
                 (saturation, SaturationJitterAug)]
        super().__init__([cls(amount) for amount, cls in parts if amount > 0])


class LightingAug(Augmenter):
    """AlexNet PCA lighting noise: add ``eigvec @ (alpha * eigval)``, ``alpha ~ N(0, alphastd)``."""

    def __init__(self, alphastd, eigval, eigvec):
        super().__init__(alphastd=alphastd, eigval=eigval, eigvec=eigvec)
        self.eigval, self.eigvec = np.asarray(eigval), np.asarray(eigvec)

    def __call__(self, src):
        alpha = np.random.normal(0, self.alphastd, size=(3,))
        shift = (self.eigvec * alpha) @ self.eigval
        return src + nd.array(shift.astype(np.float32)) if isinstance(src, NDArray) else src + shift


class ColorNormalizeAug(Augmenter):
    """``color_normalize`` with fixed ``mean`` / ``std``."""

    def __init__(self, mean, std):
        super().__init__(mean=mean, std=std)
        self.mean = None if mean is None else (mean if isinstance(mean, NDArray) else nd.array(mean))
        self.std = None if std is None else (std if isinstance(std, NDArray) else nd.array(std))

    def __call__(self, src):
        return color_normalize(src, self.mean, self.std)


# luma-ish grey projection replicated into three channels
_GREY3 = np.repeat(np.array([[0.21], [0.72], [0.07]], dtype=np.float32), 3, axis=1)


class RandomGrayAug(Augmenter):
    """With probability ``p`` replace the image with its grey version."""

    def __init__(self, p):
        super().__init__(p=p)

    def __call__(self, src):
        if _rand.random() >= self.p:
            return src
        return _like(_host(src).astype(np.float32) @ _GREY3, src)


class HorizontalFlipAug(Augmenter):
    """With probability ``p`` mirror left-right."""

    def __init__(self, p):
        super().__init__(p=p)

    def __call__(self, src):
        return nd.flip(src, axis=1) if _rand.random() < self.p else src


class CastAug(Augmenter):
    """Cast to ``typ`` (recorded as ``type`` like the reference)."""

    def __init__(self, typ='float32'):
        super().__init__(type=typ)
        self.typ = typ

    def __call__(self, src):
        return src.astype(self.typ)


def CreateAugmenter(data_shape, resize=0, rand_crop=False, rand_resize=False, rand_mirror=False, mean=None,
                    std=None, brightness=0, contrast=0, saturation=0, hue=0, pca_noise=0, rand_gray=0,
                    inter_method=2):
    """The standard classification pipeline: resize, crop, mirror, cast, colour, normalise."""
    crop = (data_shape[2], data_shape[1])
    if rand_resize:
        assert rand_crop
        cropper = RandomSizedCropAug(crop, 0.08, (3.0 / 4.0, 4.0 / 3.0), inter_method)
    else:
        cropper = (RandomCropAug if rand_crop else CenterCropAug)(crop, inter_method)
    mean = nd.array(_IMAGENET_MEAN) if mean is True else mean
    std = nd.array(_IMAGENET_STD) if std is True else std
    stages = [
        (resize > 0, lambda: ResizeAug(resize, inter_method)),
        (True, lambda: cropper),
        (rand_mirror, lambda: HorizontalFlipAug(0.5)),
        (True, CastAug),
        (brightness or contrast or saturation, lambda: ColorJitterAug(brightness, contrast, saturation)),
        (hue, lambda: HueJitterAug(hue)),
        (pca_noise > 0, lambda: LightingAug(pca_noise, _PCA_EIGVAL, _PCA_EIGVEC)),
        (rand_gray > 0, lambda: RandomGrayAug(rand_gray)),
        (mean is not None or std is not None, lambda: ColorNormalizeAug(mean, std)),
    ]
    return [make() for wanted, make in stages if wanted]


# --------------------------------------------------------------------------- ImageIter
def _read_list_file(path, dtype):
    """``index<TAB>label...<TAB>path`` lines -> (keys, {key: (label, path)})."""
    keys, table = [], {}
    with open(path) as fh:
        for line in fh:
            cols = line.strip().split('\t')
            if len(cols) < 2:
                continue
            key = int(cols[0])
            table[key] = (nd.array([float(v) for v in cols[1:-1]], dtype=dtype), cols[-1])
            keys.append(key)
    return keys, table


def _read_list_obj(items, dtype):
    """In-memory ``[label..., path]`` entries -> (keys, {key: (label, path)}), keys '1', '2', ..."""
    keys, table = [], {}
    for pos, item in enumerate(items, 1):
        key = str(pos)
        if len(item) > 2:
            label = nd.array(item[:-1], dtype=dtype)
        elif isinstance(item[0], (int, float, np.number)):
            label = nd.array([item[0]], dtype=dtype)
        else:
            label = nd.array(item[0], dtype=dtype)
        table[key] = (label, item[-1])
        keys.append(key)
    return keys, table


class ImageIter(mxio.DataIter):
    """Batches of augmented images from a RecordIO file, a ``.lst`` file or an in-memory list.

    Samples come from ``path_imgrec`` (optionally indexed by ``path_imgidx``), from
    ``path_imglist`` / ``imglist`` entries ``[label..., path]`` read under ``path_root``, or from a
    record file whose labels are overridden by a list.  ``last_batch_handle`` is ``'pad'`` (fill
    the last batch from the start of the epoch, report ``pad``), ``'discard'`` or ``'roll_over'``
    (carry the partial batch into the next epoch).  Subclasses customise one sample through
    ``next_sample`` / ``imdecode`` / ``augmentation_transform`` / ``postprocess_data``.
    """

    def __init__(self, batch_size, data_shape, label_width=1, path_imgrec=None, path_imglist=None, path_root=None,
                 path_imgidx=None, shuffle=False, part_index=0, num_parts=1, aug_list=None, imglist=None,
                 data_name='data', label_name='softmax_label', dtype='float32', last_batch_handle='pad',
                 **kwargs):
        super().__init__()
        assert path_imgrec or path_imglist or isinstance(imglist, list)
        assert dtype in ('int32', 'float32', 'int64', 'float64'), dtype + ' label not supported'
        self.imgrec, self.imgidx = None, None
        if path_imgrec and path_imgidx:
            self.imgrec = recordio.MXIndexedRecordIO(path_imgidx, path_imgrec, 'r')
            self.imgidx = list(self.imgrec.keys)
        elif path_imgrec:
            self.imgrec = recordio.MXRecordIO(path_imgrec, 'r')
        keys, self.imglist = [], None
        if path_imglist:
            keys, self.imglist = _read_list_file(path_imglist, dtype)
        elif isinstance(imglist, list):
            keys, self.imglist = _read_list_obj(imglist, dtype)
        self.path_root = path_root
        self.check_data_shape(data_shape)
        self.batch_size = batch_size
        self.data_shape = tuple(data_shape)
        self.label_width = label_width
        self.shuffle = shuffle
        self.dtype = dtype
        self.provide_data = [(data_name, (batch_size,) + self.data_shape)]
        self.provide_label = [(label_name, (batch_size, label_width) if label_width > 1 else (batch_size,))]
        # the visiting order: list keys, record index keys, or None = stream the record file
        if self.imgrec is None:
            self.seq = keys
        elif shuffle or num_parts > 1 or path_imgidx:
            assert self.imgidx is not None
            self.seq = self.imgidx
        else:
            self.seq = None
        if num_parts > 1:
            assert part_index < num_parts
            share = len(self.seq) // num_parts
            self.seq = self.seq[part_index * share:(part_index + 1) * share]
        self.num_image = None if self.seq is None else len(self.seq)
        self.auglist = CreateAugmenter(data_shape, **kwargs) if aug_list is None else aug_list
        self.last_batch_handle = last_batch_handle
        self.cur = 0
        self._allow_read = True
        self._drop_carry()
        self.reset()

    # ---------------------------------------------------------------- epoch control
    def _drop_carry(self):
        self._cache_data = self._cache_label = self._cache_idx = None

    def _rewind(self):
        if self.seq is not None and self.shuffle:
            _rand.shuffle(self.seq)
        if self.imgrec is not None:
            self.imgrec.reset()
        self.cur = 0
        self._allow_read = True

    def reset(self):
        """Start a new epoch (a ``roll_over`` carry keeps the read position)."""
        if self.last_batch_handle == 'roll_over' and self._cache_data is not None:
            if self.seq is not None and self.shuffle:
                _rand.shuffle(self.seq)
            return
        self._rewind()

    def hard_reset(self):
        """Start over and forget any ``roll_over`` carry."""
        self._rewind()
        self._drop_carry()

    # ---------------------------------------------------------------- one sample
    def next_sample(self):
        """``(label, encoded image bytes)`` of the next sample; StopIteration at epoch end."""
        if not self._allow_read:
            raise StopIteration
        if self.seq is None:
            record = self.imgrec.read()
            if record is None:
                if self.last_batch_handle != 'discard':
                    self.imgrec.reset()
                raise StopIteration
            header, payload = recordio.unpack(record)
            return header.label, payload
        if self.cur >= self.num_image:
            if self.last_batch_handle != 'discard':
                self.cur = 0
            raise StopIteration
        key = self.seq[self.cur]
        self.cur += 1
        if self.imgrec is None:
            label, fname = self.imglist[key]
            return label, self.read_image(fname)
        header, payload = recordio.unpack(self.imgrec.read_idx(key))
        return (header.label if self.imglist is None else self.imglist[key][0]), payload

    def _sample_name(self):
        """Human-readable id of the sample just read (for decode errors)."""
        pos = (self.cur % self.num_image) - 1 if self.num_image else -1
        key = self.seq[pos] if self.seq is not None else pos
        if self.imglist is not None:
            return 'Broken image filename: {}'.format(self.imglist[key][1])
        return 'Broken image index: {}'.format(key)

    def imdecode(self, s):
        """Decode one sample's bytes (errors name the offending file / index)."""
        try:
            return imdecode(s)
        except Exception as err:      # pylint: disable=broad-except
            raise RuntimeError('{}, {}'.format(self._sample_name(), err))

    def read_image(self, fname):
        """Encoded bytes of ``fname`` relative to ``path_root``."""
        with open(os.path.join(self.path_root or '', fname), 'rb') as fh:
            return fh.read()

    def check_data_shape(self, data_shape):
        if len(data_shape) != 3:
            raise ValueError('data_shape should have length 3, with dimensions CxHxW')
        if data_shape[0] != 3:
            raise ValueError('This iterator expects inputs to have 3 channels.')

    def check_valid_image(self, data):
        if len(data[0].shape) == 0:
            raise RuntimeError('Data shape is wrong')

    def augmentation_transform(self, data):
        for aug in self.auglist:
            data = aug(data)
        return data

    def postprocess_data(self, datum):
        """HWC -> CHW."""
        return nd.transpose(datum, axes=(2, 0, 1))

    def _load_one(self, label, raw):
        """Decoded, validated and augmented ``(chw image, label)``; RuntimeError skips the sample."""
        img = self.imdecode(raw)
        self.check_valid_image(img)
        return self.postprocess_data(self.augmentation_transform(img)), label

    # ---------------------------------------------------------------- batches
    def _empty_label_batch(self):
        lab = nd.empty(self.provide_label[0][1])
        lab[:] = 0
        return lab

    def _batchify(self, batch_data, batch_label, start=0):
        """Fill rows ``start..`` of the batch; returns the number of filled rows."""
        filled = start
        try:
            while filled < self.batch_size:
                label, raw = self.next_sample()
                try:
                    datum, label = self._load_one(label, raw)
                except RuntimeError as err:
                    logging.debug('Invalid image, skipping:  %s', err)
                    continue
                batch_data[filled] = datum
                batch_label[filled] = label
                filled += 1
        except StopIteration:
            if filled == 0:
                raise
        return filled

    def next(self):
        if self._cache_data is not None:
            data, label, filled = self._cache_data, self._cache_label, self._cache_idx
        else:
            data = nd.zeros((self.batch_size,) + self.data_shape)
            label = self._empty_label_batch()
            filled = self._batchify(data, label)
        pad = self.batch_size - filled
        if pad:
            if self.last_batch_handle == 'discard':
                raise StopIteration
            if self.last_batch_handle == 'roll_over' and self._cache_data is None:
                self._cache_data, self._cache_label, self._cache_idx = data, label, filled
                raise StopIteration
            # 'pad' wraps to the start of the epoch; a roll_over carry is completed the same way
            self._batchify(data, label, filled)
            if self.last_batch_handle == 'pad':
                self._allow_read = False
            else:
                self._drop_carry()
        return mxio.DataBatch([data], [label], pad=pad)
