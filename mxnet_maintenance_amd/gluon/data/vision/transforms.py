"""Vision transforms (parity: python/mxnet/gluon/data/vision/transforms.py).

Transforms consume HWC images (uint8 or float) like the reference; ``ToTensor``
switches to CHW float in [0, 1].  Hybridizable ones are HybridBlocks over the
``_image_*`` operators so they can be fused into a CachedOp.
"""
import random

import numpy as np

from ...block import Block, HybridBlock
from ...nn import Sequential, HybridSequential
from .... import image
from .... import ndarray as nd

__all__ = ['Compose', 'HybridCompose', 'Cast', 'ToTensor', 'Normalize', 'Rotate', 'RandomRotation',
           'RandomResizedCrop', 'CropResize', 'CenterCrop', 'Resize', 'RandomFlipLeftRight', 'RandomFlipTopBottom',
           'RandomBrightness', 'RandomContrast', 'RandomSaturation', 'RandomHue', 'RandomColorJitter',
           'RandomLighting', 'RandomApply', 'HybridRandomApply', 'RandomCrop']


class Compose(Sequential):
    """Chain transforms; consecutive hybridizable ones are grouped into a hybridized HybridSequential."""

    def __init__(self, transforms):
        super().__init__()
        transforms.append(None)
        hybrid = []
        for i in transforms:
            if isinstance(i, HybridBlock):
                hybrid.append(i)
                continue
            elif len(hybrid) == 1:
                self.add(hybrid[0])
                hybrid = []
            elif len(hybrid) > 1:
                hblock = HybridSequential()
                for j in hybrid:
                    hblock.add(j)
                hblock.hybridize()
                self.add(hblock)
                hybrid = []
            if i is not None:
                self.add(i)


class HybridCompose(HybridSequential):
    def __init__(self, transforms):
        super().__init__()
        for t in transforms:
            self.add(t)


class Cast(HybridBlock):
    def __init__(self, dtype='float32'):
        super().__init__()
        self._dtype = dtype

    def hybrid_forward(self, F, x):
        return F.cast(x, self._dtype)


class ToTensor(HybridBlock):
    """HWC [0,255] -> CHW float32 [0,1] (also NHWC -> NCHW)."""

    def hybrid_forward(self, F, x):
        return F.image.to_tensor(x)


class Normalize(HybridBlock):
    """Per-channel ``(x - mean) / std`` on CHW / NCHW tensors."""

    def __init__(self, mean=0.0, std=1.0):
        super().__init__()
        self._mean = mean
        self._std = std

    def hybrid_forward(self, F, x):
        return F.image.normalize(x, self._mean, self._std)


class Rotate(Block):
    def __init__(self, rotation_degrees, zoom_in=False, zoom_out=False):
        super().__init__()
        self._args = (rotation_degrees, zoom_in, zoom_out)

    def forward(self, x):
        if x.dtype != np.float32 and str(x.dtype) != 'float32':
            raise TypeError('This transformation only supports float32. Consider calling it after ToTensor')
        return image.imrotate(x, *self._args)


class RandomRotation(Block):
    def __init__(self, angle_limits, zoom_in=False, zoom_out=False, rotate_with_proba=1.0):
        super().__init__()
        lower, upper = angle_limits
        if lower >= upper:
            raise ValueError('`angle_limits` must be an ordered tuple')
        if rotate_with_proba < 0 or rotate_with_proba > 1:
            raise ValueError('Probability of rotating the image should be between 0 and 1')
        self._args = (angle_limits, zoom_in, zoom_out)
        self._rotate_with_proba = rotate_with_proba

    def forward(self, x):
        if np.random.random() > self._rotate_with_proba:
            return x
        return image.random_rotate(x, *self._args)


class RandomResizedCrop(Block):
    def __init__(self, size, scale=(0.08, 1.0), ratio=(3.0 / 4.0, 4.0 / 3.0), interpolation=1):
        super().__init__()
        if isinstance(size, int):
            size = (size, size)
        self._args = (size, scale, ratio, interpolation)

    def forward(self, x):
        return image.random_size_crop(x, *self._args)[0]


class CropResize(HybridBlock):
    def __init__(self, x, y, width, height, size=None, interpolation=None):
        super().__init__()
        self._x, self._y, self._width, self._height = x, y, width, height
        self._size = (size, size) if isinstance(size, int) else size
        self._interpolation = interpolation

    def hybrid_forward(self, F, x):
        out = F.image.crop(x, self._x, self._y, self._width, self._height)
        if self._size:
            out = F.image.resize(out, self._size, False, self._interpolation if self._interpolation is not None
                                 else 1)
        return out


class CenterCrop(Block):
    def __init__(self, size, interpolation=1):
        super().__init__()
        if isinstance(size, int):
            size = (size, size)
        self._args = (size, interpolation)

    def forward(self, x):
        return image.center_crop(x, *self._args)[0]


class RandomCrop(Block):
    """Random crop of ``size`` after optional zero padding."""

    def __init__(self, size, pad=None, interpolation=1):
        super().__init__()
        if isinstance(size, int):
            size = (size, size)
        self._args = (size, interpolation)
        self._pad = pad

    def forward(self, x):
        if self._pad:
            p = self._pad if isinstance(self._pad, (tuple, list)) else (self._pad,) * 4
            x = image.copyMakeBorder(x, p[0], p[1], p[2], p[3], 0)
        return image.random_crop(x, *self._args)[0]


class Resize(HybridBlock):
    def __init__(self, size, keep_ratio=False, interpolation=1):
        super().__init__()
        self._keep = keep_ratio
        self._size = size
        self._interpolation = interpolation

    def hybrid_forward(self, F, x):
        if isinstance(self._size, int) or len(self._size) == 1:
            s = self._size if isinstance(self._size, int) else self._size[0]
            if self._keep:
                h, w = x.shape[-3], x.shape[-2]
                if h > w:
                    size = (s, int(h * s / w))
                else:
                    size = (int(w * s / h), s)
            else:
                size = (s, s)
        else:
            size = tuple(self._size)
        return F.image.resize(x, size, False, self._interpolation)


class RandomFlipLeftRight(HybridBlock):
    def hybrid_forward(self, F, x):
        return F.image.random_flip_left_right(x)


class RandomFlipTopBottom(HybridBlock):
    def hybrid_forward(self, F, x):
        return F.image.random_flip_top_bottom(x)


class RandomBrightness(HybridBlock):
    def __init__(self, brightness):
        super().__init__()
        self._args = (max(0, 1 - brightness), 1 + brightness)

    def hybrid_forward(self, F, x):
        return F.image.random_brightness(x, *self._args)


class RandomContrast(HybridBlock):
    def __init__(self, contrast):
        super().__init__()
        self._args = (max(0, 1 - contrast), 1 + contrast)

    def hybrid_forward(self, F, x):
        return F.image.random_contrast(x, *self._args)


class RandomSaturation(HybridBlock):
    def __init__(self, saturation):
        super().__init__()
        self._args = (max(0, 1 - saturation), 1 + saturation)

    def hybrid_forward(self, F, x):
        return F.image.random_saturation(x, *self._args)


class RandomHue(HybridBlock):
    def __init__(self, hue):
        super().__init__()
        self._args = (max(0, 1 - hue), 1 + hue)

    def hybrid_forward(self, F, x):
        return F.image.random_hue(x, -abs(self._args[1] - 1), abs(self._args[1] - 1))


class RandomColorJitter(HybridBlock):
    def __init__(self, brightness=0, contrast=0, saturation=0, hue=0):
        super().__init__()
        self._args = (brightness, contrast, saturation, hue)

    def hybrid_forward(self, F, x):
        return F.image.random_color_jitter(x, *self._args)


class RandomLighting(HybridBlock):
    def __init__(self, alpha):
        super().__init__()
        self._alpha = alpha

    def hybrid_forward(self, F, x):
        return F.image.random_lighting(x, self._alpha)


class RandomApply(Sequential):
    """Apply the wrapped transforms with probability ``p``."""

    def __init__(self, transforms, p=0.5):
        super().__init__()
        self.transforms = transforms
        self.p = p

    def forward(self, x):
        if self.p < random.random():
            return x
        return self.transforms(x)


class HybridRandomApply(HybridSequential):
    def __init__(self, transforms, p=0.5):
        super().__init__()
        self.transforms = transforms
        self.p = p

    def hybrid_forward(self, F, x):
        if self.p < random.random():
            return x
        return self.transforms(x)
