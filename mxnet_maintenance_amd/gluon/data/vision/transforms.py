"""Vision transforms (API parity: python/mxnet/gluon/data/vision/transforms.py).

Images are HWC (uint8 or float) as in the reference; ``ToTensor`` switches to
CHW float in [0, 1].  Most transforms are a single ``_image_*`` operator: they
derive from ``_ImageOp`` (a HybridBlock that calls ``F.image.<_OP>(x, *args)``)
and only compute their operator arguments.  Geometric transforms that need
host-side randomness (rotation, random crops) are plain Blocks over
``mxnet.image`` helpers.  ``Compose`` fuses every run of consecutive
hybridizable transforms into one hybridized ``HybridSequential``.
"""
import itertools
import random

import numpy as np

from ...block import Block, HybridBlock
from ...nn import Sequential, HybridSequential
from .... import image

__all__ = ['Compose', 'HybridCompose', 'Cast', 'ToTensor', 'Normalize', 'Rotate', 'RandomRotation',
           'RandomResizedCrop', 'CropResize', 'CenterCrop', 'Resize', 'RandomFlipLeftRight', 'RandomFlipTopBottom',
           'RandomBrightness', 'RandomContrast', 'RandomSaturation', 'RandomHue', 'RandomColorJitter',
           'RandomLighting', 'RandomApply', 'HybridRandomApply', 'RandomCrop']


def _pair(size):
    return (size, size) if isinstance(size, int) else size


class Compose(Sequential):
    """Apply ``transforms`` in order; runs of >= 2 hybridizable transforms become one hybridized block."""

    def __init__(self, transforms):
        super().__init__()
        for hybrid, run in itertools.groupby(transforms, key=lambda t: isinstance(t, HybridBlock)):
            run = list(run)
            if hybrid and len(run) > 1:
                fused = HybridSequential()
                fused.add(*run)
                fused.hybridize()
                self.add(fused)
            else:
                self.add(*run)


class HybridCompose(HybridSequential):
    """Hybridizable chain of hybridizable transforms."""

    def __init__(self, transforms):
        super().__init__()
        self.add(*transforms)


class _ImageOp(HybridBlock):
    """``x -> F.image.<_OP>(x, *self._args)``."""

    _OP = None

    def __init__(self, *args):
        super().__init__()
        self._args = args

    def hybrid_forward(self, F, x):
        return getattr(F.image, self._OP)(x, *self._args)


class Cast(HybridBlock):
    def __init__(self, dtype='float32'):
        super().__init__()
        self._dtype = dtype

    def hybrid_forward(self, F, x):
        return F.cast(x, self._dtype)


class ToTensor(_ImageOp):
    """HWC [0, 255] -> CHW float32 [0, 1] (NHWC -> NCHW for batches)."""
    _OP = 'to_tensor'


class Normalize(_ImageOp):
    """Per-channel ``(x - mean) / std`` on CHW / NCHW tensors."""
    _OP = 'normalize'

    def __init__(self, mean=0.0, std=1.0):
        super().__init__(mean, std)


class RandomFlipLeftRight(_ImageOp):
    _OP = 'random_flip_left_right'


class RandomFlipTopBottom(_ImageOp):
    _OP = 'random_flip_top_bottom'


class _RandomFactor(_ImageOp):
    """Jitter by a factor drawn from [max(0, 1 - amount), 1 + amount]."""

    def __init__(self, amount):
        super().__init__(max(0, 1 - amount), 1 + amount)


class RandomBrightness(_RandomFactor):
    _OP = 'random_brightness'


class RandomContrast(_RandomFactor):
    _OP = 'random_contrast'


class RandomSaturation(_RandomFactor):
    _OP = 'random_saturation'


class RandomHue(_ImageOp):
    """Hue rotation by a fraction drawn from [-hue, hue]."""
    _OP = 'random_hue'

    def __init__(self, hue):
        super().__init__(-abs(hue), abs(hue))


class RandomColorJitter(_ImageOp):
    _OP = 'random_color_jitter'

    def __init__(self, brightness=0, contrast=0, saturation=0, hue=0):
        super().__init__(brightness, contrast, saturation, hue)


class RandomLighting(_ImageOp):
    """AlexNet-style PCA lighting noise with standard deviation ``alpha``."""
    _OP = 'random_lighting'

    def __init__(self, alpha):
        super().__init__(alpha)


class CropResize(HybridBlock):
    """Fixed crop ``(x, y, width, height)``, optionally resized to ``size``."""

    def __init__(self, x, y, width, height, size=None, interpolation=None):
        super().__init__()
        self._box = (x, y, width, height)
        self._size = _pair(size) if size else None
        self._interpolation = 1 if interpolation is None else interpolation

    def hybrid_forward(self, F, x):
        out = F.image.crop(x, *self._box)
        return F.image.resize(out, size=self._size, keep_ratio=False, interp=self._interpolation) if self._size \
            else out


class Resize(HybridBlock):
    """Resize to ``size`` (w, h), or the short side to ``size`` with ``keep_ratio``."""

    def __init__(self, size, keep_ratio=False, interpolation=1):
        super().__init__()
        self._size = size
        self._keep = keep_ratio
        self._interpolation = interpolation

    def hybrid_forward(self, F, x):
        # the operator sizes the target from the input (keep_ratio), so this hybridizes
        size = (self._size,) if isinstance(self._size, int) else tuple(self._size)
        return F.image.resize(x, size=size, keep_ratio=self._keep, interp=self._interpolation)


class Rotate(Block):
    """Rotate a float32 image by a fixed angle (degrees)."""

    def __init__(self, rotation_degrees, zoom_in=False, zoom_out=False):
        super().__init__()
        self._args = (rotation_degrees, zoom_in, zoom_out)

    def forward(self, x):
        if str(x.dtype) not in ('float32', "<class 'numpy.float32'>") and x.dtype != np.float32:
            raise TypeError('This transformation only supports float32. Consider calling it after ToTensor')
        return image.imrotate(x, *self._args)


class RandomRotation(Block):
    """Rotate by an angle drawn from ``angle_limits`` with probability ``rotate_with_proba``."""

    def __init__(self, angle_limits, zoom_in=False, zoom_out=False, rotate_with_proba=1.0):
        super().__init__()
        lo, hi = angle_limits
        if lo >= hi:
            raise ValueError('`angle_limits` must be an ordered tuple')
        if not 0 <= rotate_with_proba <= 1:
            raise ValueError('Probability of rotating the image should be between 0 and 1')
        self._args = (angle_limits, zoom_in, zoom_out)
        self._p = rotate_with_proba

    def forward(self, x):
        return image.random_rotate(x, *self._args) if np.random.random() <= self._p else x


class RandomResizedCrop(Block):
    """Crop a random area / aspect-ratio window and resize it to ``size``."""

    def __init__(self, size, scale=(0.08, 1.0), ratio=(3.0 / 4.0, 4.0 / 3.0), interpolation=1):
        super().__init__()
        self._args = (_pair(size), scale, ratio, interpolation)

    def forward(self, x):
        return image.random_size_crop(x, *self._args)[0]


class CenterCrop(Block):
    def __init__(self, size, interpolation=1):
        super().__init__()
        self._args = (_pair(size), interpolation)

    def forward(self, x):
        return image.center_crop(x, *self._args)[0]


class RandomCrop(Block):
    """Random ``size`` crop, after zero padding of ``pad`` pixels (int, or (top, bottom, left, right))."""

    def __init__(self, size, pad=None, interpolation=1):
        super().__init__()
        self._args = (_pair(size), interpolation)
        self._pad = None if not pad else (tuple(pad) if isinstance(pad, (tuple, list)) else (pad,) * 4)

    def forward(self, x):
        if self._pad:
            x = image.copyMakeBorder(x, *self._pad, 0)
        return image.random_crop(x, *self._args)[0]


class RandomApply(Sequential):
    """Apply ``transforms`` with probability ``p``."""

    def __init__(self, transforms, p=0.5):
        super().__init__()
        self.transforms = transforms
        self.p = p

    def forward(self, x):
        return self.transforms(x) if random.random() <= self.p else x


class HybridRandomApply(HybridSequential):
    def __init__(self, transforms, p=0.5):
        super().__init__()
        self.transforms = transforms
        self.p = p

    def hybrid_forward(self, F, x):
        return self.transforms(x) if random.random() <= self.p else x
