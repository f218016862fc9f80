"""Random, linear-algebra and image operators.

Parity: src/operator/random/sample_op.cc, multisample_op.cc, shuffle_op.cc;
src/operator/tensor/la_op.cc (_linalg_*); src/operator/image/*.cc (_image_*).
"""
import math

import numpy as np

import torch
import torch.nn.functional as F

from ..base import AsyncOpError, torch_dtype
from .registry import register
from .tensor import _dev

# ---------------------------------------------------------------------------
# random (symbol-callable; mx.nd.random has richer python wrappers)
# ---------------------------------------------------------------------------

_RP = {'shape': ('shape', ()), 'ctx': ('any', None), 'dtype': ('str', 'float32')}


def _s(shape):
    return tuple(shape) if shape else (1,)


def _check(cond, msg):
    # a sampler's parameter check runs inside the operator (reference: CHECKs in the sampler
    # kernels), so its failure is deferred to the next sync point like any execution error
    if not cond:
        raise AsyncOpError(msg)


@register('_random_uniform', aliases=('uniform', 'random_uniform'), arg_names=(),
          params=dict(low=('float', 0.0), high=('float', 1.0), **_RP))
def random_uniform(low=0.0, high=1.0, shape=(), ctx=None, dtype='float32'):
    _check(high >= low, 'Check failed: low <= high (uniform sampler: low=%s high=%s)' % (low, high))
    return torch.empty(_s(shape), dtype=torch_dtype(dtype if dtype != 'None' else 'float32'),
                       device=_dev(ctx)).uniform_(low, high)


@register('_random_normal', aliases=('normal', 'random_normal'), arg_names=(),
          params=dict(loc=('float', 0.0), scale=('float', 1.0), **_RP))
def random_normal(loc=0.0, scale=1.0, shape=(), ctx=None, dtype='float32'):
    _check(scale >= 0, 'Check failed: scale >= 0 (normal sampler: scale=%s)' % scale)
    return torch.empty(_s(shape), dtype=torch_dtype(dtype if dtype != 'None' else 'float32'),
                       device=_dev(ctx)).normal_(loc, scale)


@register('_random_gamma', arg_names=(), params=dict(alpha=('float', 1.0), beta=('float', 1.0), **_RP))
def random_gamma(alpha=1.0, beta=1.0, shape=(), ctx=None, dtype='float32'):
    _check(alpha > 0 and beta > 0, 'Check failed: alpha > 0 && beta > 0 (gamma sampler)')
    return (torch._standard_gamma(torch.full(_s(shape), alpha, device=_dev(ctx))) * beta).to(torch_dtype(dtype))


@register('_random_exponential', arg_names=(), params=dict(lam=('float', 1.0), **_RP))
def random_exponential(lam=1.0, shape=(), ctx=None, dtype='float32'):
    _check(lam > 0, 'Check failed: lambda > 0 (exponential sampler)')
    return torch.empty(_s(shape), device=_dev(ctx)).exponential_(lam).to(torch_dtype(dtype))


@register('_random_poisson', arg_names=(), params=dict(lam=('float', 1.0), **_RP))
def random_poisson(lam=1.0, shape=(), ctx=None, dtype='float32'):
    _check(lam >= 0, 'Check failed: lambda >= 0 (poisson sampler)')
    return torch.poisson(torch.full(_s(shape), lam, device=_dev(ctx))).to(torch_dtype(dtype))


@register('_random_randint', arg_names=(),
          params=dict(dict(low=('int', 0), high=('int', 1)), **dict(_RP, dtype=('str', 'int32'))))
def random_randint(low=0, high=1, shape=(), ctx=None, dtype='int32'):
    return torch.randint(low, high, _s(shape), device=_dev(ctx)).to(torch_dtype(dtype))


@register('_random_negative_binomial', arg_names=(), params=dict(k=('int', 1), p=('float', 1.0), **_RP))
def random_negative_binomial(k=1, p=1.0, shape=(), ctx=None, dtype='float32'):
    g = torch._standard_gamma(torch.full(_s(shape), float(k), device=_dev(ctx))) * ((1 - p) / p)
    return torch.poisson(g).to(torch_dtype(dtype))


@register('_random_generalized_negative_binomial', arg_names=(),
          params=dict(mu=('float', 1.0), alpha=('float', 1.0), **_RP))
def random_gen_neg_binomial(mu=1.0, alpha=1.0, shape=(), ctx=None, dtype='float32'):
    g = torch._standard_gamma(torch.full(_s(shape), 1.0 / alpha, device=_dev(ctx))) * (mu * alpha)
    return torch.poisson(g).to(torch_dtype(dtype))


def _like(f):
    def g(data, **kw):
        return f(shape=tuple(data.shape), ctx=None, dtype='float32', **kw).to(data.device, data.dtype)
    return g


register('_random_uniform_like', lambda data, low=0.0, high=1.0: torch.empty_like(data).uniform_(low, high),
         params={'low': ('float', 0.0), 'high': ('float', 1.0)})
register('_random_normal_like', lambda data, loc=0.0, scale=1.0: torch.empty_like(data).normal_(loc, scale),
         params={'loc': ('float', 0.0), 'scale': ('float', 1.0)})


def _sample_shape(p, shape):
    s = tuple(shape) if shape else ()
    return tuple(p.shape) + s, (1,) * len(s)


@register('_sample_uniform', aliases=('sample_uniform',), arg_names=('low', 'high'), params={'shape': ('shape', ()), 'dtype': ('str', 'None')})
def sample_uniform(low, high, shape=(), dtype='None'):
    full, ext = _sample_shape(low, shape)
    u = torch.rand(full, device=low.device, dtype=low.dtype)
    return low.reshape(tuple(low.shape) + ext) + (high - low).reshape(tuple(low.shape) + ext) * u


@register('_sample_normal', aliases=('sample_normal',), arg_names=('mu', 'sigma'), params={'shape': ('shape', ()), 'dtype': ('str', 'None')})
def sample_normal(mu, sigma, shape=(), dtype='None'):
    full, ext = _sample_shape(mu, shape)
    n = torch.randn(full, device=mu.device, dtype=mu.dtype)
    return mu.reshape(tuple(mu.shape) + ext) + sigma.reshape(tuple(mu.shape) + ext) * n


@register('_sample_multinomial', aliases=('sample_multinomial',), arg_names=('data',),
          num_outputs=lambda a: 2 if str(a.get('get_prob', False)) in ('True', 'true', '1') else 1,
          params={'shape': ('shape', ()), 'get_prob': ('bool', False), 'dtype': ('str', 'int32')})
def sample_multinomial(data, shape=(), get_prob=False, dtype='int32'):
    n = int(math.prod(shape)) if shape else 1
    flat = data.reshape(-1, data.shape[-1]).float()
    idx = torch.multinomial(flat, n, replacement=True)
    oshape = tuple(data.shape[:-1]) + (tuple(shape) if shape else ())
    out = idx.reshape(oshape if oshape else (1,)).to(torch_dtype(dtype))
    if get_prob:
        lp = torch.log(torch.gather(flat, 1, idx)).reshape(out.shape).to(data.dtype)
        return out, lp
    return out


@register('_shuffle', aliases=('shuffle',))
def shuffle(data):
    return data[torch.randperm(data.shape[0], device=data.device)]


# ---------------------------------------------------------------------------
# linalg (la_op.cc)
# ---------------------------------------------------------------------------

def _t(x, flag):
    return x.transpose(-1, -2) if flag else x


def _rows_to(x, axis):
    """Matrices whose rows lie on ``axis`` (reference la_op ``axis``): move that axis to -2."""
    a = axis % x.dim()
    return x if a == x.dim() - 2 else x.movedim(a, -2)


def _rows_back(y, axis, nd):
    a = axis % nd
    return y if a == nd - 2 else y.movedim(-2, a)


@register('_linalg_gemm', aliases=('linalg_gemm',), arg_names=('A', 'B', 'C'),
          params={'transpose_a': ('bool', False), 'transpose_b': ('bool', False), 'alpha': ('float', 1.0),
                  'beta': ('float', 1.0), 'axis': ('int', -2)})
def linalg_gemm(A, B, C, transpose_a=False, transpose_b=False, alpha=1.0, beta=1.0, axis=-2):
    nd = A.dim()
    A, B, C = _rows_to(A, axis), _rows_to(B, axis), _rows_to(C, axis)
    return _rows_back(alpha * torch.matmul(_t(A, transpose_a), _t(B, transpose_b)) + beta * C, axis, nd)


@register('_linalg_gemm2', aliases=('linalg_gemm2',), arg_names=('A', 'B'),
          params={'transpose_a': ('bool', False), 'transpose_b': ('bool', False), 'alpha': ('float', 1.0),
                  'axis': ('int', -2)})
def linalg_gemm2(A, B, transpose_a=False, transpose_b=False, alpha=1.0, axis=-2):
    nd = A.dim()
    A, B = _rows_to(A, axis), _rows_to(B, axis)
    return _rows_back(alpha * torch.matmul(_t(A, transpose_a), _t(B, transpose_b)), axis, nd)


@register('_linalg_potrf', aliases=('linalg_potrf',), params={'lower': ('bool', True)})
def linalg_potrf(A, lower=True):
    """Cholesky factor: lower L with A = L L^T, or (lower=False) upper U with A = U^T U."""
    return torch.linalg.cholesky(A, upper=not lower)


@register('_linalg_potri', aliases=('linalg_potri',), params={'lower': ('bool', True)})
def linalg_potri(A, lower=True):
    """Inverse of L L^T (or U^T U when lower=False) from its Cholesky factor."""
    return torch.cholesky_inverse(A, upper=not lower)


@register('_linalg_trmm', aliases=('linalg_trmm',), arg_names=('A', 'B'),
          params={'transpose': ('bool', False), 'rightside': ('bool', False), 'lower': ('bool', True),
                  'alpha': ('float', 1.0)})
def linalg_trmm(A, B, transpose=False, rightside=False, lower=True, alpha=1.0):
    T = torch.tril(A) if lower else torch.triu(A)
    T = _t(T, transpose)
    return alpha * (torch.matmul(B, T) if rightside else torch.matmul(T, B))


@register('_linalg_trsm', aliases=('linalg_trsm',), arg_names=('A', 'B'),
          params={'transpose': ('bool', False), 'rightside': ('bool', False), 'lower': ('bool', True),
                  'alpha': ('float', 1.0)})
def linalg_trsm(A, B, transpose=False, rightside=False, lower=True, alpha=1.0):
    up = not lower
    if transpose:
        A = A.transpose(-1, -2)
        up = not up
    return alpha * torch.linalg.solve_triangular(A, B, upper=up, left=not rightside)


@register('_linalg_sumlogdiag', aliases=('linalg_sumlogdiag',))
def linalg_sumlogdiag(A):
    return torch.log(torch.diagonal(A, dim1=-2, dim2=-1)).sum(-1)


@register('_linalg_syrk', aliases=('linalg_syrk',), params={'transpose': ('bool', False), 'alpha': ('float', 1.0)})
def linalg_syrk(A, transpose=False, alpha=1.0):
    return alpha * (torch.matmul(A.transpose(-1, -2), A) if transpose else torch.matmul(A, A.transpose(-1, -2)))


@register('_linalg_gelqf', aliases=('linalg_gelqf',), num_outputs=2)
def linalg_gelqf(A):
    q, r = torch.linalg.qr(A.transpose(-1, -2))
    return q.transpose(-1, -2), r.transpose(-1, -2)


@register('_linalg_syevd', aliases=('linalg_syevd',), num_outputs=2)
def linalg_syevd(A):
    """(U, L): rows of U are eigenvectors, each signed so its largest-magnitude entry (first on a tie)
    is positive -- the reference's deterministic sign rule (la_op-inl.h SyevdEigenVecSigns)."""
    w, v = torch.linalg.eigh(A)
    u = v.transpose(-1, -2)
    k = torch.argmax(u.abs(), dim=-1, keepdim=True)        # argmax returns the first maximum
    sign = torch.where(torch.gather(u, -1, k) < 0, -1.0, 1.0).to(u.dtype)
    return u * sign, w


@register('_linalg_inverse', aliases=('linalg_inverse',))
def linalg_inverse(A):
    return torch.linalg.inv(A)


@register('_linalg_det', aliases=('linalg_det',))
def linalg_det(A):
    return torch.linalg.det(A)


@register('_linalg_slogdet', aliases=('linalg_slogdet',), num_outputs=2)
def linalg_slogdet(A):
    s, l = torch.linalg.slogdet(A)
    return s, l


@register('_linalg_extractdiag', aliases=('linalg_extractdiag',), params={'offset': ('int', 0)})
def linalg_extractdiag(A, offset=0):
    return torch.diagonal(A, offset=offset, dim1=-2, dim2=-1).contiguous()


@register('_linalg_makediag', aliases=('linalg_makediag',), params={'offset': ('int', 0)})
def linalg_makediag(A, offset=0):
    return torch.diag_embed(A, offset=offset)


@register('_linalg_extracttrian', aliases=('linalg_extracttrian',), params={'offset': ('int', 0), 'lower': ('bool', True)})
def linalg_extracttrian(A, offset=0, lower=True):
    # a non-zero offset picks the side itself; ``lower`` only decides at offset 0
    # (reference src/operator/tensor/la_op.h: trian ops)
    n = A.shape[-1]
    lower = offset < 0 or (offset == 0 and lower)
    idx = torch.tril_indices(n, n, offset) if lower else torch.triu_indices(n, n, offset)
    return A[..., idx[0], idx[1]]


@register('_linalg_maketrian', aliases=('linalg_maketrian',), params={'offset': ('int', 0), 'lower': ('bool', True)})
def linalg_maketrian(A, offset=0, lower=True):
    m = A.shape[-1]
    n = int((math.sqrt(8 * m + 1) - 1) / 2) + abs(offset)
    lower = offset < 0 or (offset == 0 and lower)
    out = torch.zeros(A.shape[:-1] + (n, n), dtype=A.dtype, device=A.device)
    idx = torch.tril_indices(n, n, offset) if lower else torch.triu_indices(n, n, offset)
    out[..., idx[0], idx[1]] = A
    return out


# ---------------------------------------------------------------------------
# image ops (src/operator/image)
# ---------------------------------------------------------------------------

@register('_image_to_tensor', aliases=('to_tensor',))
def image_to_tensor(data):
    x = data.float() / 255.0
    if data.dim() == 3:
        return x.permute(2, 0, 1).contiguous()
    return x.permute(0, 3, 1, 2).contiguous()


def _image_error(msg):
    from ..base import MXNetError
    return MXNetError(msg)


@register('_image_normalize', aliases=('image_normalize',), params={'mean': ('floats', (0.0,)), 'std': ('floats', (1.0,))})
def image_normalize(data, mean=(0.0,), std=(1.0,)):
    """(x - mean) / std per channel of a CHW image or NCHW batch (src/operator/image/image_random-inl.h:
    1 or 3 channels; mean / std of length 1 or C)."""
    if data.dim() not in (3, 4):
        raise _image_error('Normalize: input must be a 3-D (CHW) or 4-D (NCHW) tensor, got shape %s'
                           % (tuple(data.shape),))
    c = data.shape[-3]
    if c not in (1, 3):
        raise _image_error('Normalize: expected 1 or 3 channels, got %d' % c)
    m = torch.tensor(list(mean) * (c if len(mean) == 1 else 1), dtype=data.dtype, device=data.device)[:c]
    s = torch.tensor(list(std) * (c if len(std) == 1 else 1), dtype=data.dtype, device=data.device)[:c]
    shape = (c, 1, 1)
    return (data - m.reshape(shape)) / s.reshape(shape)


def _resize_target(h, w, size, keep_ratio):
    """(width, height) of a resize (src/operator/image/resize-inl.h): ``size`` is (w, h) or one side;
    with ``keep_ratio`` a single size is the short side."""
    size = tuple(int(v) for v in size)
    if len(size) not in (1, 2) or any(v <= 0 for v in size):
        raise _image_error('Resize: size must be one or two positive integers, got %s' % (size,))
    if len(size) == 2:
        return size
    s = size[0]
    if not keep_ratio:
        return s, s
    return (s, int(h * s / w)) if h > w else (int(w * s / h), s)


@register('_image_resize', aliases=('image_resize',), params={'size': ('shape', ()), 'keep_ratio': ('bool', False),
                                                              'interp': ('int', 1)})
def image_resize(data, size=(), keep_ratio=False, interp=1):
    """Resize HWC images / NHWC batches.  Host tensors go through the same resampler as
    ``mx.image.imresize`` (bit-identical results); device tensors through bilinear / nearest
    interpolation on the GPU."""
    if data.dim() not in (3, 4):
        raise _image_error('Resize: input must be HWC or NHWC, got shape %s' % (tuple(data.shape),))
    w, h = _resize_target(data.shape[-3], data.shape[-2], size, keep_ratio)
    hwc = data.dim() == 3
    if data.device.type == 'cpu' and not data.requires_grad:
        from ..image.image import _resize_np
        imgs = [data] if hwc else list(data)
        outs = [torch.from_numpy(np.ascontiguousarray(_resize_np(i.numpy(), w, h, interp))) for i in imgs]
        return outs[0] if hwc else torch.stack(outs)
    x = data.permute(2, 0, 1).unsqueeze(0) if hwc else data.permute(0, 3, 1, 2)
    mode = 'nearest' if interp == 0 else 'bilinear'
    y = F.interpolate(x.float(), size=(h, w), mode=mode, align_corners=False if mode == 'bilinear' else None)
    y = y.round().clamp(0, 255) if not data.is_floating_point() else y
    y = y.to(data.dtype)
    return y[0].permute(1, 2, 0) if hwc else y.permute(0, 2, 3, 1)


@register('_image_crop', aliases=('image_crop',), params={'x': ('int', 0), 'y': ('int', 0), 'width': ('int', 1),
                                                          'height': ('int', 1)})
def image_crop(data, x=0, y=0, width=1, height=1):
    if data.dim() not in (3, 4):
        raise _image_error('Crop: input must be HWC or NHWC, got shape %s' % (tuple(data.shape),))
    H, W = data.shape[-3], data.shape[-2]
    if width <= 0 or height <= 0 or x < 0 or y < 0 or x + width > W or y + height > H:
        raise _image_error('Crop: window (x=%d, y=%d, width=%d, height=%d) is outside the %dx%d image'
                           % (x, y, width, height, W, H))
    if data.dim() == 3:
        return data[y:y + height, x:x + width].contiguous()
    return data[:, y:y + height, x:x + width].contiguous()


@register('_image_flip_left_right', aliases=('flip_left_right',))
def image_flip_lr(data):
    return torch.flip(data, dims=[-2])


@register('_image_flip_top_bottom', aliases=('flip_top_bottom',))
def image_flip_tb(data):
    return torch.flip(data, dims=[-3])


@register('_image_random_flip_left_right')
def image_random_flip_lr(data):
    return torch.flip(data, dims=[-2]) if torch.rand(()) < 0.5 else data.clone()


@register('_image_random_flip_top_bottom')
def image_random_flip_tb(data):
    return torch.flip(data, dims=[-3]) if torch.rand(()) < 0.5 else data.clone()


def _gray(x):
    w = torch.tensor([0.299, 0.587, 0.114], dtype=torch.float32, device=x.device)
    return (x.float() * w).sum(-1, keepdim=True)


@register('_image_adjust_lighting', params={'alpha': ('floats', (0.0, 0.0, 0.0))})
def image_adjust_lighting(data, alpha=(0.0, 0.0, 0.0)):
    eigval = torch.tensor([55.46, 4.794, 1.148])
    eigvec = torch.tensor([[-0.5675, 0.7192, 0.4009], [-0.5808, -0.0045, -0.8140], [-0.5836, -0.6948, 0.4203]])
    rgb = (eigvec * torch.tensor(alpha) * eigval).sum(1).to(data.device)
    return (data.float() + rgb).to(data.dtype)


@register('_image_random_brightness', params={'min_factor': ('float', 1.0), 'max_factor': ('float', 1.0)})
def image_random_brightness(data, min_factor=1.0, max_factor=1.0):
    a = float(torch.empty(()).uniform_(min_factor, max_factor))
    return (data.float() * a).to(data.dtype)


@register('_image_random_contrast', params={'min_factor': ('float', 1.0), 'max_factor': ('float', 1.0)})
def image_random_contrast(data, min_factor=1.0, max_factor=1.0):
    a = float(torch.empty(()).uniform_(min_factor, max_factor))
    m = _gray(data).mean()
    return (data.float() * a + m * (1 - a)).to(data.dtype)


@register('_image_random_saturation', params={'min_factor': ('float', 1.0), 'max_factor': ('float', 1.0)})
def image_random_saturation(data, min_factor=1.0, max_factor=1.0):
    a = float(torch.empty(()).uniform_(min_factor, max_factor))
    g = _gray(data)
    return (data.float() * a + g * (1 - a)).to(data.dtype)


def _hue_matrix(alpha, device):
    u, w = math.cos(alpha * math.pi), math.sin(alpha * math.pi)
    tyiq = torch.tensor([[0.299, 0.587, 0.114], [0.596, -0.274, -0.321], [0.211, -0.523, 0.311]])
    ityiq = torch.tensor([[1.0, 0.956, 0.621], [1.0, -0.272, -0.647], [1.0, -1.107, 1.705]])
    bt = torch.tensor([[1.0, 0.0, 0.0], [0.0, u, -w], [0.0, w, u]])
    return (ityiq @ bt @ tyiq).t().to(device)


@register('_image_random_hue', params={'min_factor': ('float', 0.0), 'max_factor': ('float', 0.0)})
def image_random_hue(data, min_factor=0.0, max_factor=0.0):
    a = float(torch.empty(()).uniform_(min_factor, max_factor))
    return (data.float() @ _hue_matrix(a, data.device)).to(data.dtype)


@register('_image_random_color_jitter', params={'brightness': ('float', 0.0), 'contrast': ('float', 0.0),
                                                'saturation': ('float', 0.0), 'hue': ('float', 0.0)})
def image_random_color_jitter(data, brightness=0.0, contrast=0.0, saturation=0.0, hue=0.0):
    ops = []
    if brightness > 0:
        ops.append(lambda x: image_random_brightness(x, 1 - brightness, 1 + brightness))
    if contrast > 0:
        ops.append(lambda x: image_random_contrast(x, 1 - contrast, 1 + contrast))
    if saturation > 0:
        ops.append(lambda x: image_random_saturation(x, 1 - saturation, 1 + saturation))
    if hue > 0:
        ops.append(lambda x: image_random_hue(x, -hue, hue))
    for i in torch.randperm(len(ops)).tolist():
        data = ops[i](data)
    return data


@register('_image_random_lighting', params={'alpha_std': ('float', 0.05)})
def image_random_lighting(data, alpha_std=0.05):
    alpha = torch.randn(3) * alpha_std
    return image_adjust_lighting(data, tuple(alpha.tolist()))
