"""Optimizer update operators (in-place on weight and state tensors).

Parity: src/operator/optimizer_op-inl.h (SGDKernel, SGDMomKernel, MP variants,
NAGMomKernel, AdamUpdateKernel, RMSPropUpdateKernel, RMSPropAlexUpdateKernel,
FtrlUpdateKernel, FTMLKernel, SignSGDKernel, SignumKernel, LambUpdatePhase*),
src/operator/contrib/{adamw,multi_lamb,multi_lars,multi_sum_sq,all_finite,
reset_arrays,preloaded_multi_sgd}*.

Each function updates its state tensors in place and writes the new weight in
place into ``weight`` (the reference ops are always called with out=weight).
On the GPU the ``multi_*`` forms run as a single fused multi-tensor HIP kernel
(ops/kernels.py: ``multi_sgd_mom``); the single-tensor forms use torch
in-place arithmetic which is already one pass over HBM per state.
"""
import math

import torch

from .registry import register
from . import kernels as _K

_COMMON = {'lr': ('float', 0.01), 'wd': ('float', 0.0), 'rescale_grad': ('float', 1.0),
           'clip_gradient': ('float', -1.0)}


def _prep(grad, rescale, clip):
    g = grad.float() * rescale if rescale != 1.0 else grad.float()
    if clip is not None and clip >= 0:
        g = torch.clamp(g, -clip, clip)
    return g


@torch.no_grad()
def _sgd(weight, grad, lr, wd, rescale_grad, clip_gradient, w32=None):
    w = weight if w32 is None else w32
    g = _prep(grad, rescale_grad, clip_gradient)
    w.mul_(1 - lr * wd).add_(g.to(w.dtype), alpha=-lr)
    if w32 is not None:
        weight.copy_(w32)
    return weight


@register('sgd_update', arg_names=('weight', 'grad'), params=dict(_COMMON, lazy_update=('bool', True)))
def sgd_update(weight, grad, lr=0.01, wd=0.0, rescale_grad=1.0, clip_gradient=-1.0, lazy_update=True):
    return _sgd(weight, grad, lr, wd, rescale_grad, clip_gradient)


@torch.no_grad()
def _sgd_mom(weight, grad, mom, lr, momentum, wd, rescale_grad, clip_gradient, w32=None):
    w = weight if w32 is None else w32
    g = _prep(grad, rescale_grad, clip_gradient)
    mom.mul_(momentum).add_((g + wd * w).to(mom.dtype), alpha=-lr)
    w.add_(mom)
    if w32 is not None:
        weight.copy_(w32)
    return weight


@register('sgd_mom_update', arg_names=('weight', 'grad', 'mom'),
          params=dict(_COMMON, momentum=('float', 0.0), lazy_update=('bool', True)))
def sgd_mom_update(weight, grad, mom, lr=0.01, momentum=0.0, wd=0.0, rescale_grad=1.0, clip_gradient=-1.0,
                   lazy_update=True):
    return _sgd_mom(weight, grad, mom, lr, momentum, wd, rescale_grad, clip_gradient)


@register('mp_sgd_update', arg_names=('weight', 'grad', 'weight32'), params=dict(_COMMON, lazy_update=('bool', True)))
def mp_sgd_update(weight, grad, weight32, lr=0.01, wd=0.0, rescale_grad=1.0, clip_gradient=-1.0, lazy_update=True):
    return _sgd(weight, grad, lr, wd, rescale_grad, clip_gradient, w32=weight32)


@register('mp_sgd_mom_update', arg_names=('weight', 'grad', 'mom', 'weight32'),
          params=dict(_COMMON, momentum=('float', 0.0), lazy_update=('bool', True)))
def mp_sgd_mom_update(weight, grad, mom, weight32, lr=0.01, momentum=0.0, wd=0.0, rescale_grad=1.0,
                      clip_gradient=-1.0, lazy_update=True):
    return _sgd_mom(weight, grad, mom, lr, momentum, wd, rescale_grad, clip_gradient, w32=weight32)


@torch.no_grad()
def _nag(weight, grad, mom, lr, momentum, wd, rescale_grad, clip_gradient, w32=None):
    w = weight if w32 is None else w32
    g = _prep(grad, rescale_grad, clip_gradient) + wd * w.float()
    mom.mul_(momentum)
    new_w = w.float() - mom.float() + (momentum + 1) * (mom.float() - lr * g)
    mom.sub_((lr * g).to(mom.dtype))
    w.copy_(new_w)
    if w32 is not None:
        weight.copy_(w32)
    return weight


@register('nag_mom_update', arg_names=('weight', 'grad', 'mom'), params=dict(_COMMON, momentum=('float', 0.0)))
def nag_mom_update(weight, grad, mom, lr=0.01, momentum=0.0, wd=0.0, rescale_grad=1.0, clip_gradient=-1.0):
    return _nag(weight, grad, mom, lr, momentum, wd, rescale_grad, clip_gradient)


@register('mp_nag_mom_update', arg_names=('weight', 'grad', 'mom', 'weight32'),
          params=dict(_COMMON, momentum=('float', 0.0)))
def mp_nag_mom_update(weight, grad, mom, weight32, lr=0.01, momentum=0.0, wd=0.0, rescale_grad=1.0,
                      clip_gradient=-1.0):
    return _nag(weight, grad, mom, lr, momentum, wd, rescale_grad, clip_gradient, w32=weight32)


_ADAM = dict(_COMMON, beta1=('float', 0.9), beta2=('float', 0.999), epsilon=('float', 1e-8),
             lazy_update=('bool', True))


@register('adam_update', arg_names=('weight', 'grad', 'mean', 'var'), params=_ADAM)
@torch.no_grad()
def adam_update(weight, grad, mean, var, lr=0.01, beta1=0.9, beta2=0.999, epsilon=1e-8, wd=0.0,
                rescale_grad=1.0, clip_gradient=-1.0, lazy_update=True):
    g = grad.float() * rescale_grad + wd * weight.float()
    if clip_gradient >= 0:
        g = torch.clamp(g, -clip_gradient, clip_gradient)
    mean.mul_(beta1).add_(g.to(mean.dtype), alpha=1 - beta1)
    var.mul_(beta2).addcmul_(g.to(var.dtype), g.to(var.dtype), value=1 - beta2)
    weight.sub_((lr * mean.float() / (torch.sqrt(var.float()) + epsilon)).to(weight.dtype))
    return weight


_ADAMW = {'lr': ('float', 0.001), 'beta1': ('float', 0.9), 'beta2': ('float', 0.999),
          'epsilon': ('float', 1e-8), 'wd': ('float', 0.0), 'eta': ('float', 1.0),
          'clip_gradient': ('float', -1.0)}


@torch.no_grad()
def _adamw(weight, grad, mean, var, rescale_grad, lr, beta1, beta2, epsilon, wd, eta, clip_gradient, w32=None):
    w = weight if w32 is None else w32
    rs = float(rescale_grad.reshape(-1)[0]) if torch.is_tensor(rescale_grad) else rescale_grad
    if not math.isfinite(rs) or rs == 0:      # skipped update (adamw-inl.h: non-finite or zero scale)
        return weight
    g = grad.float() * rs
    if clip_gradient >= 0:
        g = torch.clamp(g, -clip_gradient, clip_gradient)
    mean.mul_(beta1).add_(g, alpha=1 - beta1)
    var.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    w.sub_(eta * (lr * mean / (torch.sqrt(var) + epsilon) + wd * w))
    if w32 is not None:
        weight.copy_(w32)
    return weight


@register('_adamw_update', aliases=('_contrib_adamw_update', 'adamw_update'),
          arg_names=('weight', 'grad', 'mean', 'var', 'rescale_grad'), params=_ADAMW)
def adamw_update(weight, grad, mean, var, rescale_grad, lr=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8,
                 wd=0.0, eta=1.0, clip_gradient=-1.0):
    return _adamw(weight, grad, mean, var, rescale_grad, lr, beta1, beta2, epsilon, wd, eta, clip_gradient)


@register('_mp_adamw_update', aliases=('_contrib_mp_adamw_update', 'mp_adamw_update'),
          arg_names=('weight', 'grad', 'mean', 'var', 'weight32', 'rescale_grad'), params=_ADAMW)
def mp_adamw_update(weight, grad, mean, var, weight32, rescale_grad, lr=0.001, beta1=0.9, beta2=0.999,
                    epsilon=1e-8, wd=0.0, eta=1.0, clip_gradient=-1.0):
    return _adamw(weight, grad, mean, var, rescale_grad, lr, beta1, beta2, epsilon, wd, eta, clip_gradient,
                  w32=weight32)


@register('rmsprop_update', arg_names=('weight', 'grad', 'n'),
          params=dict(_COMMON, gamma1=('float', 0.95), epsilon=('float', 1e-8), clip_weights=('float', -1.0)))
@torch.no_grad()
def rmsprop_update(weight, grad, n, lr=0.01, gamma1=0.95, epsilon=1e-8, wd=0.0, rescale_grad=1.0,
                   clip_gradient=-1.0, clip_weights=-1.0):
    g = grad.float() * rescale_grad + wd * weight.float()
    if clip_gradient >= 0:
        g = torch.clamp(g, -clip_gradient, clip_gradient)
    n.mul_(gamma1).addcmul_(g, g, value=1 - gamma1)
    w = weight.float() - lr * g / torch.sqrt(n.float() + epsilon)
    if clip_weights >= 0:
        w = torch.clamp(w, -clip_weights, clip_weights)
    weight.copy_(w)
    return weight


@register('rmspropalex_update', arg_names=('weight', 'grad', 'n', 'g', 'delta'),
          params=dict(_COMMON, gamma1=('float', 0.95), gamma2=('float', 0.9), epsilon=('float', 1e-8),
                      clip_weights=('float', -1.0)))
@torch.no_grad()
def rmspropalex_update(weight, grad, n, g, delta, lr=0.01, gamma1=0.95, gamma2=0.9, epsilon=1e-8, wd=0.0,
                       rescale_grad=1.0, clip_gradient=-1.0, clip_weights=-1.0):
    gr = grad.float() * rescale_grad + wd * weight.float()
    if clip_gradient >= 0:
        gr = torch.clamp(gr, -clip_gradient, clip_gradient)
    n.mul_(gamma1).addcmul_(gr, gr, value=1 - gamma1)
    g.mul_(gamma1).add_(gr, alpha=1 - gamma1)
    delta.mul_(gamma2).sub_(lr * gr / torch.sqrt(n - g * g + epsilon))
    w = weight + delta
    if clip_weights >= 0:
        w = torch.clamp(w, -clip_weights, clip_weights)
    weight.copy_(w)
    return weight


@register('ftrl_update', arg_names=('weight', 'grad', 'z', 'n'),
          params=dict(_COMMON, lamda1=('float', 0.01), beta=('float', 1.0)))
@torch.no_grad()
def ftrl_update(weight, grad, z, n, lr=0.01, lamda1=0.01, beta=1.0, wd=0.0, rescale_grad=1.0,
                clip_gradient=-1.0):
    g = _prep(grad, rescale_grad, clip_gradient)
    z.add_(g - (torch.sqrt(n + g * g) - torch.sqrt(n)) * weight / lr)
    n.add_(g * g)
    w = (torch.sign(z) * lamda1 - z) / ((beta + torch.sqrt(n)) / lr + wd) * (torch.abs(z) > lamda1)
    weight.copy_(w)
    return weight


@register('ftml_update', arg_names=('weight', 'grad', 'd', 'v', 'z'),
          params={'lr': ('float', 0.0025), 'beta1': ('float', 0.6), 'beta2': ('float', 0.999),
                  'epsilon': ('float', 1e-8), 't': ('int', 1), 'wd': ('float', 0.0),
                  'rescale_grad': ('float', 1.0), 'clip_grad': ('float', -1.0)})
@torch.no_grad()
def ftml_update(weight, grad, d, v, z, lr=0.0025, beta1=0.6, beta2=0.999, epsilon=1e-8, t=1, wd=0.0,
                rescale_grad=1.0, clip_grad=-1.0):
    g = grad * rescale_grad + wd * weight
    if clip_grad >= 0:
        g = torch.clamp(g, -clip_grad, clip_grad)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    d_t = (1 - beta1 ** t) / lr * (torch.sqrt(v / (1 - beta2 ** t)) + epsilon)
    z.mul_(beta1).add_(g, alpha=1 - beta1).sub_((d_t - beta1 * d) * weight)
    d.copy_(d_t)
    weight.copy_(-z / d_t)
    return weight


@register('signsgd_update', arg_names=('weight', 'grad'), params=_COMMON)
@torch.no_grad()
def signsgd_update(weight, grad, lr=0.01, wd=0.0, rescale_grad=1.0, clip_gradient=-1.0):
    weight.mul_(1 - lr * wd).sub_(lr * torch.sign(grad))
    return weight


@register('signum_update', arg_names=('weight', 'grad', 'mom'),
          params=dict(_COMMON, momentum=('float', 0.0), wd_lh=('float', 0.0)))
@torch.no_grad()
def signum_update(weight, grad, mom, lr=0.01, momentum=0.0, wd=0.0, rescale_grad=1.0, clip_gradient=-1.0,
                  wd_lh=0.0):
    g = _prep(grad, rescale_grad, clip_gradient)
    mom.mul_(momentum).sub_((1 - momentum) * wd * weight).sub_((1 - momentum) * g)
    weight.mul_(1 - lr * wd_lh).add_(lr * torch.sign(mom))
    return weight


_LAMB1 = {'beta1': ('float', 0.9), 'beta2': ('float', 0.999), 'epsilon': ('float', 1e-6), 't': ('int', 1),
          'bias_correction': ('bool', True), 'wd': ('float', 0.0), 'rescale_grad': ('float', 1.0),
          'clip_gradient': ('float', -1.0)}


@torch.no_grad()
def _lamb1(weight, grad, mean, var, beta1, beta2, epsilon, t, bias_correction, wd, rescale_grad, clip_gradient):
    g = _prep(grad, rescale_grad, clip_gradient)
    mean.mul_(beta1).add_(g, alpha=1 - beta1)
    var.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    if bias_correction:
        m = mean / (1 - beta1 ** t)
        v = var / (1 - beta2 ** t)
    else:
        m, v = mean, var
    return m / (torch.sqrt(v) + epsilon) + wd * weight.float()


@register('lamb_update_phase1', arg_names=('weight', 'grad', 'mean', 'var'), params=_LAMB1)
def lamb_update_phase1(weight, grad, mean, var, **kw):
    return _lamb1(weight, grad, mean, var, **kw)


@register('mp_lamb_update_phase1', arg_names=('weight', 'grad', 'mean', 'var', 'weight32'), params=_LAMB1)
def mp_lamb_update_phase1(weight, grad, mean, var, weight32, **kw):
    return _lamb1(weight32, grad, mean, var, **kw)


_LAMB2 = {'lr': ('float', 0.001), 'lower_bound': ('float', -1.0), 'upper_bound': ('float', -1.0)}


@torch.no_grad()
def _lamb2(weight, g, r1, r2, lr, lower_bound, upper_bound, w32=None):
    w = weight if w32 is None else w32
    nr1 = r1.reshape(-1)[0].float()
    if lower_bound >= 0:
        nr1 = torch.clamp(nr1, min=lower_bound)
    if upper_bound >= 0:
        nr1 = torch.clamp(nr1, max=upper_bound)
    r2v = r2.reshape(-1)[0].float()
    ratio = torch.where((nr1 == 0) | (r2v == 0), torch.ones_like(nr1), nr1 / r2v)
    w.sub_((lr * ratio * g).to(w.dtype))
    if w32 is not None:
        weight.copy_(w32)
    return weight


@register('lamb_update_phase2', arg_names=('weight', 'g', 'r1', 'r2'), params=_LAMB2)
def lamb_update_phase2(weight, g, r1, r2, lr=0.001, lower_bound=-1.0, upper_bound=-1.0):
    return _lamb2(weight, g, r1, r2, lr, lower_bound, upper_bound)


@register('mp_lamb_update_phase2', arg_names=('weight', 'g', 'r1', 'r2', 'weight32'), params=_LAMB2)
def mp_lamb_update_phase2(weight, g, r1, r2, weight32, lr=0.001, lower_bound=-1.0, upper_bound=-1.0):
    return _lamb2(weight, g, r1, r2, lr, lower_bound, upper_bound, w32=weight32)


# ---------------------------------------------------------------------------
# multi-tensor forms
# ---------------------------------------------------------------------------

def _ntensors(a):
    return int(a.get('num_weights', 1))


def _floats(v, n):
    if isinstance(v, (int, float)):
        return [float(v)] * n
    if isinstance(v, str):
        import ast
        v = ast.literal_eval(v)
    return [float(x) for x in v]


_MULTI = {'lrs': ('any', ()), 'wds': ('any', ()), 'momentum': ('float', 0.0), 'rescale_grad': ('float', 1.0),
          'clip_gradient': ('float', -1.0), 'num_weights': ('int', 1)}


def _multi(per, stride):
    def names(a):
        n = _ntensors(a)
        base = ['weight', 'grad', 'mom', 'weight32'][:stride]
        return ['%s_%d' % (b, i) for i in range(n) for b in base]

    def f(*tensors, lrs=(), wds=(), momentum=0.0, rescale_grad=1.0, clip_gradient=-1.0, num_weights=1):
        lrs = _floats(lrs, num_weights)
        wds = _floats(wds, num_weights)
        groups = [tensors[i * stride:(i + 1) * stride] for i in range(num_weights)]
        if stride >= 3 and groups and groups[0][0].is_cuda and _K.available() and _K.enabled() \
                and hasattr(_K, 'multi_sgd_mom'):
            _K.multi_sgd_mom(groups, lrs, wds, momentum, rescale_grad, clip_gradient, mp=(stride == 4))
        else:
            for gi, grp in enumerate(groups):
                per(grp, lrs[gi], wds[gi], momentum, rescale_grad, clip_gradient)
        return tuple(g[0] for g in groups)
    return names, f


def _p_sgd(g, lr, wd, m, rs, cl):
    _sgd(g[0], g[1], lr, wd, rs, cl)


def _p_sgd_mom(g, lr, wd, m, rs, cl):
    _sgd_mom(g[0], g[1], g[2], lr, m, wd, rs, cl)


def _p_mp_sgd(g, lr, wd, m, rs, cl):
    _sgd(g[0], g[1], lr, wd, rs, cl, w32=g[2])


def _p_mp_sgd_mom(g, lr, wd, m, rs, cl):
    _sgd_mom(g[0], g[1], g[2], lr, m, wd, rs, cl, w32=g[3])


for _name, _per, _stride in [('multi_sgd_update', _p_sgd, 2), ('multi_sgd_mom_update', _p_sgd_mom, 3),
                             ('multi_mp_sgd_update', _p_mp_sgd, 3), ('multi_mp_sgd_mom_update', _p_mp_sgd_mom, 4)]:
    _names, _f = _multi(_per, _stride)
    register(_name, _f, arg_names=_names, params=_MULTI, num_outputs=_ntensors)


@register('multi_sum_sq', arg_names=lambda a: ['array_%d' % i for i in range(int(a.get('num_arrays', 1)))],
          params={'num_arrays': ('int', 1)})
def multi_sum_sq(*arrays, num_arrays=1):
    return torch.stack([a.float().pow(2).sum() for a in arrays])


@register('multi_all_finite', arg_names=lambda a: ['array_%d' % i for i in range(int(a.get('num_arrays', 1)))],
          params={'num_arrays': ('int', 1), 'init_output': ('bool', True)})
def multi_all_finite(*arrays, num_arrays=1, init_output=True):
    ok = torch.stack([torch.isfinite(a).all() for a in arrays]).all()
    return ok.to(torch.float32).reshape(1)


@register('all_finite', params={'init_output': ('bool', True)})
def all_finite(data, init_output=True):
    return torch.isfinite(data).all().to(torch.float32).reshape(1)


@register('reset_arrays', arg_names=lambda a: ['array_%d' % i for i in range(int(a.get('num_arrays', 1)))],
          params={'num_arrays': ('int', 1)}, num_outputs=0)
@torch.no_grad()
def reset_arrays(*arrays, num_arrays=1):
    torch._foreach_zero_(list(arrays))
    return ()


@register('multi_lars', arg_names=('lrs', 'weights_sum_sq', 'grads_sum_sq', 'wds'),
          params={'eta': ('float', 0.001), 'eps': ('float', 1e-8), 'rescale_grad': ('float', 1.0)})
def multi_lars(lrs, weights_sum_sq, grads_sum_sq, wds, eta=0.001, eps=1e-8, rescale_grad=1.0):
    wn = torch.sqrt(weights_sum_sq)
    gn = torch.sqrt(grads_sum_sq) * rescale_grad
    ratio = torch.where((wn > 0) & (gn > 0), eta * wn / (gn + wds * wn + eps), torch.ones_like(wn))
    return lrs * ratio
