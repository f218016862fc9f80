"""Probability density / mass functions of the sampling distributions (``random_pdf_*``).

Parity: src/operator/random/pdf_op.{h,cc} (``_random_pdf_normal`` ... ``_random_pdf_dirichlet``):
``sample`` has the distribution parameters' shape plus trailing sample dimension(s); every sample is
evaluated under the parameters of its leading index; ``is_log`` returns the log density.  Written
as log densities in torch so autograd gives the gradients with respect to the sample and to every
parameter.
"""
import math

import torch

from .registry import register

_LOG_2PI = math.log(2.0 * math.pi)


def _bcast(p, sample):
    """Parameter of shape S -> broadcastable against a sample of shape S + (n,)."""
    return p.reshape(tuple(p.shape) + (1,) * (sample.dim() - p.dim()))


def _finish(logp, is_log):
    return logp if is_log else torch.exp(logp)


def _reg(name, args):
    return register('_random_pdf_' + name, aliases=('random_pdf_' + name,), arg_names=('sample',) + args,
                    params={'is_log': ('bool', False)})


@_reg('normal', ('mu', 'sigma'))
def pdf_normal(sample, mu, sigma, is_log=False):
    mu, sigma = _bcast(mu, sample), _bcast(sigma, sample)
    return _finish(-0.5 * ((sample - mu) / sigma) ** 2 - torch.log(sigma) - 0.5 * _LOG_2PI, is_log)


@_reg('uniform', ('low', 'high'))
def pdf_uniform(sample, low, high, is_log=False):
    low, high = _bcast(low, sample), _bcast(high, sample)
    inside = (sample >= low) & (sample <= high)
    logp = torch.where(inside, -torch.log(high - low), torch.full_like(sample, -math.inf))
    return _finish(logp, is_log)


@_reg('gamma', ('alpha', 'beta'))
def pdf_gamma(sample, alpha, beta, is_log=False):
    a, b = _bcast(alpha, sample), _bcast(beta, sample)      # beta is the rate
    return _finish(a * torch.log(b) + (a - 1) * torch.log(sample) - b * sample - torch.lgamma(a), is_log)


@_reg('exponential', ('lam',))
def pdf_exponential(sample, lam, is_log=False):
    lam = _bcast(lam, sample)
    return _finish(torch.log(lam) - lam * sample, is_log)


@_reg('poisson', ('lam',))
def pdf_poisson(sample, lam, is_log=False):
    lam = _bcast(lam, sample)
    return _finish(sample * torch.log(lam) - lam - torch.lgamma(sample + 1), is_log)


def _nb_logpmf(x, k, p):
    return torch.lgamma(x + k) - torch.lgamma(x + 1) - torch.lgamma(k) + k * torch.log(p) + x * torch.log1p(-p)


@_reg('negative_binomial', ('k', 'p'))
def pdf_negative_binomial(sample, k, p, is_log=False):
    return _finish(_nb_logpmf(sample, _bcast(k, sample), _bcast(p, sample)), is_log)


@_reg('generalized_negative_binomial', ('mu', 'alpha'))
def pdf_generalized_negative_binomial(sample, mu, alpha, is_log=False):
    mu, alpha = _bcast(mu, sample), _bcast(alpha, sample)
    return _finish(_nb_logpmf(sample, 1.0 / alpha, 1.0 / (1.0 + alpha * mu)), is_log)


@_reg('dirichlet', ('alpha',))
def pdf_dirichlet(sample, alpha, is_log=False):
    # alpha (..., k), sample (..., n, k) -> (..., n)
    a = alpha.reshape(tuple(alpha.shape[:-1]) + (1,) * (sample.dim() - alpha.dim()) + (alpha.shape[-1],))
    logp = (torch.lgamma(a.sum(-1)) - torch.lgamma(a).sum(-1) + ((a - 1) * torch.log(sample)).sum(-1))
    return _finish(logp, is_log)
