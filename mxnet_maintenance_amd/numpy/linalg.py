"""``mx.np.linalg`` (parity: python/mxnet/numpy/linalg.py, fallback_linalg.py,
src/operator/numpy/linalg/*).  Each function is a registered ``_npi_*`` op
(torch.linalg underneath: rocSOLVER/hipBLAS on the GPU), differentiable where
torch.linalg is."""
from .multiarray import _call, _as_nd, _is_sym
from ..ndarray.ndarray import NDArray

__all__ = ['norm', 'svd', 'cholesky', 'inv', 'det', 'slogdet', 'solve', 'tensorinv', 'tensorsolve', 'pinv',
           'eigvals', 'eig', 'eigvalsh', 'eigh', 'qr', 'lstsq', 'matrix_rank', 'matrix_power', 'multi_dot', 'cond']


def norm(x, ord=None, axis=None, keepdims=False):  # pylint: disable=redefined-builtin
    if isinstance(axis, list):
        axis = tuple(axis)
    if ord in ('inf', '-inf'):
        ord = float(ord)
    return _call('_npi_norm', _as_nd(x), ord=ord, axis=axis, keepdims=keepdims)


def svd(a):
    """Returns ``(u, s, vt)`` with ``a == u @ diag(s) @ vt`` (reduced)."""
    return tuple(_call('_npi_svd', _as_nd(a)))


def cholesky(a):
    return _call('_npi_cholesky', _as_nd(a))


def inv(a):
    return _call('_npi_inv', _as_nd(a))


def det(a):
    return _call('_npi_det', _as_nd(a))


def slogdet(a):
    return tuple(_call('_npi_slogdet', _as_nd(a)))


def solve(a, b):
    return _call('_npi_solve', _as_nd(a), _as_nd(b))


def tensorinv(a, ind=2):
    return _call('_npi_tensorinv', _as_nd(a), ind=ind)


def tensorsolve(a, b, axes=None):
    return _call('_npi_tensorsolve', _as_nd(a), _as_nd(b), a_axes=axes)


def pinv(a, rcond=1e-15, hermitian=False):
    if isinstance(rcond, NDArray) or _is_sym(rcond):
        return _call('_npi_pinv', _as_nd(a), rcond, hermitian=hermitian)
    return _call('_npi_pinv_scalar_rcond', _as_nd(a), rcond=float(rcond), hermitian=hermitian)


def eigvals(a):
    return _call('_npi_eigvals', _as_nd(a))


def eig(a):
    return tuple(_call('_npi_eig', _as_nd(a)))


def eigvalsh(a, UPLO='L'):
    return _call('_npi_eigvalsh', _as_nd(a), UPLO=UPLO)


def eigh(a, UPLO='L'):
    return tuple(_call('_npi_eigh', _as_nd(a), UPLO=UPLO))


def qr(a, mode='reduced'):
    return tuple(_call('_npi_qr', _as_nd(a), mode=mode))


def lstsq(a, b, rcond='warn'):
    rc = None if rcond in ('warn', None) else float(rcond)
    return tuple(_call('_npi_lstsq', _as_nd(a), _as_nd(b), rcond=rc))


def matrix_rank(M, tol=None, hermitian=False):
    return _call('_npi_matrix_rank', _as_nd(M), tol=tol, hermitian=hermitian)


def matrix_power(a, n):
    return _call('_npi_matrix_power', _as_nd(a), n=int(n))


def multi_dot(arrays):
    return _call('_npi_multi_dot', *[_as_nd(x) for x in arrays])


def cond(x, p=None):
    return _call('_npi_cond', _as_nd(x), p=p)
