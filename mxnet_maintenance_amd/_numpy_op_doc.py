"""Documentation and Python signatures of the registered ``_np_*`` operators.

Parity: python/mxnet/_numpy_op_doc.py -- every backend operator named ``_np_<name>`` has a
documentation stub here whose signature is the one ``mx.np.<name>`` presents
(numpy_op_signature._get_builtin_op attaches it as ``__signature__``).  The stubs are never called;
the implementations are the registered operators in ops/np_ops.py, reached through
numpy/multiarray.py.
"""
# pylint: disable=unused-argument,redefined-builtin


def _np_all(a, axis=None, out=None, keepdims=False):
    """True where every element along ``axis`` is non-zero (all axes when ``axis`` is None).

    Returns a bool ndarray; with ``keepdims`` the reduced axes stay as size-1 dimensions.
    """


def _np_any(a, axis=None, out=None, keepdims=False):
    """True where at least one element along ``axis`` is non-zero (all axes when ``axis`` is None)."""


def _np_broadcast_to(array, shape):
    """Broadcast ``array`` to ``shape`` following NumPy's broadcasting rules (a copy, not a view)."""


def _np_clip(a, a_min=None, a_max=None, out=None):
    """Limit the values of ``a`` to ``[a_min, a_max]``; either bound may be None (not both)."""


def _np_concatenate(seq, axis=0, out=None):
    """Join a sequence of arrays along an existing ``axis`` (flattened inputs when ``axis`` is None)."""


def _np_cumsum(a, axis=None, dtype=None, out=None):
    """Cumulative sum along ``axis`` (over the flattened array when ``axis`` is None).

    ``dtype`` is the accumulator and result type; integer inputs default to the platform integer.
    """


def _np_diag(v, k=0):
    """A 1-D ``v``: the 2-D array with ``v`` on diagonal ``k``.  A 2-D ``v``: its ``k``-th diagonal."""


def _np_diagflat(v, k=0):
    """The 2-D array with the flattened ``v`` on diagonal ``k``."""


def _np_diagonal(a, offset=0, axis1=0, axis2=1):
    """Diagonal ``offset`` of the 2-D sub-arrays spanned by ``axis1`` and ``axis2``; that pair of axes
    is removed and the diagonal becomes the last axis."""


def _np_dot(a, b, out=None):
    """Dot product: scalar multiplication for 0-d operands, inner product for two vectors, matrix
    product for 2-D operands, and a sum over the last axis of ``a`` and the second-to-last of ``b``
    otherwise."""


def _np_max(a, axis=None, out=None, keepdims=False, initial=None):
    """Maximum along ``axis``; ``initial`` is included in every reduction (required for empty ones)."""


def _np_min(a, axis=None, out=None, keepdims=False, initial=None):
    """Minimum along ``axis``; ``initial`` is included in every reduction (required for empty ones)."""


def _np_negative(x, out=None, **kwargs):
    """Numerical negative, element-wise."""


def _np_prod(a, axis=None, dtype=None, out=None, keepdims=False, initial=None):
    """Product of the elements along ``axis``, multiplied by ``initial`` when given."""


def _np_ravel(x, order='C'):
    """The flattened (1-D, row-major) array; only ``order='C'`` is supported."""


def _np_repeat(a, repeats, axis=None):
    """Repeat every element ``repeats`` times along ``axis`` (the flattened array when None)."""


def _np_reshape(a, newshape, order='C'):
    """Give ``a`` a new shape with the same number of elements; one dimension may be -1 (inferred)."""


def _np_squeeze(a, axis=None):
    """Remove size-1 dimensions (only those listed in ``axis`` when given)."""


def _np_sum(a, axis=None, dtype=None, out=None, keepdims=False, initial=None, where=None):
    """Sum of the elements along ``axis``.

    Half and single precision inputs accumulate one precision up; ``dtype`` sets the result type;
    ``initial`` is added to every sum.  ``where`` is accepted for NumPy compatibility (None only).
    """


def _np_swapaxes(a, axis1, axis2):
    """Interchange two axes of ``a``."""


def _np_tile(A, reps):
    """Repeat ``A`` the number of times given by ``reps`` along each axis."""


def _np_trace(a, offset=0, axis1=0, axis2=1, out=None):
    """Sum along diagonal ``offset`` of the 2-D sub-arrays spanned by ``axis1`` and ``axis2``."""


def _np_transpose(a, axes=None):
    """Permute the axes of ``a`` (reverse them when ``axes`` is None)."""
