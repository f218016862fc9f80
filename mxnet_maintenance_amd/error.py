"""Typed framework errors.

Parity: python/mxnet/error.py:25-59 and base.py register_error.  An error
message of the form ``"<TypeName>: detail"`` (the convention the reference's C++
core uses) is raised as the registered Python class for ``TypeName`` -- e.g.
``"ValueError: ..."`` becomes an exception that is both an ``MXNetError`` and a
``ValueError`` -- so callers can catch the builtin type.
"""
from .base import MXNetError

__all__ = ['MXNetError', 'register', 'register_error', 'InternalError', 'error_class', 'make_error']

_ERRORS = {}


def register_error(func_name=None, cls=None):
    """Register ``cls`` for messages prefixed ``func_name:``; usable as ``@register_error`` or
    ``@register_error('Name')`` or ``register_error('Name', cls)``."""
    if callable(func_name) and cls is None:
        klass = func_name
        _ERRORS[klass.__name__] = klass
        return klass

    def deco(klass):
        _ERRORS[func_name or klass.__name__] = klass
        return klass
    return deco(cls) if cls is not None else deco


register = register_error


@register_error
class InternalError(MXNetError):
    """An internal invariant of the framework was violated."""

    def __init__(self, msg):
        if 'MXNet hint:' not in msg:
            msg += ('\nMXNet hint: You hit an internal error of the framework; please report it with the '
                    'failing program.')
        super().__init__(msg)


def _combined(builtin):
    """An MXNetError subclass that is also ``builtin`` (cached)."""
    name = 'MXNet' + builtin.__name__
    klass = _COMBINED.get(name)
    if klass is None:
        klass = _COMBINED[name] = type(name, (MXNetError, builtin), {'__module__': __name__})
    return klass


_COMBINED = {}

for _b in (ValueError, TypeError, AttributeError, IndexError, NotImplementedError, KeyError):
    register_error(_b.__name__, _combined(_b))


def error_class(name):
    """The class registered for ``name`` (MXNetError when unknown)."""
    return _ERRORS.get(name, MXNetError)


def make_error(msg):
    """The exception for message ``msg``: the registered class of its ``Type:`` prefix, if any."""
    head, sep, _rest = msg.partition(':')
    if sep and head.strip() in _ERRORS:
        return _ERRORS[head.strip()](msg)
    return MXNetError(msg)
