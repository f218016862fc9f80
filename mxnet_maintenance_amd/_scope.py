"""Thread-local "current object" stacks shared by NameManager and AttrScope.

A scope class derived from ``_ThreadScope`` gets the class property ``current`` (lazily
creating a default instance per thread; assignable) and ``with``-statement support that
pushes / pops itself on a per-thread stack.  ``_on_enter(outer)`` lets a
scope inherit state from the scope it is nested in.
"""
import threading


class _ScopeMeta(type):
    """``Scope.current`` is a thread-local class property: reading gives this thread's innermost
    scope, assigning replaces it (reference: ``AttrScope._current = threading.local()`` with the
    ``current`` class property of python/mxnet/attribute.py and name.py)."""

    @property
    def current(cls):
        return cls._stack()[-1]

    @current.setter
    def current(cls, scope):
        cls._stack()[-1] = scope


class _ThreadScope(metaclass=_ScopeMeta):
    _tls = None            # each subclass gets its own threading.local (see __init_subclass__)

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        if '_tls' not in cls.__dict__ and not any('_tls' in b.__dict__ and b is not _ThreadScope
                                                   for b in cls.__mro__[1:]):
            cls._tls = threading.local()

    @classmethod
    def _stack(cls):
        st = getattr(cls._tls, 'stack', None)
        if st is None:
            st = cls._tls.stack = [cls._default()]
        return st

    @classmethod
    def _default(cls):
        # the default lives on the class that owns the stack (NameManager, not its Prefix subclass,
        # whose constructor needs arguments)
        owner = next(c for c in cls.__mro__ if '_tls' in c.__dict__ and c is not _ThreadScope)
        return owner()

    def _on_enter(self, outer):
        """Hook: adapt to the enclosing scope ``outer``."""

    def __enter__(self):
        st = self._stack()
        self._on_enter(st[-1])
        st.append(self)
        return self

    def __exit__(self, *exc):
        st = self._stack()
        if st and st[-1] is self:
            st.pop()
