"""Automatic naming of symbols / blocks (API parity: python/mxnet/name.py).

``NameManager().get(name, hint)`` returns ``name`` when given, else
``<hint><k>`` with a per-hint counter; ``Prefix(p)`` prepends ``p``.  Managers
are thread-local scopes (``with Prefix('net_'): ...``).
"""
import collections

from ._scope import _ThreadScope

__all__ = ['NameManager', 'Prefix', 'current']


class NameManager(_ThreadScope):
    def __init__(self):
        self._counter = collections.Counter()

    def get(self, name, hint):
        if name:
            return name
        k = self._counter[hint]
        self._counter[hint] = k + 1
        return '%s%d' % (hint, k)


class Prefix(NameManager):
    def __init__(self, prefix):
        super().__init__()
        self._prefix = prefix

    def get(self, name, hint):
        return self._prefix + super().get(name, hint)


def current():
    return NameManager.current
