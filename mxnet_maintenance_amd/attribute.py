"""Symbol attribute scopes (API parity: python/mxnet/attribute.py).

``with AttrScope(ctx_group='dev1', lr_mult='0.1'): ...`` attaches string
attributes to every symbol created inside; nested scopes merge outer and inner
attributes (inner wins), and explicit attributes passed to a symbol win over
both.
"""
from collections import defaultdict

from ._scope import _ThreadScope

__all__ = ['AttrScope']


class AttrScope(_ThreadScope):
    # how many control-flow subgraphs were built under each name (symbol/contrib.py numbers them
    # <name>0, <name>1, ... like the reference's _get_unique_subgraph_name)
    _subgraph_names = defaultdict(int)

    def __init__(self, **kwargs):
        bad = [k for k, v in kwargs.items() if not isinstance(v, str)]
        if bad:
            raise ValueError('Attributes need to be string (got non-string %s)' % bad)
        self._attr = dict(kwargs)

    def get(self, attr):
        """Scope attributes overlaid with the explicit ``attr`` dict."""
        merged = dict(self._attr)
        merged.update(attr or {})
        return merged

    def _on_enter(self, outer):
        self._attr = dict(outer._attr, **self._attr)
