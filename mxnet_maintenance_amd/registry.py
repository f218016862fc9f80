"""Name -> class registries with register / alias / create factories.

Parity: python/mxnet/registry.py:31-175 (get_registry, get_register_func,
get_alias_func, get_create_func).  Used by plug-in style subsystems (optimizers,
initializers, metrics) and by user code that wants the same ``create('name',
...)`` / JSON-config construction.
"""
import json
import warnings

from .base import string_types

__all__ = ['get_registry', 'get_register_func', 'get_alias_func', 'get_create_func']

# base class -> {lower-case name: class}
_TABLES = {}


def _table(base_class):
    return _TABLES.setdefault(base_class, {})


def get_registry(base_class):
    """A snapshot (copy) of the registry of ``base_class``."""
    return dict(_table(base_class))


def get_register_func(base_class, nickname):
    """A decorator ``register(klass, name=None)`` adding subclasses of ``base_class`` under their
    lower-cased name (or ``name``); re-registering a name warns and replaces."""
    table = _table(base_class)

    def register(klass, name=None):
        if not issubclass(klass, base_class):
            raise AssertionError('Can only register subclass of %s' % base_class.__name__)
        key = (klass.__name__ if name is None else name).lower()
        old = table.get(key)
        if old is not None and old is not klass:
            warnings.warn('New %s %s.%s registered with name %s is overriding existing %s %s.%s'
                          % (nickname, klass.__module__, klass.__name__, key, nickname, old.__module__,
                             old.__name__), UserWarning, stacklevel=2)
        table[key] = klass
        return klass

    register.__doc__ = 'Register %s to the %s factory' % (nickname, nickname)
    return register


def get_alias_func(base_class, nickname):
    """A decorator factory ``alias(*names)`` registering the decorated class under every name."""
    register = get_register_func(base_class, nickname)

    def alias(*aliases):
        def deco(klass):
            for a in aliases:
                register(klass, a)
            return klass
        return deco
    return alias


def get_create_func(base_class, nickname):
    """A factory ``create(spec, *args, **kwargs)``.

    ``spec`` may be an instance (returned as is), a registered name, a dict of constructor
    arguments holding the name under ``nickname``, or a JSON string of either form
    (``'["name", {kwargs}]'`` or ``'{"nickname": "name", ...}'``)."""
    table = _table(base_class)

    def create(*args, **kwargs):
        if args:
            spec, args = args[0], args[1:]
        else:
            spec = kwargs.pop(nickname)
        if isinstance(spec, base_class):
            if args or kwargs:
                raise AssertionError('%s is already an instance. Additional arguments are invalid' % nickname)
            return spec
        if isinstance(spec, dict):
            return create(**spec)
        if not isinstance(spec, string_types):
            raise AssertionError('%s must be of string type' % nickname)
        text = spec.strip()
        if text[:1] in ('[', '{'):
            if args or kwargs:
                raise AssertionError('a JSON %s config takes no extra arguments' % nickname)
            cfg = json.loads(text)
            if isinstance(cfg, list):
                return create(cfg[0], **(cfg[1] if len(cfg) > 1 else {}))
            return create(**cfg)
        key = text.lower()
        if key not in table:
            raise AssertionError('%s is not registered. Please register with %s.register first' % (key, nickname))
        return table[key](*args, **kwargs)

    create.__doc__ = ('Create a %s instance from a name, dict or JSON config (an instance is returned '
                      'unchanged).' % nickname)
    return create
