"""nose.tools subset: raises, assert_raises, make_decorator, with_setup, nottest, assert_* aliases."""
import functools
import unittest

import pytest

_tc = unittest.TestCase('__init__')
assert_equal = _tc.assertEqual
assert_not_equal = _tc.assertNotEqual
assert_true = _tc.assertTrue
assert_false = _tc.assertFalse
assert_almost_equal = _tc.assertAlmostEqual
assert_in = _tc.assertIn
assert_raises = _tc.assertRaises


def raises(*exceptions):
    def deco(fn):
        @functools.wraps(fn)
        def wrapper(*a, **k):
            with pytest.raises(exceptions):
                fn(*a, **k)
        return wrapper
    return deco


def make_decorator(func):
    def deco(newfunc):
        return functools.wraps(func)(newfunc)
    return deco


def with_setup(setup=None, teardown=None):
    def deco(fn):
        @functools.wraps(fn)
        def wrapper(*a, **k):
            if setup:
                setup()
            try:
                return fn(*a, **k)
            finally:
                if teardown:
                    teardown()
        return wrapper
    return deco


def nottest(fn):
    fn.__test__ = False
    return fn


def ok_(expr, msg=None):
    """nose.tools.ok_: assert ``expr`` is truthy."""
    if not expr:
        raise AssertionError(msg)


def eq_(a, b, msg=None):
    """nose.tools.eq_: assert ``a == b``."""
    if not a == b:
        raise AssertionError(msg or '%r != %r' % (a, b))


assert_is_instance = _tc.assertIsInstance
assert_is_none = _tc.assertIsNone
assert_greater = _tc.assertGreater
assert_less = _tc.assertLess
