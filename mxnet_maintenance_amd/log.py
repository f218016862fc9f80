"""Logging helpers (reference: python/mxnet/log.py:84 ``get_logger``).

``get_logger`` returns a standard :mod:`logging` logger whose records are prefixed glog-style:
a one-letter level, the time, the process id and the call site, coloured on a terminal.
"""
import logging
import sys
import warnings

CRITICAL = logging.CRITICAL
ERROR = logging.ERROR
WARNING = logging.WARNING
INFO = logging.INFO
DEBUG = logging.DEBUG
NOTSET = logging.NOTSET

_LETTER = {CRITICAL: 'C', ERROR: 'E', WARNING: 'W', INFO: 'I', DEBUG: 'D'}


def _colour(level):
    if level >= WARNING:
        return '\x1b[31m'
    return '\x1b[32m' if level >= INFO else '\x1b[34m'


class _Formatter(logging.Formatter):
    """``<L>MMDD HH:MM:SS pid file:func:line] message`` (colour codes only on a terminal stream)."""

    def __init__(self, colour=True):
        super().__init__(datefmt='%m%d %H:%M:%S')
        self._use_colour = colour

    def format(self, record):
        head = '%s%%(asctime)s %%(process)d %%(pathname)s:%%(funcName)s:%%(lineno)d]' % \
            _LETTER.get(record.levelno, 'U')
        if self._use_colour:
            head = _colour(record.levelno) + head + '\x1b[0m'
        self._style._fmt = head + ' %(message)s'
        return super().format(record)


def get_logger(name=None, filename=None, filemode=None, level=WARNING):
    """A logger named ``name`` writing to ``filename`` (mode ``filemode``, default 'a') or to stderr,
    at ``level``.  Calling it again for the same name adds no second handler."""
    logger = logging.getLogger(name)
    if name is not None and not getattr(logger, '_mxamd_init', False):
        logger._mxamd_init = True
        if filename:
            handler = logging.FileHandler(filename, filemode or 'a')
            handler.setFormatter(_Formatter(colour=False))
        else:
            handler = logging.StreamHandler()
            handler.setFormatter(_Formatter(colour=sys.stderr.isatty()))
        logger.addHandler(handler)
        logger.setLevel(level)
    return logger


def getLogger(name=None, filename=None, filemode=None, level=WARNING):  # pylint: disable=invalid-name
    """Deprecated alias of :func:`get_logger`."""
    warnings.warn('getLogger is deprecated, Use get_logger instead.', DeprecationWarning, stacklevel=2)
    return get_logger(name, filename, filemode, level)
