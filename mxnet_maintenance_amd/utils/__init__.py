"""Framework utilities: environment-knob registry (``env``), timing helpers."""
from . import env
from .timing import Timer, cuda_time

__all__ = ['env', 'Timer', 'cuda_time']
