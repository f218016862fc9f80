"""Dispatcher-level automatic mixed precision (used by contrib.amp.init).

When active, every operator call (imperative ``invoke`` and graph programs)
passes its input tensors through ``cast_inputs``: LP16 ops get fp16/bf16
inputs, FP32 ops fp32 inputs, WIDEST ops the widest floating input type.
"""
import torch

active = False
target = torch.float16
_lp16 = frozenset()
_fp32 = frozenset()
_widest = frozenset()
_cond = {}


def configure(target_dtype, lp16, fp32, widest, cond):
    global active, target, _lp16, _fp32, _widest, _cond
    target = target_dtype
    _lp16 = frozenset(lp16)
    _fp32 = frozenset(fp32)
    _widest = frozenset(widest)
    _cond = {}
    for op, param, values in cond:
        _cond[op] = (param, set(values))
    active = True


def deactivate():
    global active
    active = False


_FLOATS = (torch.float16, torch.bfloat16, torch.float32, torch.float64)


def _cast(ts, dt):
    return [t.to(dt) if (t is not None and t.dtype in _FLOATS and t.dtype != dt) else t for t in ts]


def cast_inputs(opname, ts, attrs):
    if opname in _lp16:
        return _cast(ts, target)
    if opname in _fp32:
        return _cast(ts, torch.float32)
    c = _cond.get(opname)
    if c is not None and str(attrs.get(c[0])) in c[1]:
        return _cast(ts, torch.float32)
    if opname in _widest:
        fl = [t.dtype for t in ts if t is not None and t.dtype in _FLOATS]
        if len(set(fl)) > 1:
            widest = max(fl, key=lambda d: (torch.finfo(d).bits, d == torch.float32))
            return _cast(ts, widest)
    return ts
