"""Automatic mixed precision (parity: python/mxnet/contrib/amp/amp.py).

Two modes, as in the reference:

* ``amp.init()`` — dynamic: every operator call is routed through the
  precision classes of ``lists.py`` (LP16 ops on fp16/bf16, FP32 ops in fp32,
  widest-type casts for multi-input ops).  ``amp.init_trainer(trainer)`` +
  ``amp.scale_loss(loss, trainer)`` add dynamic loss scaling with overflow
  skipping inside ``Trainer.step``.
* ``convert_symbol`` / ``convert_model`` / ``convert_hybrid_block`` — static:
  rewrite a graph with explicit ``amp_cast`` / ``amp_multicast`` nodes so the
  converted model runs mixed precision with no runtime hook.

MI355X note: bf16 has fp32's exponent range, so with
``target_dtype='bfloat16'`` loss scaling is unnecessary (the scaler stays at
1 and never skips); fp16 keeps the dynamic scaler.
"""
import contextlib
import logging

import numpy as np
import torch

from ... import symbol as sym_mod
from ...base import MXNetError, torch_dtype
from ...ops import amp_dispatch
from . import lists
from .loss_scaler import LossScaler

__all__ = ['init', 'init_trainer', 'scale_loss', 'unscale', 'convert_symbol', 'convert_model',
           'convert_hybrid_block', 'convert_bucketing_module', 'list_lp16_ops', 'list_fp32_ops',
           'list_lp16_fp32_ops', 'list_conditional_fp32_ops', 'list_widest_type_cast', 'list_loss_output_functions',
           'list_lp16_use_fp32_params', 'is_initialized']

_amp_initialized = [False]
_target = ['float16']


def _norm_dtype(target_dtype):
    t = np.dtype(target_dtype).name if not isinstance(target_dtype, str) else target_dtype
    if t in ('float16', 'fp16'):
        return 'float16'
    if t in ('bfloat16', 'bf16'):
        return 'bfloat16'
    raise MXNetError('AMP target_dtype must be float16 or bfloat16, got %s' % target_dtype)


def init(target_dtype='float16', target_precision_ops=None, conditional_fp32_ops=None, fp32_ops=None):
    """Turn on dispatcher-level mixed precision for every subsequent operator call."""
    target = _norm_dtype(target_dtype)
    lp16 = list(lists.LP16) + list(target_precision_ops or [])
    fp32 = [op for op in lists.FP32 if op not in (target_precision_ops or [])] + list(fp32_ops or [])
    cond = list(lists.CONDITIONAL_FP32) + list(conditional_fp32_ops or [])
    amp_dispatch.configure(torch_dtype(target), lp16, fp32, lists.WIDEST, cond)
    _amp_initialized[0] = True
    _target[0] = target
    logging.info('Using AMP (target %s)', target)


def is_initialized():
    return _amp_initialized[0]


def init_trainer(optimizer_or_trainer):
    """Attach a dynamic loss scaler to a gluon Trainer (or an Optimizer used with Module)."""
    from ...gluon.trainer import Trainer
    from ...optimizer import Optimizer
    scaler = LossScaler()
    if _target[0] == 'bfloat16':
        # bf16 shares fp32's exponent range: no scaling, never skip
        scaler = LossScaler(init_scale=1.0, scale_window=1 << 62, max_scale=1.0)
    if isinstance(optimizer_or_trainer, Trainer):
        optimizer_or_trainer._amp_loss_scaler = scaler
        optimizer_or_trainer._amp_original_scale = optimizer_or_trainer._scale
    elif isinstance(optimizer_or_trainer, Optimizer):
        optimizer_or_trainer._amp_loss_scaler = scaler
        optimizer_or_trainer._amp_original_scale = optimizer_or_trainer.rescale_grad
    else:
        raise TypeError('optimizer_or_trainer should be a Gluon Trainer or an optimizer, instead is %s'
                        % type(optimizer_or_trainer))


@contextlib.contextmanager
def scale_loss(loss, optimizer_or_trainer):
    """``with amp.scale_loss(loss, trainer) as scaled: autograd.backward(scaled)``."""
    scaler = optimizer_or_trainer._amp_loss_scaler
    ls = scaler.loss_scale
    if hasattr(optimizer_or_trainer, '_scale'):
        optimizer_or_trainer._scale = optimizer_or_trainer._amp_original_scale / ls
    else:
        optimizer_or_trainer.rescale_grad = optimizer_or_trainer._amp_original_scale / ls
    from ... import autograd
    # the scaling multiply must be on the tape even when called after record() ended
    ctx = autograd.record(train_mode=autograd.is_training()) if not autograd.is_recording() else \
        contextlib.nullcontext()
    with ctx:
        scaled = [l * ls for l in loss] if isinstance(loss, (list, tuple)) else loss * ls
    yield scaled


def unscale(optimizer_or_trainer):
    """Divide the gradients by the current loss scale (e.g. before gradient clipping)."""
    scaler = optimizer_or_trainer._amp_loss_scaler
    inv = 1.0 / scaler.loss_scale
    params = optimizer_or_trainer._params
    with torch.no_grad():
        for p in params:
            if p.grad_req != 'null' and p._grad is not None:
                for g in p._grad:
                    g._data.mul_(inv)
    optimizer_or_trainer._scale = optimizer_or_trainer._amp_original_scale


# ---------------------------------------------------------------------------
# static graph conversion
# ---------------------------------------------------------------------------

def _op_class(node, lp16, fp32, widest, cond):
    if node.op in lp16:
        return 'lp16'
    if node.op in fp32:
        return 'fp32'
    for op, param, values in cond:
        if node.op == op and str(node.attrs.get(param)) in values:
            return 'fp32'
    if node.op in widest:
        return 'widest'
    return None


def convert_symbol(sym, target_dtype='float16', target_dtype_ops=None, fp32_ops=None, conditional_fp32_ops=None,
                   excluded_sym_names=None, data_names=None, cast_optional_params=False):
    """Insert ``amp_cast`` / ``amp_multicast`` nodes so LP16 ops run in ``target_dtype``."""
    from ...symbol.symbol import _Node, Symbol
    target = _norm_dtype(target_dtype)
    lp16 = set(lists.LP16) | set(target_dtype_ops or [])
    fp32 = (set(lists.FP32) - set(target_dtype_ops or [])) | set(fp32_ops or [])
    cond = list(lists.CONDITIONAL_FP32) + list(conditional_fp32_ops or [])
    excluded = set(excluded_sym_names or [])
    out = sym_mod.load_json(sym.tojson())   # work on a copy
    order = out._topo()
    cast_cache = {}

    def cast_entry(entry, dtype):
        key = (id(entry[0]), entry[1], dtype)
        if key not in cast_cache:
            node = _Node('amp_cast', '%s_amp_cast_%s' % (entry[0].name, dtype), {'dtype': dtype}, [entry])
            cast_cache[key] = (node, 0)
        return cast_cache[key]
    for n in order:
        if n.op is None or n.name in excluded:
            continue
        cls = _op_class(n, lp16, fp32, lists.WIDEST, cond)
        if cls == 'lp16':
            n.inputs = [cast_entry(e, target) for e in n.inputs]
        elif cls == 'fp32':
            n.inputs = [cast_entry(e, 'float32') for e in n.inputs]
        elif cls == 'widest' and len(n.inputs) > 1:
            k = len(n.inputs)
            mc = _Node('amp_multicast', '%s_amp_multicast' % n.name, {'num_outputs': str(k)}, list(n.inputs))
            n.inputs = [(mc, i) for i in range(k)]
        n._parsed = None
    return out


def convert_model(sym, arg_params, aux_params, target_dtype='float16', target_dtype_ops=None, fp32_ops=None,
                  conditional_fp32_ops=None, excluded_sym_names=None, cast_optional_params=False):
    """Convert the symbol; params stay fp32 (``amp_cast`` nodes cast them) unless ``cast_optional_params``."""
    new_sym = convert_symbol(sym, target_dtype, target_dtype_ops, fp32_ops, conditional_fp32_ops,
                             excluded_sym_names, cast_optional_params=cast_optional_params)
    if cast_optional_params:
        tgt = _norm_dtype(target_dtype)
        lp16_inputs = set()
        for n in new_sym._topo():
            if n.op == 'amp_cast' and n.attrs.get('dtype') == tgt:
                src = n.inputs[0][0]
                if src.op is None:
                    lp16_inputs.add(src.name)
        arg_params = {k: (v.astype(tgt) if k in lp16_inputs else v) for k, v in arg_params.items()}
    return new_sym, arg_params, aux_params


def convert_hybrid_block(block, target_dtype='float16', target_dtype_ops=None, fp32_ops=None,
                         conditional_fp32_ops=None, excluded_sym_names=None, ctx=None, cast_optional_params=False):
    """Hybridized block -> SymbolBlock running the AMP-converted graph with the same parameters."""
    from ...gluon.block import SymbolBlock
    if not block._cached_graph:
        raise RuntimeError('Please first call block.hybridize() and then run forward with this block at least '
                           'once before calling convert_hybrid_block')
    inputs, out = block._cached_graph
    converted = convert_symbol(out, target_dtype, target_dtype_ops, fp32_ops, conditional_fp32_ops,
                               excluded_sym_names)
    params = block.collect_params()
    ret = SymbolBlock(converted, inputs, params=None)
    arg_names = set(converted.list_arguments()) | set(converted.list_auxiliary_states())
    rp = ret.collect_params()
    for name, p in params.items():
        if name in rp._params and name in arg_names:
            rp[name]._load_init(p.data(), ctx or p.list_ctx()[0]) if hasattr(rp[name], '_load_init') else \
                rp[name].set_data(p.data())
    return ret


def convert_bucketing_module(bucketing_mod, target_dtype='float16', target_dtype_ops=None, fp32_ops=None,
                             conditional_fp32_ops=None, excluded_sym_names=None, cast_optional_params=False):
    from ...module import BucketingModule
    sym_gen = bucketing_mod._sym_gen

    def amp_sym_gen(key):
        s, d, l = sym_gen(key)
        return convert_symbol(s, target_dtype, target_dtype_ops, fp32_ops, conditional_fp32_ops,
                              excluded_sym_names), d, l
    arg, aux = bucketing_mod.get_params() if bucketing_mod.binded and bucketing_mod.params_initialized else \
        ({}, {})
    mod = BucketingModule(amp_sym_gen, bucketing_mod._default_bucket_key, context=bucketing_mod._context)
    mod._preload = (arg, aux)
    return mod


def list_lp16_ops(target_dtype):
    return list(lists.LP16)


def list_fp32_ops(target_dtype):
    return list(lists.FP32)


def list_lp16_fp32_ops(target_dtype):
    return []


def list_conditional_fp32_ops(target_dtype):
    return list(lists.CONDITIONAL_FP32)


def list_widest_type_cast(target_dtype):
    return list(lists.WIDEST)


def list_loss_output_functions(target_dtype):
    return list(lists.LOSS_OUTPUT)


def list_lp16_use_fp32_params(target_dtype):
    return {'BatchNorm': ['gamma', 'beta', 'moving_mean', 'moving_var']}
