"""Autograd front-end.

Parity: python/mxnet/autograd.py (record, pause, train_mode, predict_mode,
is_recording, is_training, set_recording, set_training, mark_variables,
backward, grad, get_symbol, Function) and src/imperative/imperative.cc
(Imperative::Backward).

The tape is PyTorch's autograd graph; what this module adds is MXNet's
variable semantics: ``grad_req`` of 'write' (overwrite), 'add' (accumulate) or
'null', gradient buffers that stay bound to the same storage across
iterations (so the data-parallel all-reduce can use flat bucket views), and the
record/train scopes.
"""
from contextlib import contextmanager


import torch

from . import _state
from .base import MXNetError

__all__ = ['record', 'pause', 'train_mode', 'predict_mode', 'is_recording', 'is_training',
           'set_recording', 'set_training', 'mark_variables', 'backward', 'grad', 'Function',
           'get_symbol']


def set_recording(is_recording):  # pylint: disable=redefined-outer-name
    prev = _state.STATE.recording
    _state.STATE.recording = bool(is_recording)
    return prev


def set_training(train_mode):  # pylint: disable=redefined-outer-name
    prev = _state.STATE.training
    _state.STATE.training = bool(train_mode)
    return prev


def is_recording():
    return _state.STATE.recording


def is_training():
    return _state.STATE.training


class _RecordingStateScope:
    def __init__(self, is_record, train_mode):  # pylint: disable=redefined-outer-name
        self._enter_is_record = is_record
        self._enter_train_mode = train_mode
        self._prev_is_record = None
        self._prev_train_mode = None

    def __enter__(self):
        if self._enter_is_record is not None:
            self._prev_is_record = set_recording(self._enter_is_record)
        if self._enter_train_mode is not None:
            self._prev_train_mode = set_training(self._enter_train_mode)
        return self

    def __exit__(self, ptype, value, trace):
        if self._enter_is_record is not None and self._prev_is_record != self._enter_is_record:
            set_recording(self._prev_is_record)
        if self._enter_train_mode is not None and self._prev_train_mode != self._enter_train_mode:
            set_training(self._prev_train_mode)


def record(train_mode=True):  # pylint: disable=redefined-outer-name
    """Scope in which operations are recorded for gradient computation."""
    return _RecordingStateScope(True, train_mode)


def pause(train_mode=False):  # pylint: disable=redefined-outer-name
    return _RecordingStateScope(False, train_mode)


def train_mode():
    return _RecordingStateScope(None, True)


def predict_mode():
    return _RecordingStateScope(None, False)


def mark_variables(variables, gradients, grad_reqs='write'):
    """Mark NDArrays as variables whose gradient is written into ``gradients``."""
    from .ndarray.ndarray import NDArray
    if isinstance(variables, NDArray):
        variables, gradients = [variables], [gradients]
    if isinstance(grad_reqs, str):
        grad_reqs = [grad_reqs] * len(variables)
    for v, g, r in zip(variables, gradients, grad_reqs):
        if r == 'null':
            v._grad_req = None
            continue
        if not v._data.is_floating_point() or getattr(v, '_idt', None) is not None:
            # integer variable: carried in float64 with its dtype in _idt (NDArray.attach_grad); the
            # gradient buffer becomes a float64 buffer reporting the integer dtype as well
            import torch
            idt = getattr(v, '_idt', None) or v._data.dtype
            if not v._data.is_floating_point():
                v._data = v._data.detach().to(torch.float64)
                v._idt = idt
            if not g._data.is_floating_point():
                gidt = g._data.dtype
                g._data = g._data.to(torch.float64)
                g._idt = gidt
        v._set_grad_buffer(g._data, r)
        v._grad = g


# recorded graphs a backward without retain_graph released (reference: the engine frees the graph
# nodes; differentiating through them again is an error even when torch could replay them).  Keyed on
# the head's torch tensor, i.e. on the recording: an op with out= or an in-place assignment under
# record() rebinds the NDArray to a fresh tensor with a fresh graph, which is differentiable again.
# The mark is an attribute on that tensor (torch tensors compare elementwise, so they cannot be keys
# of a weak dictionary).
_RELEASED_ATTR = '_mxamd_graph_released'


def _collect_leaves(retain):
    leaves = list(_state.STATE.tape_leaves.values())
    if not retain:
        _state.STATE.tape_leaves = {}
    return leaves


def _add_touch_hook(v, t):
    """Record (in _state.GRAD_TOUCHED) that a backward pass reached leaf ``v`` -- a leaf used only
    through a detached path keeps a stale gradient, as in the reference."""
    import weakref
    ref = weakref.ref(v)

    def touched(_t, ref=ref):
        a = ref()
        if a is not None:
            _state.GRAD_TOUCHED.add(id(a))
    t.register_post_accumulate_grad_hook(touched)
    t._mxamd_touch_hook = True


def _zero_marked_grads():
    """Backward of recorded heads with no differentiable path: 'write' gradients of the recorded
    variables become zero and each is marked fresh."""
    leaves = _collect_leaves(False)
    _prepare_leaves(leaves)
    for v in leaves:
        if v._grad is not None:
            v._fresh_grad = True


def _prepare_leaves(leaves):
    """Zero 'write' buffers (grouped in one multi-tensor launch) and rebind stale .grad."""
    zero = []
    arenas = {}
    for v in leaves:
        t = v._data
        if not t.requires_grad or v._grad is None:
            continue
        if not getattr(t, '_mxamd_touch_hook', False):
            _add_touch_hook(v, t)
        gbuf = v._grad._data
        if t.grad is not gbuf:
            t.grad = gbuf
        if v._grad_req == 'write':
            a = v._arena
            if a is not None and a.all_write:
                arenas.setdefault(id(a), (a, []))[1].append(gbuf)
            else:
                zero.append(gbuf)
    with torch.no_grad():
        for a, bufs in arenas.values():
            if len(bufs) == len(a.params):
                a.g.zero_()            # every parameter of the flat arena is on the tape: one memset
            else:
                zero.extend(bufs)      # others keep their gradients ('write' is per parameter)
        if zero:
            torch._foreach_zero_(zero)


def _finish_leaves(leaves):
    touched = _state.GRAD_TOUCHED
    for v in leaves:
        t = v._data
        if v._grad is None:
            continue
        g = t.grad
        if g is not None and g is not v._grad._data:
            # create_graph path builds a new tensor instead of accumulating in place
            v._grad._data = g
            t.grad = g
        if id(v) in touched or not getattr(t, '_mxamd_touch_hook', False):
            v._fresh_grad = True
        else:
            # not reached by this backward (another head's graph, or a detached path): it stays on
            # the tape for a later backward of the same recording
            _state.STATE.tape_leaves.setdefault(id(v), v)
    touched.clear()


def _head_grad(g, t):
    """Match a head gradient to its output's shape.

    The reference binds the head-gradient array as the output-gradient buffer
    (src/imperative/imperative.cc Backward: ``ograd_entries`` take the given arrays),
    so a larger buffer of the same element type is read through its first
    ``t.numel()`` elements. Smaller buffers are an error, as there.
    """
    if g.shape == t.shape:
        return g
    if g.numel() == t.numel() or (g.numel() > t.numel() and g.dim() == t.dim()
                                  and g.shape[1:] == t.shape[1:]):
        return g.reshape(-1)[:t.numel()].reshape(t.shape)
    try:
        return g.expand(t.shape)
    except RuntimeError:
        pass
    raise MXNetError(f'head gradient of shape {tuple(g.shape)} does not match output shape {tuple(t.shape)}')


def backward(heads, head_grads=None, retain_graph=False, train_mode=True, create_graph=False):  # pylint: disable=redefined-outer-name
    """Compute gradients of ``heads`` w.r.t. previously marked variables."""
    from .ndarray.ndarray import NDArray
    if isinstance(heads, NDArray):
        heads = [heads]
    if head_grads is not None and isinstance(head_grads, NDArray):
        head_grads = [head_grads]
    tensors, grads = [], []
    for i, h in enumerate(heads):
        t = h._data
        if not t.requires_grad:
            continue
        tensors.append(t)
        hg = None if head_grads is None else head_grads[i]
        grads.append(torch.ones_like(t) if hg is None else _head_grad(hg._data.to(t.dtype), t))
    if not tensors and heads and all(getattr(h, '_recorded', False) for h in heads):
        # recorded outputs without a differentiable path (integer results, constant outputs): the
        # marked variables get zero gradients, as the reference's backward writes them
        _zero_marked_grads()
        return
    if not tensors:
        raise MXNetError('Cannot differentiate node because it is not in a computational graph. '
                         'You need to set is_recording to true or use autograd.record() to save '
                         'computational graphs for backward.')
    for h in heads:
        if getattr(getattr(h, '_data', None), _RELEASED_ATTR, False):
            raise MXNetError('Check failed: the graph of this output was already freed by a backward pass '
                             'without retain_graph=True; record it again or pass retain_graph=True')
    if not (retain_graph or create_graph):
        for h in heads:
            # only a recorded result owns a graph to free (an identity op may hand back its leaf input)
            if getattr(h, '_data', None) is not None and h._data.grad_fn is not None:
                setattr(h._data, _RELEASED_ATTR, True)
    leaves = _collect_leaves(retain_graph)
    _prepare_leaves(leaves)
    prev_train = set_training(train_mode)
    prev_rec = set_recording(False)
    direct = not create_graph
    if direct:
        _state.DIRECT_GRAD[0] += 1
    try:
        with torch.enable_grad() if create_graph else torch.no_grad():
            torch.autograd.backward(tensors, grads, retain_graph=retain_graph or create_graph,
                                    create_graph=create_graph)
    finally:
        set_training(prev_train)
        set_recording(prev_rec)
        if direct:
            _state.DIRECT_GRAD[0] -= 1
    _finish_leaves(leaves)


def grad(heads, variables, head_grads=None, retain_graph=None, create_graph=False, train_mode=True):  # pylint: disable=redefined-outer-name
    """Return gradients of heads w.r.t. variables (does not touch .grad buffers)."""
    from .ndarray.ndarray import NDArray
    if isinstance(heads, NDArray):
        heads = [heads]
    if isinstance(variables, NDArray):
        variables = [variables]
    if head_grads is not None and isinstance(head_grads, NDArray):
        head_grads = [head_grads]
    hts = [h._data for h in heads]
    if head_grads is None:
        hgs = [torch.ones_like(h) for h in hts]
    else:
        hgs = [torch.ones_like(h) if g is None else g._data for h, g in zip(hts, head_grads)]
    if retain_graph is None:
        retain_graph = create_graph
    # a head without history (e.g. the constant first derivative of a linear op, differentiated
    # again) contributes nothing: the reference's backward gives zero gradients for it
    live = [(h, g) for h, g in zip(hts, hgs) if h.requires_grad]
    gs = [None] * len(variables)
    if live:
        prev_train = set_training(train_mode)
        prev_rec = set_recording(create_graph)
        try:
            with torch.enable_grad():
                gs = torch.autograd.grad([h for h, _ in live], [v._data for v in variables],
                                         grad_outputs=[g for _, g in live], retain_graph=retain_graph,
                                         create_graph=create_graph, allow_unused=True)
        finally:
            set_training(prev_train)
            set_recording(prev_rec)

    def dense(g, v):
        if g is None or g._is_zerotensor():      # torch's symbolic zeros (abs'' etc.) become real arrays
            return torch.zeros_like(v._data)
        return g
    # always a list, even for a single variable: the reference rebinds ``variables`` to a list before
    # its final isinstance check (python/mxnet/autograd.py:318-345), so callers index [0]
    return [NDArray(dense(g, v)) for g, v in zip(gs, variables)]


def get_symbol(x):
    """Return a Symbol for the recorded history of ``x`` (only available for
    arrays produced by a hybridized block; see gluon.block)."""
    sym = getattr(x, '_symbol', None)
    if isinstance(sym, tuple):
        block, i = sym                  # an output of a hybridized block (gluon/block.py)
        return block._recorded_symbols()[i]
    if sym is not None:
        return sym
    if getattr(x, '_hist', None) is None:
        raise MXNetError('get_symbol: the array was not produced by a recorded operator')
    # rebuild the recorded operator history (reference: Imperative::GetSymbol over the autograd
    # entries); arrays without history become variables var0, var1, ...
    from .symbol.symbol import _op_func, var
    memo, nvars = {}, [0]

    def build(a):
        key = id(a)
        if key in memo:
            return memo[key]
        h = getattr(a, '_hist', None)
        if h is None:
            s = var('var%d' % nvars[0])
            nvars[0] += 1
        else:
            (opname, attrs, ins), i = h
            kw = {k: v for k, v in attrs.items() if v is not None}
            node = _op_func(opname)(*[build(b) for b in ins if b is not None], **kw)
            s = node[i] if len(node.list_outputs()) > 1 else node
        memo[key] = s
        return s
    return build(x)


class Function:
    """Customised differentiation (mx.autograd.Function).

    Subclass and implement ``forward`` and ``backward`` over NDArrays; the
    pair is wrapped into a torch.autograd.Function so it composes with the tape.
    """

    def __init__(self):
        self._saved = ()
        self._used = False

    def save_for_backward(self, *args):
        self._saved = args

    @property
    def saved_tensors(self):
        return self._saved

    def __call__(self, *inputs):
        from .ndarray.ndarray import NDArray
        if self._used:
            raise MXNetError('Each Function instance can only be called once.')
        self._used = True
        fself = self
        nin = len(inputs)

        class _Bridge(torch.autograd.Function):
            @staticmethod
            def forward(ctx, *tins):
                with pause():
                    outs = fself.forward(*[NDArray(t.detach()) for t in tins])
                single = isinstance(outs, NDArray)
                ctx.single = single
                outs = [outs] if single else list(outs)
                return tuple(o._data for o in outs)

            @staticmethod
            def backward(ctx, *gouts):
                with pause():
                    gins = fself.backward(*[NDArray(g) for g in gouts])
                if isinstance(gins, NDArray):
                    gins = [gins]
                return tuple(None if g is None else g._data for g in gins)

        from .ndarray.register import _note_leaves
        _note_leaves(inputs)
        tins = [x._data for x in inputs]
        if _state.STATE.recording:
            with torch.enable_grad():
                res = _Bridge.apply(*tins)
        else:
            with torch.no_grad():
                res = _Bridge.apply(*tins)
        outs = [NDArray(r) for r in res]
        return outs[0] if len(outs) == 1 else outs

    def forward(self, *inputs):
        raise NotImplementedError

    def backward(self, *output_grads):
        raise NotImplementedError
