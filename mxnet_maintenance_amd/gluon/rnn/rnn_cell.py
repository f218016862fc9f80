"""Recurrent cells: one time step ``(output, new_states) = cell(input, states)``.

API parity with the reference's python/mxnet/gluon/rnn/rnn_cell.py (cell
classes, constructor arguments, parameter names ``i2h_weight`` / ``h2h_weight``
/ ``i2h_bias`` / ``h2h_bias``, per-step operator names ``t<k>_*`` that show up
in symbolic graphs, ``unroll`` layouts and ``valid_length`` semantics).

Design here: every gated cell is a :class:`_GatedCell` -- one input projection
and one recurrent projection of ``gates * hidden`` rows, followed by a
cell-specific gate combination (:meth:`_combine`).  Sequence plumbing (the many
accepted input forms of ``unroll``) lives in :class:`_Steps`.  The fused
multi-layer cuDNN-style path is rnn_layer.py; cells serve custom recurrences,
decoders and the unfused semantics.
"""
from ... import ndarray, symbol
from ...ndarray.ndarray import NDArray
from ...symbol.symbol import Symbol
from ..block import Block, HybridBlock
from ..utils import _indent

__all__ = ['RecurrentCell', 'HybridRecurrentCell', 'RNNCell', 'LSTMCell', 'GRUCell', 'SequentialRNNCell',
           'HybridSequentialRNNCell', 'DropoutCell', 'ModifierCell', 'ZoneoutCell', 'ResidualCell',
           'BidirectionalCell', 'LSTMPCell', 'VariationalDropoutCell']

tensor_types = (Symbol, NDArray)


def _listify(x):
    if isinstance(x, (list, tuple)):
        return list(x)
    if isinstance(x, Symbol) and len(x.list_outputs()) > 1:
        return [x[i] for i in range(len(x.list_outputs()))]     # e.g. a split into per-step outputs
    return [x]


def _namespace(x):
    """The operator namespace (``symbol`` or ``ndarray``) a tensor / list of tensors belongs to."""
    first = x[0] if isinstance(x, (list, tuple)) else x
    return symbol if isinstance(first, Symbol) else ndarray


# ---------------------------------------------------------------------------------------------
# sequence plumbing
# ---------------------------------------------------------------------------------------------
class _Steps:
    """Normalised view of ``unroll`` inputs.

    Accepted forms: one tensor laid out as ``in_layout`` (default ``layout``), or a list of per-step
    ``(N, C)`` tensors.  ``as_list()`` gives per-step tensors, ``as_tensor()`` one tensor in
    ``layout``; ``F`` is the operator namespace, ``t_axis`` the time axis of ``layout`` and
    ``batch`` the batch size (0 for symbols, whose shape is unknown)."""

    def __init__(self, inputs, layout, length=None, in_layout=None):
        if inputs is None:
            raise AssertionError('unroll(inputs=None) has been deprecated.')
        self.t_axis = layout.find('T')
        self.src_axis = self.t_axis if in_layout is None else in_layout.find('T')
        self.F = _namespace(inputs)
        self.data = inputs
        self.length = length
        if isinstance(inputs, (list, tuple)):
            if length is not None and len(inputs) != length:
                raise AssertionError('unroll: %d steps given for length %d' % (len(inputs), length))
            self.batch = 0 if self.F is symbol else inputs[0].shape[0]
        else:
            self.batch = 0 if self.F is symbol else inputs.shape[layout.find('N')]

    def as_list(self):
        x = self.data
        if isinstance(x, (list, tuple)):
            return list(x)
        if self.F is symbol:
            return list(symbol.split(x, axis=self.src_axis, num_outputs=self.length, squeeze_axis=1))
        n = x.shape[self.src_axis]
        if self.length is not None and self.length != n:
            raise AssertionError('unroll: input has %d steps, length is %d' % (n, self.length))
        return _listify(ndarray.split(x, axis=self.src_axis, num_outputs=n, squeeze_axis=1))

    def as_tensor(self):
        x = self.data
        if isinstance(x, (list, tuple)):
            return self.F.stack(*x, axis=self.t_axis)
        if self.src_axis != self.t_axis:
            x = self.F.swapaxes(x, dim1=self.t_axis, dim2=self.src_axis)
        return x

    def shaped(self, merge):
        """``merge`` True: one tensor; False: a list; None: whatever form was given (a tensor still gets
        its time axis moved to ``layout``)."""
        if merge is False:
            return self.as_list()
        if merge is True or not isinstance(self.data, (list, tuple)):
            return self.as_tensor()
        return list(self.data)


def _format_sequence(length, inputs, layout, merge, in_layout=None):
    """(inputs in the requested form, time axis, namespace, batch size) -- the helper contrib cells use."""
    st = _Steps(inputs, layout, length, in_layout)
    return st.shaped(merge), st.t_axis, st.F, st.batch


def _zero_states(cell, F, begin_state, steps, batch):
    if begin_state is not None:
        return begin_state
    if F is not ndarray and isinstance(steps, (list, tuple)) and steps:
        # traced graph: zeros sized by the first step's batch (N, ...) on every call, not zeros with an
        # unknown batch dim that a cached graph would fix at its first input shape
        x0 = steps[0]
        z = F.zeros_like(F.slice_axis(x0, axis=1, begin=0, end=1))
        out = []
        for info in cell.state_info(0):
            shp = tuple(info['shape'])
            zz = F.reshape(z, shape=(-1,) + (1,) * (len(shp) - 1))
            out.append(F.broadcast_to(zz, shape=(0,) + shp[1:]))
        return out
    kwargs = {'func': F.zeros, 'batch_size': batch}
    if F is ndarray:
        kwargs['ctx'] = steps[0].context if isinstance(steps, (list, tuple)) else steps.context
    return cell.begin_state(**kwargs)


def _masked(F, outputs, length, valid_length, t_axis, merge):
    """Zero the steps beyond each sequence's valid length (SequenceMask), in the requested form."""
    stacked = outputs if isinstance(outputs, tensor_types) else F.stack(*outputs, axis=t_axis)
    out = F.SequenceMask(stacked, sequence_length=valid_length, use_sequence_length=True, axis=t_axis)
    return out if merge else _listify(F.split(out, num_outputs=length, axis=t_axis, squeeze_axis=True))


def _time_reversed(steps, length, valid_length=None):
    """Per-step list in reverse time order; with ``valid_length`` each sequence reverses only its valid
    prefix (SequenceReverse), padding stays in place."""
    if valid_length is None:
        return steps[::-1]
    F = _namespace(steps)
    rev = F.SequenceReverse(F.stack(*steps, axis=0), sequence_length=valid_length, use_sequence_length=True)
    if F is ndarray and length == 1:
        return [rev[0]]
    return _listify(F.split(rev, axis=0, num_outputs=length, squeeze_axis=True))


def _state_info_of(cells, batch_size):
    out = []
    for c in cells:
        out.extend(c.state_info(batch_size))
    return out


def _begin_state_of(cells, **kwargs):
    out = []
    for c in cells:
        out.extend(c.begin_state(**kwargs))
    return out


_MODIFIED_MSG = ('After applying modifier cells (e.g. ZoneoutCell) the base cell cannot be called directly. '
                 'Call the modifier cell instead.')


# ---------------------------------------------------------------------------------------------
# base classes
# ---------------------------------------------------------------------------------------------
class RecurrentCell(Block):
    """Abstract base class for RNN cells: ``state_info`` describes the states, ``begin_state``
    creates them, calling the cell advances one step, ``unroll`` runs a whole sequence."""

    def __init__(self, prefix=None, params=None):
        super().__init__(prefix=prefix, params=params)
        self._modified = False
        self.reset()

    def reset(self):
        """Restart the step / begin-state counters (called at the start of every unroll)."""
        self._init_counter = -1
        self._counter = -1
        for child in self._children.values():
            child.reset()

    def state_info(self, batch_size=0):
        raise NotImplementedError()

    def begin_state(self, batch_size=0, func=ndarray.zeros, **kwargs):
        """Initial states made by ``func`` (``ndarray.zeros``, ``symbol.Variable`` ...), one per
        ``state_info`` entry, named ``<prefix>begin_state_<k>``."""
        if self._modified:
            raise AssertionError(_MODIFIED_MSG)
        symbolic = 'symbol' in getattr(func, '__module__', '')
        out = []
        for info in self.state_info(batch_size):
            self._init_counter += 1
            spec = dict(info or {})
            spec.update(kwargs)
            spec.pop('__layout__', None)
            if symbolic:
                spec.pop('ctx', None)
            out.append(func(name='%sbegin_state_%d' % (self._prefix, self._init_counter), **spec))
        return out

    def unroll(self, length, inputs, begin_state=None, layout='NTC', merge_outputs=None, valid_length=None):
        """Run ``length`` steps; returns ``(outputs, final_states)``.  With ``valid_length`` the
        returned states are each sequence's state at its last valid step and outputs past it are 0."""
        self.reset()
        seq = _Steps(inputs, layout, length)
        steps = seq.as_list()
        states = _zero_states(self, seq.F, begin_state, steps, seq.batch)
        outputs, history = [], []
        for x in steps[:length]:
            y, states = self(x, states)
            outputs.append(y)
            history.append(states)
        F, t_axis = seq.F, seq.t_axis
        if valid_length is None:
            return _Steps(outputs, layout).shaped(merge_outputs), states
        last = [F.SequenceLast(F.stack(*per_step, axis=0), sequence_length=valid_length, use_sequence_length=True,
                               axis=0) for per_step in zip(*history)]
        masked = _masked(F, outputs, length, valid_length, t_axis, True)
        return _Steps(masked, layout, length).shaped(merge_outputs), last

    def _get_activation(self, F, inputs, activation, **kwargs):
        """``activation`` may be a name (fast paths for the common ones, else ``Activation``), a Block
        or any callable."""
        if isinstance(activation, str):
            fast = getattr(F, activation, None) if activation in ('tanh', 'relu', 'sigmoid', 'softsign') else None
            return fast(inputs, **kwargs) if fast is not None else F.Activation(inputs, act_type=activation,
                                                                                **kwargs)
        if callable(activation):
            return activation(inputs, **kwargs)
        return activation

    def forward(self, inputs, states):
        self._counter += 1
        return super().forward(inputs, states)


class HybridRecurrentCell(RecurrentCell, HybridBlock):
    """RecurrentCell that supports hybridize()."""

    def __init__(self, prefix=None, params=None):
        super().__init__(prefix=prefix, params=params)

    def forward(self, x, *args):
        self._counter += 1
        return HybridBlock.forward(self, x, *args)

    def hybrid_forward(self, F, x, *args, **kwargs):
        raise NotImplementedError


class _GatedCell(HybridRecurrentCell):
    """``gates`` projections of width ``hidden_size`` from the input (i2h) and from the first state
    (h2h, of width ``recurrent_size``), combined per cell type by :meth:`_combine`."""

    _gates = 1

    def __init__(self, hidden_size, recurrent_size, i2h_weight_initializer, h2h_weight_initializer,
                 i2h_bias_initializer, h2h_bias_initializer, input_size, prefix, params):
        super().__init__(prefix=prefix, params=params)
        self._hidden_size = hidden_size
        self._input_size = input_size
        rows = self._gates * hidden_size
        get = self.params.get
        self.i2h_weight = get('i2h_weight', shape=(rows, input_size), init=i2h_weight_initializer,
                              allow_deferred_init=True)
        self.h2h_weight = get('h2h_weight', shape=(rows, recurrent_size), init=h2h_weight_initializer,
                              allow_deferred_init=True)
        self._extra_weights()
        self.i2h_bias = get('i2h_bias', shape=(rows,), init=i2h_bias_initializer, allow_deferred_init=True)
        self.h2h_bias = get('h2h_bias', shape=(rows,), init=h2h_bias_initializer, allow_deferred_init=True)

    def __repr__(self):
        rows, cols = self.i2h_weight.shape
        return '%s(%s -> %s%s)' % (type(self).__name__, cols if cols else None, rows, self._repr_extra())

    def _repr_extra(self):
        return ''

    def _extra_weights(self):
        """Hook for cells with more weights (registered between the projections and the biases, the
        reference's parameter order)."""

    def _project(self, F, tag, data, weight, bias):
        return F.FullyConnected(data=data, weight=weight, bias=bias, num_hidden=self._gates * self._hidden_size,
                                name='t%d_%s' % (self._counter, tag))

    def hybrid_forward(self, F, inputs, states, i2h_weight, h2h_weight, i2h_bias, h2h_bias):
        i2h = self._project(F, 'i2h', inputs, i2h_weight, i2h_bias)
        h2h = self._project(F, 'h2h', states[0], h2h_weight, h2h_bias)
        return self._combine(F, 't%d_' % self._counter, i2h, h2h, states)

    def _combine(self, F, tag, i2h, h2h, states):
        raise NotImplementedError


# ---------------------------------------------------------------------------------------------
# concrete cells
# ---------------------------------------------------------------------------------------------
class RNNCell(_GatedCell):
    r"""Elman cell: ``h' = act(W_ih x + b_ih + W_hh h + b_hh)``; state ``[h]``."""

    _gates = 1

    def __init__(self, hidden_size, activation='tanh', i2h_weight_initializer=None, h2h_weight_initializer=None,
                 i2h_bias_initializer='zeros', h2h_bias_initializer='zeros', input_size=0, prefix=None,
                 params=None):
        self._activation = activation
        super().__init__(hidden_size, hidden_size, i2h_weight_initializer, h2h_weight_initializer,
                         i2h_bias_initializer, h2h_bias_initializer, input_size, prefix, params)

    def _alias(self):
        return 'rnn'

    def _repr_extra(self):
        return ', %s' % (self._activation,)

    def state_info(self, batch_size=0):
        return [{'shape': (batch_size, self._hidden_size), '__layout__': 'NC'}]

    def _combine(self, F, tag, i2h, h2h, states):
        h = self._get_activation(F, F.elemwise_add(i2h, h2h, name=tag + 'plus0'), self._activation, name=tag + 'out')
        return h, [h]


class LSTMCell(_GatedCell):
    r"""LSTM cell (Hochreiter & Schmidhuber); gate blocks ordered input, forget, candidate, output.
    States ``[h, c]``."""

    _gates = 4

    def __init__(self, hidden_size, i2h_weight_initializer=None, h2h_weight_initializer=None,
                 i2h_bias_initializer='zeros', h2h_bias_initializer='zeros', input_size=0, prefix=None,
                 params=None, activation='tanh', recurrent_activation='sigmoid'):
        super().__init__(hidden_size, hidden_size, i2h_weight_initializer, h2h_weight_initializer,
                         i2h_bias_initializer, h2h_bias_initializer, input_size, prefix, params)
        self._activation = activation
        self._recurrent_activation = recurrent_activation

    def _alias(self):
        return 'lstm'

    def state_info(self, batch_size=0):
        shape = (batch_size, self._hidden_size)
        return [{'shape': shape, '__layout__': 'NC'}, {'shape': shape, '__layout__': 'NC'}]

    def _combine(self, F, tag, i2h, h2h, states):
        parts = F.SliceChannel(F.elemwise_add(i2h, h2h, name=tag + 'plus0'), num_outputs=4, name=tag + 'slice')
        sig, act = self._recurrent_activation, self._activation
        gate_i = self._get_activation(F, parts[0], sig, name=tag + 'i')
        gate_f = self._get_activation(F, parts[1], sig, name=tag + 'f')
        cand = self._get_activation(F, parts[2], act, name=tag + 'c')
        gate_o = self._get_activation(F, parts[3], sig, name=tag + 'o')
        kept = F.elemwise_mul(gate_f, states[1], name=tag + 'mul0')
        added = F.elemwise_mul(gate_i, cand, name=tag + 'mul1')
        c = F.elemwise_add(kept, added, name=tag + 'state')
        h = F.elemwise_mul(gate_o, self._get_activation(F, c, act, name=tag + 'activation0'), name=tag + 'out')
        return h, [h, c]


class GRUCell(_GatedCell):
    r"""GRU cell (Cho et al.); the reset gate multiplies the recurrent projection *after* the matmul
    (the cuDNN formulation).  Gate blocks ordered reset, update, candidate; state ``[h]``."""

    _gates = 3

    def __init__(self, hidden_size, i2h_weight_initializer=None, h2h_weight_initializer=None,
                 i2h_bias_initializer='zeros', h2h_bias_initializer='zeros', input_size=0, prefix=None,
                 params=None, activation='tanh', recurrent_activation='sigmoid'):
        super().__init__(hidden_size, hidden_size, i2h_weight_initializer, h2h_weight_initializer,
                         i2h_bias_initializer, h2h_bias_initializer, input_size, prefix, params)
        self._activation = activation
        self._recurrent_activation = recurrent_activation

    def _alias(self):
        return 'gru'

    def state_info(self, batch_size=0):
        return [{'shape': (batch_size, self._hidden_size), '__layout__': 'NC'}]

    def _combine(self, F, tag, i2h, h2h, states):
        h_prev = states[0]
        x_r, x_z, x_n = F.SliceChannel(i2h, num_outputs=3, name=tag + 'i2h_slice')
        h_r, h_z, h_n = F.SliceChannel(h2h, num_outputs=3, name=tag + 'h2h_slice')
        sig = self._recurrent_activation
        r = self._get_activation(F, F.elemwise_add(x_r, h_r, name=tag + 'plus0'), sig, name=tag + 'r_act')
        z = self._get_activation(F, F.elemwise_add(x_z, h_z, name=tag + 'plus1'), sig, name=tag + 'z_act')
        n = self._get_activation(F, F.elemwise_add(x_n, F.elemwise_mul(r, h_n, name=tag + 'mul0'), name=tag + 'plus2'),
                                 self._activation, name=tag + 'h_act')
        keep_new = F.elemwise_sub(F.ones_like(z, name=tag + 'ones_like0'), z, name=tag + 'minus0')
        h = F.elemwise_add(F.elemwise_mul(keep_new, n, name=tag + 'mul1'),
                           F.elemwise_mul(z, h_prev, name=tag + 'mul20'), name=tag + 'out')
        return h, [h]


class LSTMPCell(_GatedCell):
    """LSTM with a recurrent projection (Sak et al. 2014): the carried output is ``r = W_hr h`` of
    width ``projection_size``; states ``[r, c]``."""

    _gates = 4

    def __init__(self, hidden_size, projection_size, i2h_weight_initializer=None, h2h_weight_initializer=None,
                 h2r_weight_initializer=None, i2h_bias_initializer='zeros', h2h_bias_initializer='zeros',
                 input_size=0, prefix=None, params=None):
        self._projection_size = projection_size
        self._h2r_init = h2r_weight_initializer
        super().__init__(hidden_size, projection_size, i2h_weight_initializer, h2h_weight_initializer,
                         i2h_bias_initializer, h2h_bias_initializer, input_size, prefix, params)

    def _extra_weights(self):
        self.h2r_weight = self.params.get('h2r_weight', shape=(self._projection_size, self._hidden_size),
                                          init=self._h2r_init, allow_deferred_init=True)

    def _alias(self):
        return 'lstmp'

    def state_info(self, batch_size=0):
        return [{'shape': (batch_size, self._projection_size), '__layout__': 'NC'},
                {'shape': (batch_size, self._hidden_size), '__layout__': 'NC'}]

    def hybrid_forward(self, F, inputs, states, i2h_weight, h2h_weight, h2r_weight, i2h_bias, h2h_bias):
        tag = 't%d_' % self._counter
        i2h = self._project(F, 'i2h', inputs, i2h_weight, i2h_bias)
        h2h = self._project(F, 'h2h', states[0], h2h_weight, h2h_bias)
        parts = F.SliceChannel(i2h + h2h, num_outputs=4, name=tag + 'slice')
        acts = [F.Activation(parts[k], act_type=t, name=tag + n)
                for k, (t, n) in enumerate((('sigmoid', 'i'), ('sigmoid', 'f'), ('tanh', 'c'), ('sigmoid', 'o')))]
        c = F.elemwise_add(acts[1] * states[1], acts[0] * acts[2], name=tag + 'state')
        h = F.elemwise_mul(acts[3], F.Activation(c, act_type='tanh'), name=tag + 'hidden')
        r = F.FullyConnected(data=h, num_hidden=self._projection_size, weight=h2r_weight, no_bias=True,
                             name=tag + 'out')
        return r, [r, c]


# ---------------------------------------------------------------------------------------------
# containers
# ---------------------------------------------------------------------------------------------
def _step_through(cells, inputs, states):
    """One step through stacked cells, each taking its slice of the flat state list."""
    flat, pos = [], 0
    for cell in cells:
        n = len(cell.state_info())
        inputs, new = cell(inputs, states[pos:pos + n])
        pos += n
        flat.extend(new)
    return inputs, flat


def _unroll_through(owner, length, inputs, begin_state, layout, merge_outputs, valid_length):
    owner.reset()
    seq = _Steps(inputs, layout, length)
    data = seq.shaped(None)
    cells = list(owner._children.values())
    states = _zero_states(owner, seq.F, begin_state, data, seq.batch)
    finals, pos = [], 0
    for k, cell in enumerate(cells):
        n = len(cell.state_info())
        last = k == len(cells) - 1
        data, st = cell.unroll(length, inputs=data, begin_state=states[pos:pos + n], layout=layout,
                               merge_outputs=merge_outputs if last else None, valid_length=valid_length)
        pos += n
        finals.extend(st)
    return data, finals


class SequentialRNNCell(RecurrentCell):
    """Stack of cells; the output of one feeds the next."""

    def __init__(self, prefix=None, params=None):
        super().__init__(prefix=prefix, params=params)

    def __repr__(self):
        body = '\n'.join('({}): {}'.format(k, _indent(repr(c), 2)) for k, c in self._children.items())
        return '%s(\n%s\n)' % (type(self).__name__, body)

    def add(self, cell):
        """Append ``cell`` to the stack."""
        self.register_child(cell)

    def state_info(self, batch_size=0):
        return _state_info_of(self._children.values(), batch_size)

    def begin_state(self, **kwargs):
        if self._modified:
            raise AssertionError(_MODIFIED_MSG)
        return _begin_state_of(self._children.values(), **kwargs)

    def unroll(self, length, inputs, begin_state=None, layout='NTC', merge_outputs=None, valid_length=None):
        return _unroll_through(self, length, inputs, begin_state, layout, merge_outputs, valid_length)

    def __getitem__(self, i):
        return list(self._children.values())[i]

    def __len__(self):
        return len(self._children)

    def __call__(self, inputs, states):
        self._counter += 1
        if any(isinstance(c, BidirectionalCell) for c in self._children.values()):
            raise AssertionError('BidirectionalCell cannot be stepped inside a SequentialRNNCell; use unroll')
        return _step_through(self._children.values(), inputs, states)

    def hybrid_forward(self, *args, **kwargs):
        raise NotImplementedError


class HybridSequentialRNNCell(HybridRecurrentCell):
    """Hybridizable stack of cells."""

    def __init__(self, prefix=None, params=None):
        super().__init__(prefix=prefix, params=params)

    __repr__ = SequentialRNNCell.__repr__
    add = SequentialRNNCell.add
    state_info = SequentialRNNCell.state_info
    begin_state = SequentialRNNCell.begin_state
    unroll = SequentialRNNCell.unroll
    __getitem__ = SequentialRNNCell.__getitem__
    __len__ = SequentialRNNCell.__len__

    def __call__(self, inputs, states):
        self._counter += 1
        return _step_through(self._children.values(), inputs, states)

    def hybrid_forward(self, F, inputs, states):
        return self.__call__(inputs, states)


class DropoutCell(HybridRecurrentCell):
    """Dropout on the step input (stateless); ``axes`` share the mask along those axes."""

    def __init__(self, rate, axes=(), prefix=None, params=None):
        super().__init__(prefix, params)
        if not isinstance(rate, (int, float)):
            raise AssertionError('rate must be a number')
        self._rate = rate
        self._axes = axes

    def __repr__(self):
        return '%s(rate=%s, axes=%s)' % (type(self).__name__, self._rate, self._axes)

    def state_info(self, batch_size=0):
        return []

    def _alias(self):
        return 'dropout'

    def hybrid_forward(self, F, inputs, states):
        if self._rate > 0:
            inputs = F.Dropout(data=inputs, p=self._rate, axes=self._axes, name='t%d_fwd' % self._counter)
        return inputs, states

    def unroll(self, length, inputs, begin_state=None, layout='NTC', merge_outputs=None, valid_length=None):
        self.reset()
        seq = _Steps(inputs, layout, length)
        data = seq.shaped(merge_outputs)
        if isinstance(data, tensor_types):      # one dropout over the whole sequence tensor
            return self.hybrid_forward(seq.F, data, begin_state or [])
        return super().unroll(length, data, begin_state=begin_state, layout=layout, merge_outputs=merge_outputs)


class ModifierCell(HybridRecurrentCell):
    """Base class for cells that wrap (modify) another cell; shares the wrapped cell's parameters."""

    def __init__(self, base_cell):
        if base_cell._modified:
            raise AssertionError('Cell %s is already modified. One cell cannot be modified twice' % base_cell.name)
        base_cell._modified = True
        super().__init__(prefix=base_cell.prefix + self._alias(), params=None)
        self.base_cell = base_cell

    @property
    def params(self):
        return self.base_cell.params

    def state_info(self, batch_size=0):
        return self.base_cell.state_info(batch_size)

    def begin_state(self, func=ndarray.zeros, **kwargs):
        if self._modified:
            raise AssertionError(_MODIFIED_MSG)
        self.base_cell._modified = False
        try:
            return self.base_cell.begin_state(func=func, **kwargs)
        finally:
            self.base_cell._modified = True

    def hybrid_forward(self, F, inputs, states):
        raise NotImplementedError

    def __repr__(self):
        return '%s(%r)' % (type(self).__name__, self.base_cell)


class ZoneoutCell(ModifierCell):
    """Zoneout (Krueger et al. 2016): each output / state unit keeps its previous value with
    probability ``zoneout_outputs`` / ``zoneout_states`` during training."""

    def __init__(self, base_cell, zoneout_outputs=0., zoneout_states=0.):
        if isinstance(base_cell, BidirectionalCell):
            raise AssertionError("BidirectionalCell doesn't support zoneout since it doesn't support step. "
                                 "Please add ZoneoutCell to the cells underneath instead.")
        super().__init__(base_cell)
        self.zoneout_outputs = zoneout_outputs
        self.zoneout_states = zoneout_states
        self._prev_output = None

    def __repr__(self):
        return '%s(p_out=%s, p_state=%s, %r)' % (type(self).__name__, self.zoneout_outputs, self.zoneout_states,
                                                 self.base_cell)

    def _alias(self):
        return 'zoneout'

    def reset(self):
        super().reset()
        self._prev_output = None

    def hybrid_forward(self, F, inputs, states):
        new_out, new_states = self.base_cell(inputs, states)

        def keep_new(p, like):      # 1 where the new value is taken (dropout of ones: 0 or 1/(1-p))
            return F.Dropout(F.ones_like(like), p=p)
        prev = self._prev_output if self._prev_output is not None else F.zeros_like(new_out)
        out = new_out if self.zoneout_outputs == 0. else F.where(keep_new(self.zoneout_outputs, new_out), new_out,
                                                                  prev)
        if self.zoneout_states != 0.:
            new_states = [F.where(keep_new(self.zoneout_states, n), n, o) for n, o in zip(new_states, states)]
        self._prev_output = out
        return out, new_states


class ResidualCell(ModifierCell):
    """Adds the step input to the wrapped cell's output (He et al. residual connection)."""

    def __init__(self, base_cell):
        super().__init__(base_cell)

    def hybrid_forward(self, F, inputs, states):
        out, states = self.base_cell(inputs, states)
        return F.elemwise_add(out, inputs, name='t%d_fwd' % self._counter), states

    def unroll(self, length, inputs, begin_state=None, layout='NTC', merge_outputs=None, valid_length=None):
        self.reset()
        self.base_cell._modified = False
        try:
            outs, states = self.base_cell.unroll(length, inputs=inputs, begin_state=begin_state, layout=layout,
                                                 merge_outputs=merge_outputs, valid_length=valid_length)
        finally:
            self.base_cell._modified = True
        merge = isinstance(outs, tensor_types) if merge_outputs is None else merge_outputs
        seq = _Steps(inputs, layout, length)
        skip = seq.shaped(merge)
        if valid_length is not None:
            skip = _masked(seq.F, skip, length, valid_length, seq.t_axis, merge)
        if merge:
            return seq.F.elemwise_add(outs, skip), states
        return [seq.F.elemwise_add(a, b) for a, b in zip(outs, skip)], states


class BidirectionalCell(HybridRecurrentCell):
    """Runs ``l_cell`` forward and ``r_cell`` backward in time and concatenates their outputs on the
    feature axis; can only be unrolled."""

    def __init__(self, l_cell, r_cell, output_prefix='bi_'):
        super().__init__(prefix='', params=None)
        self.register_child(l_cell, 'l_cell')
        self.register_child(r_cell, 'r_cell')
        self._output_prefix = output_prefix

    def __call__(self, inputs, states):
        raise NotImplementedError('Bidirectional cannot be stepped. Please use unroll')

    def __repr__(self):
        return '%s(forward=%r, backward=%r)' % (type(self).__name__, self._children['l_cell'],
                                                self._children['r_cell'])

    def state_info(self, batch_size=0):
        return _state_info_of(self._children.values(), batch_size)

    def begin_state(self, **kwargs):
        if self._modified:
            raise AssertionError(_MODIFIED_MSG)
        return _begin_state_of(self._children.values(), **kwargs)

    def unroll(self, length, inputs, begin_state=None, layout='NTC', merge_outputs=None, valid_length=None):
        self.reset()
        seq = _Steps(inputs, layout, length)
        steps = seq.as_list()
        F, t_axis = seq.F, seq.t_axis
        fwd, bwd = self._children['l_cell'], self._children['r_cell']
        states = _zero_states(self, F, begin_state, steps, seq.batch)
        n_fwd = len(fwd.state_info(seq.batch))
        f_out, f_states = fwd.unroll(length, inputs=steps, begin_state=states[:n_fwd], layout=layout,
                                     merge_outputs=merge_outputs, valid_length=valid_length)
        b_out, b_states = bwd.unroll(length, inputs=_time_reversed(steps, length, valid_length),
                                     begin_state=states[n_fwd:], layout=layout, merge_outputs=False,
                                     valid_length=valid_length)
        b_out = _time_reversed(b_out, length, valid_length)
        if merge_outputs is None:
            merge_outputs = isinstance(f_out, tensor_types)
            f_out = _Steps(f_out, layout).shaped(merge_outputs)
            b_out = _Steps(b_out, layout).shaped(merge_outputs)
        if merge_outputs:
            if not isinstance(b_out, tensor_types):
                b_out = F.stack(*b_out, axis=t_axis)
            outputs = F.concat(f_out, b_out, dim=2, name='%sout' % self._output_prefix)
        else:
            outputs = [F.concat(a, b, dim=1, name='%st%d' % (self._output_prefix, k))
                       for k, (a, b) in enumerate(zip(f_out, b_out))]
        if valid_length is not None:
            outputs = _masked(F, outputs, length, valid_length, t_axis, merge_outputs)
        return outputs, f_states + b_states


class VariationalDropoutCell(ModifierCell):
    """Variational dropout (Gal & Ghahramani 2016): one mask per sequence (drawn at the first step
    after ``reset``) for the inputs, the first state and the outputs."""

    def __init__(self, base_cell, drop_inputs=0., drop_states=0., drop_outputs=0.):
        if drop_states and isinstance(base_cell, BidirectionalCell):
            raise AssertionError("BidirectionalCell doesn't support variational state dropout.")
        super().__init__(base_cell)
        self.drop_inputs = drop_inputs
        self.drop_states = drop_states
        self.drop_outputs = drop_outputs
        self.drop_inputs_mask = None
        self.drop_states_mask = None
        self.drop_outputs_mask = None

    def _alias(self):
        return 'vardrop'

    def reset(self):
        super().reset()
        self.drop_inputs_mask = self.drop_states_mask = self.drop_outputs_mask = None

    @staticmethod
    def _mask(F, p, like):
        return F.Dropout(F.ones_like(like), p=p)

    def _initialize_input_masks(self, F, inputs, states):
        if self.drop_states and self.drop_states_mask is None:
            self.drop_states_mask = self._mask(F, self.drop_states, states[0])
        if self.drop_inputs and self.drop_inputs_mask is None:
            self.drop_inputs_mask = self._mask(F, self.drop_inputs, inputs)

    def _initialize_output_mask(self, F, output):
        if self.drop_outputs and self.drop_outputs_mask is None:
            self.drop_outputs_mask = self._mask(F, self.drop_outputs, output)

    def hybrid_forward(self, F, inputs, states):
        self._initialize_input_masks(F, inputs, states)
        if self.drop_states:
            states = [states[0] * self.drop_states_mask] + list(states[1:])
        if self.drop_inputs:
            inputs = inputs * self.drop_inputs_mask
        out, new_states = self.base_cell(inputs, states)
        self._initialize_output_mask(F, out)
        if self.drop_outputs:
            out = out * self.drop_outputs_mask
        return out, new_states

    def __repr__(self):
        return '%s(p_out = %s, p_state = %s)' % (type(self).__name__, self.drop_outputs, self.drop_states)
