"""Contributed recurrent-cell utilities (parity: python/mxnet/gluon/contrib/rnn/rnn_cell.py).

``VariationalDropoutCell`` and ``LSTMPCell`` live with the core cells (gluon/rnn/rnn_cell.py) and are
re-exported here.  ``dynamic_unroll`` runs a cell over a sequence through the ``foreach`` control-flow
operator, so a hybridized model holds ONE loop node instead of ``length`` copies of the cell.
"""
from ...rnn.rnn_cell import VariationalDropoutCell, LSTMPCell, _Steps

__all__ = ['VariationalDropoutCell', 'LSTMPCell', 'dynamic_unroll']


def _time_first(F, x, t_axis, ndim):
    if t_axis == 0:
        return x, None
    perm = list(range(ndim))
    perm[0], perm[t_axis] = perm[t_axis], perm[0]
    return F.transpose(x, axes=perm), perm


def dynamic_unroll(cell, inputs, begin_state, drop_inputs=0, drop_outputs=0, layout='TNC', valid_length=None):
    """Unroll ``cell`` over ``inputs`` (``layout`` 'TNC' or 'NTC') with ``foreach``.

    Returns ``(outputs, states)``; outputs keep ``layout``.  With ``valid_length`` (batch,) each
    sequence stops updating its states after its last valid step and the padded outputs are zero.
    Dropout on inputs / outputs shares its mask across time (axes = the time axis)."""
    seq = _Steps(inputs, layout)
    F, t_axis = seq.F, seq.t_axis
    data = seq.as_tensor()
    data, perm = _time_first(F, data, t_axis, len(layout))
    if drop_inputs:
        data = F.Dropout(data, p=drop_inputs, axes=(0,))
    states = list(begin_state) if isinstance(begin_state, (list, tuple)) else [begin_state]
    if valid_length is None:
        body = cell
    else:
        states = states + [F.zeros((1,))]          # step counter rides along as an extra state

        def body(x, st):
            step = st[-1]
            out, new = cell(x, st[:-1])
            live = F.broadcast_greater(valid_length, step)
            new = [F.where(live, n, o) for n, o in zip(new, st[:-1])]
            return out, new + [step + 1]
    outputs, states = F.contrib.foreach(body, data, states)
    if drop_outputs:
        outputs = F.Dropout(outputs, p=drop_outputs, axes=(0,))
    if perm is not None:
        outputs = F.transpose(outputs, axes=perm)
    if valid_length is None:
        return outputs, states
    outputs = F.SequenceMask(outputs, sequence_length=valid_length, use_sequence_length=True, axis=t_axis)
    return outputs, states[:-1]
