"""RNN checkpoint helpers (API parity: python/mxnet/rnn/rnn.py).

Cells keep gate weights fused (``i2h_weight`` holds all gates); a checkpoint
stores them *unpacked* per gate so it is portable between fused
(``FusedRNNCell``) and unfused cell stacks.
"""
from .. import model as _model

__all__ = ['save_rnn_checkpoint', 'load_rnn_checkpoint', 'do_rnn_checkpoint']


def _cell_list(cells):
    return cells if isinstance(cells, (list, tuple)) else [cells]


def save_rnn_checkpoint(cells, prefix, epoch, symbol, arg_params, aux_params):
    """``model.save_checkpoint`` with every cell's weights unpacked first."""
    args = dict(arg_params)
    for cell in _cell_list(cells):
        args = cell.unpack_weights(args)
    _model.save_checkpoint(prefix, epoch, symbol, args, aux_params)


def load_rnn_checkpoint(cells, prefix, epoch):
    """``model.load_checkpoint`` with the cells' weights re-packed; returns (symbol, args, auxs)."""
    sym, args, auxs = _model.load_checkpoint(prefix, epoch)
    for cell in _cell_list(cells):
        args = cell.pack_weights(args)
    return sym, args, auxs


def do_rnn_checkpoint(cells, prefix, period=1):
    """Epoch-end callback saving an RNN checkpoint every ``period`` epochs."""
    period = max(1, int(period))

    def _callback(epoch, sym=None, arg=None, aux=None):
        if (epoch + 1) % period == 0:
            save_rnn_checkpoint(cells, prefix, epoch + 1, sym, arg, aux)
    return _callback
