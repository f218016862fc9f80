"""Word-level RNN language model.

Parity: example/gluon/word_language_model/model.py + train.py in the
reference (Embedding -> stacked LSTM/GRU/RNN -> Dense decoder, optional weight
tying, truncated BPTT with detached hidden state).  The recurrent stack is the
fused ``RNN`` operator, which on the GPU runs the in-tree gfx950 recurrent
kernels (src/kernels/rnn.hip: per-step MFMA gate GEMM fused with the cell).
"""
from ..gluon import nn, rnn, HybridBlock

__all__ = ['RNNModel', 'standard_lstm_lm_200', 'standard_lstm_lm_650', 'standard_lstm_lm_1500', 'detach']


class RNNModel(HybridBlock):
    """``forward(inputs (T, B) int, states) -> (logits (T, B, V), new_states)``."""

    def __init__(self, mode='lstm', vocab_size=10000, num_embed=200, num_hidden=200, num_layers=2, dropout=0.5,
                 tie_weights=False, prefix=None, params=None):
        super().__init__(prefix=prefix, params=params)
        if tie_weights and num_embed != num_hidden:
            raise ValueError('tie_weights requires num_embed == num_hidden')
        self._mode = mode
        self._num_hidden = num_hidden
        with self.name_scope():
            self.drop = nn.Dropout(dropout)
            self.encoder = nn.Embedding(vocab_size, num_embed, weight_initializer='uniform')
            layer = {'lstm': rnn.LSTM, 'gru': rnn.GRU, 'rnn_relu': rnn.RNN, 'rnn_tanh': rnn.RNN}[mode]
            kw = {'activation': mode[4:]} if mode.startswith('rnn_') else {}
            self.rnn = layer(num_hidden, num_layers, dropout=dropout, input_size=num_embed, **kw)
            if tie_weights:
                self.decoder = nn.Dense(vocab_size, in_units=num_hidden, flatten=False, params=self.encoder.params)
            else:
                self.decoder = nn.Dense(vocab_size, in_units=num_hidden, flatten=False)

    def begin_state(self, *args, **kwargs):
        return self.rnn.begin_state(*args, **kwargs)

    def hybrid_forward(self, F, inputs, *states):
        emb = self.drop(self.encoder(inputs))
        output, new_states = self.rnn(emb, list(states))
        output = self.drop(output)
        return self.decoder(output), new_states


def detach(states):
    """Cut the autograd history of hidden states between truncated-BPTT segments."""
    if isinstance(states, (list, tuple)):
        return [detach(s) for s in states]
    return states.detach()


def standard_lstm_lm_200(vocab_size=10000, **kw):
    return RNNModel('lstm', vocab_size, 200, 200, 2, kw.pop('dropout', 0.2), **kw)


def standard_lstm_lm_650(vocab_size=10000, **kw):
    return RNNModel('lstm', vocab_size, 650, 650, 2, kw.pop('dropout', 0.5), **kw)


def standard_lstm_lm_1500(vocab_size=10000, **kw):
    return RNNModel('lstm', vocab_size, 1500, 1500, 2, kw.pop('dropout', 0.65), **kw)
