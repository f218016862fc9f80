"""BERT (Transformer encoder) in Gluon HybridBlocks.

Parity: the BERT models MXNet 1.x users build from GluonNLP on top of
src/operator/contrib/transformer.cc (interleaved_matmul_selfatt_*), LayerNorm
(src/operator/nn/layer_norm*) and GELU (LeakyReLU act_type='gelu'); the
reference repo's own transformer test is tests/python/unittest/test_operator.py
(test_multihead_attention_selfatt).

MI355X layout decisions: activations are kept time-major (S, B, C) inside the
encoder so the fused QKV projection output feeds attention without a
transpose; attention runs as one fused ``_contrib_sdp_attention`` op (ROCm
flash-attention kernel) or, with ``fused_attention=False``, as the reference's
interleaved QK / softmax / VAL-ATT op sequence.  All GEMMs are large
(B*S x C) x (C x 3C|4C) hipBLASLt calls in bf16/fp16.
"""
from ..gluon import nn, HybridBlock
from .. import initializer as init

__all__ = ['BERTEncoderCell', 'BERTEncoder', 'BERTModel', 'get_bert_model', 'bert_12_768_12', 'bert_24_1024_16',
           'BERT_CONFIGS']

BERT_CONFIGS = {
    'bert_12_768_12': dict(num_layers=12, units=768, hidden_size=3072, num_heads=12, max_length=512, dropout=0.1),
    'bert_24_1024_16': dict(num_layers=24, units=1024, hidden_size=4096, num_heads=16, max_length=512, dropout=0.1),
}


class _ResidualLayerNorm(nn.LayerNorm):
    """LayerNorm(residual + Dropout(data)): the sub-layer tail as the fused add_dropout_layernorm
    operator (same parameters as the LayerNorm it replaces)."""

    def __init__(self, dropout=0.0, **kwargs):
        super().__init__(**kwargs)
        self._p = dropout

    def hybrid_forward(self, F, data, residual, gamma, beta):
        # data = sub-layer(residual) starts with a Dense on residual: its data gradient absorbs the
        # residual gradient (no separate accumulation)
        return F.contrib.add_dropout_layernorm(data, residual, gamma, beta, p=self._p, eps=self._epsilon,
                                               fuse_residual_grad=True)


class BERTEncoderCell(HybridBlock):
    """Post-LN transformer layer: x + Attn(x) -> LN -> x + FFN(x) -> LN on (S, B, C) inputs."""

    def __init__(self, units=768, hidden_size=3072, num_heads=12, dropout=0.1, layer_norm_eps=1e-12,
                 fused_attention=True, prefix=None, params=None):
        super().__init__(prefix=prefix, params=params)
        assert units % num_heads == 0
        self._units = units
        self._heads = num_heads
        self._dropout = dropout
        self._fused = fused_attention
        with self.name_scope():
            # one (C -> 3C) projection whose output is interleaved per head as [q k v]
            self.attn_qkv = nn.Dense(3 * units, flatten=False, in_units=units, prefix='attn_qkv_')
            self.attn_proj = nn.Dense(units, flatten=False, in_units=units, prefix='attn_proj_')
            self.ln1 = _ResidualLayerNorm(dropout=dropout, epsilon=layer_norm_eps, in_channels=units, prefix='ln1_')
            self.ffn_1 = nn.Dense(hidden_size, flatten=False, in_units=units, activation=None, prefix='ffn1_')
            self.ffn_2 = nn.Dense(units, flatten=False, in_units=hidden_size, prefix='ffn2_')
            self.ln2 = _ResidualLayerNorm(dropout=dropout, epsilon=layer_norm_eps, in_channels=units, prefix='ln2_')

    def hybrid_forward(self, F, x, mask=None):
        qkv = self.attn_qkv(x)
        if self._fused:
            if mask is not None:
                ctx = F.contrib.sdp_attention(qkv, mask, heads=self._heads, dropout=self._dropout, use_mask=True)
            else:
                ctx = F.contrib.sdp_attention(qkv, heads=self._heads, dropout=self._dropout)
        else:
            scores = F.contrib.interleaved_matmul_selfatt_qk(qkv, heads=self._heads)
            if mask is not None:
                # mask (B, S_k) -> (B*H, 1, S_k) additive
                m = F.reshape(F.repeat(F.expand_dims(mask, axis=1), repeats=self._heads, axis=1), shape=(-3, 1, -1))
                scores = F.broadcast_add(scores, (1 - m) * -1e4)
            att = F.softmax(scores, axis=-1)
            if self._dropout:
                att = F.Dropout(att, p=self._dropout)
            ctx = F.contrib.interleaved_matmul_selfatt_valatt(qkv, att, heads=self._heads)
        x = self.ln1(self.attn_proj(ctx), x)             # LN(x + dropout(h)), one fused kernel
        f = self.ffn_2(F.LeakyReLU(self.ffn_1(x), act_type='gelu'))
        return self.ln2(f, x)


class BERTEncoder(HybridBlock):
    def __init__(self, num_layers=12, units=768, hidden_size=3072, num_heads=12, dropout=0.1, fused_attention=True,
                 prefix=None, params=None):
        super().__init__(prefix=prefix, params=params)
        with self.name_scope():
            self.layers = nn.HybridSequential(prefix='')
            for i in range(num_layers):
                self.layers.add(BERTEncoderCell(units, hidden_size, num_heads, dropout, fused_attention=fused_attention,
                                                prefix='layer%d_' % i))

    def hybrid_forward(self, F, x, mask=None):
        for cell in self.layers._children.values():
            x = cell(x, mask) if mask is not None else cell(x)
        return x


class BERTModel(HybridBlock):
    """BERT with embeddings, encoder, pooler, masked-LM decoder (tied embedding) and NSP classifier.

    ``forward(inputs, token_types, valid_length=None, masked_positions=None)`` with inputs (B, S)
    returns ``(sequence_output (B,S,C), pooled (B,C), nsp_scores (B,2), mlm_scores (B,P,V))``
    (the latter two only when the corresponding heads are enabled).
    """

    def __init__(self, vocab_size=30522, token_type_vocab_size=2, units=768, hidden_size=3072, num_layers=12,
                 num_heads=12, max_length=512, dropout=0.1, use_pooler=True, use_decoder=True, use_classifier=True,
                 fused_attention=True, prefix=None, params=None):
        super().__init__(prefix=prefix, params=params)
        self._units = units
        self._use_pooler = use_pooler
        self._use_decoder = use_decoder
        self._use_classifier = use_classifier
        self._vocab = vocab_size
        with self.name_scope():
            self.word_embed_weight = self.params.get('word_embed_weight', shape=(vocab_size, units),
                                                     init=init.Normal(0.02))
            self.token_type_embed = nn.Embedding(token_type_vocab_size, units, prefix='token_type_embed_',
                                                 weight_initializer=init.Normal(0.02))
            self.position_weight = self.params.get('position_weight', shape=(max_length, units),
                                                   init=init.Normal(0.02))
            self.embed_ln = nn.LayerNorm(epsilon=1e-12, in_channels=units, prefix='embed_ln_')
            self.embed_drop = nn.Dropout(dropout) if dropout else None
            self.encoder = BERTEncoder(num_layers, units, hidden_size, num_heads, dropout, fused_attention,
                                       prefix='enc_')
            if use_pooler:
                self.pooler = nn.Dense(units, activation='tanh', flatten=False, in_units=units, prefix='pooler_')
            if use_classifier:
                self.classifier = nn.Dense(2, in_units=units, prefix='cls_')
            if use_decoder:
                self.dec_transform = nn.Dense(units, flatten=False, in_units=units, prefix='dec_transform_')
                self.dec_ln = nn.LayerNorm(epsilon=1e-12, in_channels=units, prefix='dec_ln_')
                self.dec_bias = self.params.get('dec_bias', shape=(vocab_size,), init='zeros')

    def hybrid_forward(self, F, inputs, token_types, valid_length=None, masked_positions=None, word_embed_weight=None,
                       position_weight=None, dec_bias=None):
        emb = F.Embedding(inputs, word_embed_weight, input_dim=self._vocab, output_dim=self._units)
        emb = emb + self.token_type_embed(token_types)
        pos = F.slice_like(position_weight, F.transpose(emb, axes=(1, 0, 2)), axes=(0,))   # (S, C)
        emb = F.broadcast_add(emb, F.expand_dims(pos, axis=0))
        emb = self.embed_ln(emb)
        if self.embed_drop is not None:
            emb = self.embed_drop(emb)
        x = F.transpose(emb, axes=(1, 0, 2))                                              # (S, B, C)
        mask = None
        if valid_length is not None:
            steps = F.contrib.arange_like(inputs, axis=1)                                 # (S,)
            mask = F.broadcast_lesser(F.reshape(steps, shape=(1, -1)), F.reshape(valid_length, shape=(-1, 1)))
            mask = F.cast(mask, dtype='float32')
        x = self.encoder(x, mask) if mask is not None else self.encoder(x)
        seq = F.transpose(x, axes=(1, 0, 2))                                              # (B, S, C)
        outputs = [seq]
        if self._use_pooler:
            cls = F.squeeze(F.slice_axis(seq, axis=1, begin=0, end=1), axis=1)
            pooled = self.pooler(cls)
            outputs.append(pooled)
            if self._use_classifier:
                outputs.append(self.classifier(pooled))
        if self._use_decoder and masked_positions is not None:
            bidx = F.broadcast_like(F.reshape(F.contrib.arange_like(masked_positions, axis=0), shape=(-1, 1)),
                                    masked_positions)
            idx = F.stack(bidx, F.cast(masked_positions, dtype='float32'), axis=0)
            picked = F.gather_nd(seq, idx)                                                # (B, P, C)
            h = self.dec_ln(F.LeakyReLU(self.dec_transform(picked), act_type='gelu'))
            scores = F.FullyConnected(h, word_embed_weight, dec_bias, num_hidden=self._vocab, flatten=False)
            outputs.append(scores)
        return tuple(outputs) if len(outputs) > 1 else outputs[0]


def get_bert_model(name='bert_12_768_12', vocab_size=30522, **kwargs):
    cfg = dict(BERT_CONFIGS[name])
    cfg.update(kwargs)
    return BERTModel(vocab_size=vocab_size, **cfg)


def bert_12_768_12(**kwargs):
    return get_bert_model('bert_12_768_12', **kwargs)


def bert_24_1024_16(**kwargs):
    return get_bert_model('bert_24_1024_16', **kwargs)
