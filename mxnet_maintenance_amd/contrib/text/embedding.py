"""Token embeddings (API parity: contrib/text/embedding.py).

A token embedding is a Vocabulary plus an ``idx_to_vec`` matrix (row i = vector of
token i, row 0 = unknown).  Vectors come from a text file: one token per line
followed by its ``elem_delim``-separated values (the GloVe / fastText ``.vec``
format).  There is no network here, so ``GloVe`` / ``FastText`` load the named
file from ``embedding_root`` (default ``~/.mxnet/embeddings/<name>``) and fail
with a clear message when it is absent; ``CustomEmbedding`` takes any path.
"""
import io
import logging
import os
import warnings

import numpy as np

from ... import ndarray as nd
from . import vocab as _vocab

__all__ = ['register', 'create', 'get_pretrained_file_names', 'GloVe', 'FastText', 'CustomEmbedding',
           'CompositeEmbedding']

_REGISTRY = {}


def register(embedding_cls):
    """Class decorator: make an embedding creatable by ``create(<lower-case class name>)``."""
    _REGISTRY[embedding_cls.__name__.lower()] = embedding_cls
    return embedding_cls


def create(embedding_name, **kwargs):
    try:
        cls = _REGISTRY[embedding_name.lower()]
    except KeyError:
        raise KeyError('Cannot find `embedding_name` %s. Use `get_pretrained_file_names()` to list the '
                       'registered embeddings.' % embedding_name) from None
    return cls(**kwargs)


def get_pretrained_file_names(embedding_name=None):
    """Known pre-trained file names, per embedding (or for one embedding)."""
    if embedding_name is not None:
        if embedding_name.lower() not in _REGISTRY:
            raise KeyError('Cannot find `embedding_name` %s.' % embedding_name)
        return list(_REGISTRY[embedding_name.lower()].pretrained_file_names)
    return {name: list(cls.pretrained_file_names) for name, cls in _REGISTRY.items()
            if getattr(cls, 'pretrained_file_names', None)}


class _TokenEmbedding(_vocab.Vocabulary):
    """Vocabulary with one vector per token."""

    pretrained_file_names = ()

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self._idx_to_vec = None

    # ---------------------------------------------------------------- loading
    def _load_embedding(self, path, elem_delim, init_unknown_vec, encoding='utf8'):
        if not os.path.isfile(path):
            raise ValueError('`pretrained_file_path` must be a valid path to the pre-trained token '
                             'embedding file: %s' % path)
        tokens, vecs, dim = [], [], None
        loaded_unknown = None
        with io.open(path, 'r', encoding=encoding) as f:
            for lineno, line in enumerate(f):
                parts = line.rstrip().split(elem_delim)
                if len(parts) < 2:
                    continue
                tok, vals = parts[0], parts[1:]
                if dim is None and len(vals) == 1 and lineno == 0:
                    continue          # fastText header "<count> <dim>"
                try:
                    vec = [float(v) for v in vals]
                except ValueError:
                    warnings.warn('line %d of %s is not a vector; skipped' % (lineno, path))
                    continue
                if dim is None:
                    dim = len(vec)
                elif len(vec) != dim:
                    warnings.warn('line %d of %s has %d values, expected %d; skipped' % (lineno, path, len(vec), dim))
                    continue
                if tok == self.unknown_token:
                    loaded_unknown = vec
                    continue
                if tok in self._token_to_idx:
                    warnings.warn('token %s repeated in %s; the first vector is kept' % (tok, path))
                    continue
                self._token_to_idx[tok] = len(self._idx_to_token)
                self._idx_to_token.append(tok)
                tokens.append(tok)
                vecs.append(vec)
        if dim is None:
            raise ValueError('no vectors found in %s' % path)
        table = np.zeros((len(self._idx_to_token), dim), dtype=np.float32)
        base = len(self._idx_to_token) - len(vecs)
        if vecs:
            table[base:] = np.asarray(vecs, dtype=np.float32)
        unk = np.asarray(loaded_unknown, dtype=np.float32) if loaded_unknown is not None else \
            init_unknown_vec(shape=(dim,)).asnumpy()
        table[:base] = unk           # unknown and reserved tokens
        self._idx_to_vec = nd.array(table)
        logging.info('loaded %d vectors of dimension %d from %s', len(vecs), dim, path)

    def _restrict_to(self, vocabulary, source):
        """Re-index onto ``vocabulary``'s tokens, taking vectors from the embedding(s) ``source``."""
        tokens = list(vocabulary.idx_to_token)
        blocks = [emb.get_vecs_by_tokens(tokens) for emb in source]     # before self is re-indexed
        self._unknown_token = vocabulary.unknown_token
        self._reserved_tokens = vocabulary.reserved_tokens
        self._idx_to_token = tokens
        self._token_to_idx = dict(vocabulary.token_to_idx)
        self._idx_to_vec = nd.concat(*blocks, dim=1) if len(blocks) > 1 else blocks[0]

    # ---------------------------------------------------------------- queries
    @property
    def vec_len(self):
        return self._idx_to_vec.shape[1]

    @property
    def idx_to_vec(self):
        return self._idx_to_vec

    def get_vecs_by_tokens(self, tokens, lower_case_backup=False):
        """Vectors of a token / list of tokens (unknown -> row 0; optional lower-case retry)."""
        single = not isinstance(tokens, list)
        toks = [tokens] if single else tokens
        idx = []
        for t in toks:
            i = self._token_to_idx.get(t)
            if i is None and lower_case_backup:
                i = self._token_to_idx.get(t.lower())
            idx.append(0 if i is None else i)
        vecs = nd.Embedding(nd.array(idx), self._idx_to_vec, input_dim=self._idx_to_vec.shape[0],
                            output_dim=self._idx_to_vec.shape[1])
        return vecs[0] if single else vecs

    def update_token_vectors(self, tokens, new_vectors):
        """Overwrite the vectors of known tokens."""
        toks = [tokens] if not isinstance(tokens, list) else tokens
        vecs = new_vectors if new_vectors.ndim == 2 else new_vectors.expand_dims(0)
        if vecs.shape != (len(toks), self.vec_len):
            raise AssertionError('new_vectors must have shape (%d, %d)' % (len(toks), self.vec_len))
        rows = []
        for t in toks:
            if t not in self._token_to_idx:
                raise ValueError('Token %s is unknown. To update the embedding vector for an unknown token, '
                                 'please specify it explicitly as the `unknown_token` %s.' % (t, self.unknown_token))
            rows.append(self._token_to_idx[t])
        self._idx_to_vec[nd.array(rows)] = vecs

    def __contains__(self, token):
        return token in self._token_to_idx

    def __getitem__(self, tokens):
        return self.get_vecs_by_tokens(tokens)


class _PretrainedFile(_TokenEmbedding):
    """Embedding read from a named pre-trained file under ``embedding_root``."""

    _subdir = ''

    def __init__(self, pretrained_file_name, embedding_root, init_unknown_vec, vocabulary, elem_delim=' ',
                 **kwargs):
        if pretrained_file_name not in self.pretrained_file_names:
            raise KeyError('Cannot find pretrained file %s for token embedding %s. Valid names: %s'
                           % (pretrained_file_name, type(self).__name__.lower(), ', '.join(self.pretrained_file_names)))
        super().__init__(**kwargs)
        root = os.path.expanduser(embedding_root)
        path = os.path.join(root, self._subdir, pretrained_file_name)
        if not os.path.exists(path):
            raise IOError('%s not found. There is no network access here: copy the pre-trained file there '
                          '(or use CustomEmbedding with its path).' % path)
        self._load_embedding(path, elem_delim, init_unknown_vec)
        if vocabulary is not None:
            self._restrict_to(vocabulary, [self])


@register
class GloVe(_PretrainedFile):
    pretrained_file_names = ('glove.42B.300d.txt', 'glove.6B.50d.txt', 'glove.6B.100d.txt', 'glove.6B.200d.txt',
                             'glove.6B.300d.txt', 'glove.840B.300d.txt', 'glove.twitter.27B.25d.txt',
                             'glove.twitter.27B.50d.txt', 'glove.twitter.27B.100d.txt',
                             'glove.twitter.27B.200d.txt')
    _subdir = 'glove'

    def __init__(self, pretrained_file_name='glove.840B.300d.txt',
                 embedding_root=os.path.join('~', '.mxnet', 'embeddings'), init_unknown_vec=nd.zeros,
                 vocabulary=None, **kwargs):
        super().__init__(pretrained_file_name, embedding_root, init_unknown_vec, vocabulary, **kwargs)


@register
class FastText(_PretrainedFile):
    pretrained_file_names = ('wiki.simple.vec', 'wiki.en.vec', 'crawl-300d-2M.vec', 'wiki-news-300d-1M.vec',
                             'wiki-news-300d-1M-subword.vec', 'cc.en.300.vec')
    _subdir = 'fasttext'

    def __init__(self, pretrained_file_name='wiki.simple.vec',
                 embedding_root=os.path.join('~', '.mxnet', 'embeddings'), init_unknown_vec=nd.zeros,
                 vocabulary=None, **kwargs):
        super().__init__(pretrained_file_name, embedding_root, init_unknown_vec, vocabulary, **kwargs)


class CustomEmbedding(_TokenEmbedding):
    """Embedding read from any file in the ``token<delim>v1<delim>v2...`` text format."""

    def __init__(self, pretrained_file_path, elem_delim=' ', encoding='utf8', init_unknown_vec=nd.zeros,
                 vocabulary=None, **kwargs):
        super().__init__(**kwargs)
        self._load_embedding(pretrained_file_path, elem_delim, init_unknown_vec, encoding)
        if vocabulary is not None:
            self._restrict_to(vocabulary, [self])


class CompositeEmbedding(_TokenEmbedding):
    """Vectors of several embeddings concatenated, indexed by ``vocabulary``."""

    def __init__(self, vocabulary, token_embeddings):
        embs = token_embeddings if isinstance(token_embeddings, list) else [token_embeddings]
        if not all(isinstance(e, _TokenEmbedding) for e in embs):
            raise AssertionError('token_embeddings must be token embedding instances')
        super().__init__(unknown_token=vocabulary.unknown_token, reserved_tokens=vocabulary.reserved_tokens)
        self._restrict_to(vocabulary, embs)
