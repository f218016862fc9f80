"""Language-model corpora (parity: python/mxnet/gluon/contrib/data/text.py).

WikiText-2 / WikiText-103 token files are read from ``root`` (no network on
the target nodes); tokens are mapped through a vocabulary built on the
training split and served as (data, label) sequences of ``seq_len``.
"""
import io
import os

import numpy as np

from ...data.dataset import Dataset
from ....base import MXNetError


class _LMDataset(Dataset):
    _files = {}

    def __init__(self, root, segment='train', vocab=None, seq_len=35):
        self._root = os.path.expanduser(root)
        self._segment = segment
        self._seq_len = seq_len
        self._vocab = vocab
        fname = os.path.join(self._root, self._files[segment])
        if not os.path.exists(fname):
            raise MXNetError('%s not found (no network: place the WikiText files under %s)' % (fname, self._root))
        with io.open(fname, encoding='utf8') as f:
            tokens = [t for line in f for t in (line.split() + ['<eos>']) if line.strip()]
        if self._vocab is None:
            uniq = sorted(set(tokens))
            self._vocab = {t: i for i, t in enumerate(uniq)}
        unk = self._vocab.get('<unk>', 0)
        ids = np.array([self._vocab.get(t, unk) for t in tokens], dtype=np.int32)
        n = (len(ids) - 1) // seq_len
        self._data = ids[:n * seq_len].reshape(n, seq_len)
        self._label = ids[1:n * seq_len + 1].reshape(n, seq_len)

    @property
    def vocabulary(self):
        return self._vocab

    def __getitem__(self, idx):
        return self._data[idx], self._label[idx]

    def __len__(self):
        return len(self._label)


class WikiText2(_LMDataset):
    _files = {'train': 'wiki.train.tokens', 'validation': 'wiki.valid.tokens', 'test': 'wiki.test.tokens'}

    def __init__(self, root=os.path.join('~', '.mxnet', 'datasets', 'wikitext-2'), segment='train', vocab=None,
                 seq_len=35):
        super().__init__(root, segment, vocab, seq_len)


class WikiText103(_LMDataset):
    _files = {'train': 'wiki.train.tokens', 'validation': 'wiki.valid.tokens', 'test': 'wiki.test.tokens'}

    def __init__(self, root=os.path.join('~', '.mxnet', 'datasets', 'wikitext-103'), segment='train', vocab=None,
                 seq_len=35):
        super().__init__(root, segment, vocab, seq_len)
