"""Sentence encoding and the bucketing sentence iterator (API parity: python/mxnet/rnn/io.py).

``BucketSentenceIter`` groups variable-length integer sentences into buckets
(each sentence goes to the smallest bucket that fits it, padded with
``invalid_label``), shuffles within and across buckets per epoch, and emits
``DataBatch`` es whose ``bucket_key`` selects the unrolled graph in a
``BucketingModule``.  Labels are the inputs shifted left by one token.
"""
import bisect
import random

import numpy as np

from .. import ndarray as nd
from ..io import DataIter, DataBatch, DataDesc

__all__ = ['encode_sentences', 'BucketSentenceIter']


def encode_sentences(sentences, vocab=None, invalid_label=-1, invalid_key='\n', start_label=0,
                     unknown_token=None):
    """Map token lists to integer lists, building (or extending) ``vocab``; returns (encoded, vocab)."""
    grow = vocab is None
    if grow:
        vocab = {invalid_key: invalid_label}
    ids_from = [start_label]

    def fresh_id():
        if ids_from[0] == invalid_label:
            ids_from[0] += 1
        ids_from[0] += 1
        return ids_from[0] - 1

    encoded = []
    for sent in sentences:
        ids = []
        for tok in sent:
            if tok not in vocab:
                if not grow and unknown_token is None:
                    raise AssertionError('Unknown token %s' % tok)
                if unknown_token is not None:
                    tok = unknown_token            # unknown words share the unknown token's id
                if tok not in vocab:
                    vocab[tok] = fresh_id()
            ids.append(vocab[tok])
        encoded.append(ids)
    return encoded, vocab


class BucketSentenceIter(DataIter):
    """Bucketed, padded batches of integer sentences for language modelling."""

    def __init__(self, sentences, batch_size, buckets=None, invalid_label=-1, data_name='data',
                 label_name='softmax_label', dtype='float32', layout='NT'):
        super().__init__()
        if not buckets:
            # every length that occurs in at least one full batch worth of sentences
            lengths = np.bincount([len(s) for s in sentences])
            buckets = [n for n, c in enumerate(lengths) if c >= batch_size]
        buckets = sorted(buckets)
        self.data = [[] for _ in buckets]
        dropped = 0
        for sent in sentences:
            b = bisect.bisect_left(buckets, len(sent))
            if b == len(buckets):
                dropped += 1
                continue
            row = np.full((buckets[b],), invalid_label, dtype=dtype)
            row[:len(sent)] = sent
            self.data[b].append(row)
        self.data = [np.asarray(rows, dtype=dtype) for rows in self.data]
        if dropped:
            print('WARNING: discarded %d sentences longer than the largest bucket.' % dropped)
        self.batch_size = batch_size
        self.buckets = buckets
        self.data_name = data_name
        self.label_name = label_name
        self.dtype = dtype
        self.invalid_label = invalid_label
        self.layout = layout
        self.major_axis = layout.find('N')
        self.default_bucket_key = max(buckets)
        shape = (batch_size, self.default_bucket_key) if self.major_axis == 0 else \
            (self.default_bucket_key, batch_size)
        self.provide_data = [DataDesc(data_name, shape, layout=layout)]
        self.provide_label = [DataDesc(label_name, shape, layout=layout)]
        self.idx = [(b, start) for b, rows in enumerate(self.data)
                    for start in range(0, len(rows) - batch_size + 1, batch_size)]
        self.curr_idx = 0
        self.nddata = []
        self.ndlabel = []
        self.reset()

    def reset(self):
        self.curr_idx = 0
        random.shuffle(self.idx)
        self.nddata, self.ndlabel = [], []
        for rows in self.data:
            np.random.shuffle(rows)
            label = np.full_like(rows, self.invalid_label)
            if rows.size:
                label[:, :-1] = rows[:, 1:]
            self.nddata.append(nd.array(rows, dtype=self.dtype))
            self.ndlabel.append(nd.array(label, dtype=self.dtype))

    def next(self):
        if self.curr_idx == len(self.idx):
            raise StopIteration
        b, start = self.idx[self.curr_idx]
        self.curr_idx += 1
        data = self.nddata[b][start:start + self.batch_size]
        label = self.ndlabel[b][start:start + self.batch_size]
        if self.major_axis == 1:
            data, label = data.T, label.T
        return DataBatch([data], [label], pad=0, bucket_key=self.buckets[b],
                         provide_data=[DataDesc(self.data_name, data.shape, layout=self.layout)],
                         provide_label=[DataDesc(self.label_name, label.shape, layout=self.layout)])
