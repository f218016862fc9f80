"""Text utilities: token counting, vocabularies and token embeddings (``mx.contrib.text``).

API parity: python/mxnet/contrib/text/ (utils.py, vocab.py, embedding.py).
"""
from . import utils, vocab, embedding  # noqa: F401
