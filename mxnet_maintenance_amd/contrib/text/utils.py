"""Token counting (API parity: contrib/text/utils.py)."""
import collections
import re

__all__ = ['count_tokens_from_str']


def count_tokens_from_str(source_str, token_delim=' ', seq_delim='\n', to_lower=False, counter_to_update=None):
    """Count the tokens of ``source_str`` (split on both delimiters) into a ``collections.Counter``."""
    pattern = '|'.join(re.escape(d) for d in (token_delim, seq_delim))
    tokens = [t for t in re.split(pattern, source_str) if t]
    if to_lower:
        tokens = [t.lower() for t in tokens]
    counter = counter_to_update if counter_to_update is not None else collections.Counter()
    counter.update(tokens)
    return counter
