"""Vocabulary: token <-> index maps (API parity: contrib/text/vocab.py).

Index 0 is the unknown token, then the reserved tokens, then counted tokens
by decreasing frequency (ties broken alphabetically), keeping at most
``most_freq_count`` of them with frequency >= ``min_freq``.
"""
__all__ = ['Vocabulary']


class Vocabulary:
    def __init__(self, counter=None, most_freq_count=None, min_freq=1, unknown_token='<unk>',
                 reserved_tokens=None):
        if min_freq <= 0:
            raise AssertionError('min_freq must be positive')
        reserved = list(reserved_tokens or [])
        if unknown_token in reserved:
            raise AssertionError('unknown_token must not be a reserved token')
        if len(set(reserved)) != len(reserved):
            raise AssertionError('reserved tokens must be unique')
        self._unknown_token = unknown_token
        self._reserved_tokens = reserved or None
        self._idx_to_token = [unknown_token] + reserved
        if counter is not None:
            ranked = sorted(counter.items(), key=lambda kv: (-kv[1], kv[0]))
            skip = set(self._idx_to_token)
            budget = len(ranked) if most_freq_count is None else most_freq_count
            for tok, freq in ranked:
                if budget <= 0 or freq < min_freq:
                    break
                if tok in skip:
                    continue
                self._idx_to_token.append(tok)
                budget -= 1
        self._token_to_idx = {t: i for i, t in enumerate(self._idx_to_token)}

    def __len__(self):
        return len(self._idx_to_token)

    @property
    def token_to_idx(self):
        return self._token_to_idx

    @property
    def idx_to_token(self):
        return self._idx_to_token

    @property
    def unknown_token(self):
        return self._unknown_token

    @property
    def reserved_tokens(self):
        return self._reserved_tokens

    def to_indices(self, tokens):
        """Index of a token (0 = unknown) or list of indices for a list of tokens."""
        if isinstance(tokens, list):
            return [self._token_to_idx.get(t, 0) for t in tokens]
        return self._token_to_idx.get(tokens, 0)

    def to_tokens(self, indices):
        single = not isinstance(indices, list)
        out = []
        for i in ([indices] if single else indices):
            if not isinstance(i, int) or not 0 <= i < len(self._idx_to_token):
                raise ValueError('Token index %s in the provided `indices` is invalid.' % i)
            out.append(self._idx_to_token[i])
        return out[0] if single else out
