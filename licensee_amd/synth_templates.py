"""Synthetic template corpus for BASELINE config 3 ("~600 SPDX templates").

No SPDX license texts exist offline, so ~550 derived templates are added to
the 47 real ones: each is a mixture of contiguous chunks of 1-3 real normalized templates
with a share of tokens replaced by words from a synthetic lexicon (growing the vocabulary
to ~10^4 words), alt segments = 0 and no fields. They behave like
License objects for TemplateCorpus / SyntheticCorpus (normalized space only).
"""
from __future__ import annotations

import random
from typing import List, Sequence

from .content_helper import FIELD_REGEX, WORDSET_REGEX


class SyntheticTemplate:
    def __init__(self, key: str, normalized: str):
        self.key = key
        self._normalized = normalized
        self._wordset = frozenset(WORDSET_REGEX.findall(normalized))
        self._fields = FIELD_REGEX.findall(normalized)

    def content_normalized(self, wrap=None):
        return self._normalized

    def wordset(self):
        return self._wordset

    def fields_normalized(self):
        return self._fields

    def wordset_fieldless(self):
        return self._wordset - frozenset(self._fields)

    def length(self):
        return len(self._normalized)

    def creative_commons(self):
        return False

    def has_spdx_alt_segments(self):
        return True

    def spdx_alt_segments(self):
        return 0


def _lexicon(n: int, rng: random.Random) -> List[str]:
    letters = 'abcdefghijklmnopqrstuvwxyz'
    out, seen = [], set()
    while len(out) < n:
        w = ''.join(rng.choice(letters) for _ in range(rng.randint(4, 10)))
        if w not in seen:
            seen.add(w)
            out.append(w)
    return out


def synthetic_templates(real: Sequence, total: int = 600, seed: int = 20250202, lexicon: int = 20000,
                        replace_frac: float = 0.3) -> List:
    """47 real templates + (total - len(real)) derived ones, in key order."""
    rng = random.Random(seed)
    lex = _lexicon(lexicon, rng)
    token_lists = [r.content_normalized().split(' ') for r in real]
    out = list(real)
    for i in range(total - len(real)):
        parts = []
        for _ in range(rng.randint(1, 3)):
            toks = token_lists[rng.randrange(len(token_lists))]
            size = min(len(toks), rng.randint(100, 800))
            start = rng.randrange(len(toks) - size + 1)
            parts.extend(toks[start:start + size])
        toks = [lex[rng.randrange(lexicon)] if rng.random() < replace_frac else t for t in parts]
        out.append(SyntheticTemplate(f'syn-{i:04d}', ' '.join(toks)))
    out.sort(key=lambda t: t.key)
    return out
