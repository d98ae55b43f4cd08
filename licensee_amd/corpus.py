"""Host interning: word sets -> bitsets over the template vocabulary.

The template vocabulary V is the union of every template's ``wordset_fieldless``
(content_helper.rb:323-325). A file's wordset (content_helper.rb:108-110) is interned to a
V-bit bitset; words outside V can never overlap a template and only count towards
|W_F| (``other.wordset.size``, content_helper.rb:130).

Vocabulary order is free (any bijection gives identical overlaps), so it is chosen for the
device: words are grouped by their template-membership signature, which clusters each
template's words into few 32-bit dwords and keeps the sparse scoring program short
(DESIGN.md "sparse program").
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Sequence, Tuple

import numpy as np

from ._native import FileBatch, words64


class TemplateCorpus:
    """Per-template constants + vocabulary for a key-ordered template list.

    ``templates`` items need: ``wordset_fieldless()``, ``fields_normalized()``,
    ``length()``, ``creative_commons()`` and either ``spdx_alt_segments()`` (License self)
    or nothing (simple delta, content_helper.rb:343)."""

    def __init__(self, templates: Sequence):
        self.templates = list(templates)
        lfs = [t.wordset_fieldless() for t in self.templates]
        members: Dict[str, List[int]] = {}
        for i, lf in enumerate(lfs):
            for w in lf:
                members.setdefault(w, []).append(i)
        # signature order: templates containing the word, then the word itself (determinism)
        self.vocab: List[str] = sorted(members, key=lambda w: (tuple(members[w]), w))
        self.index: Dict[str, int] = {w: i for i, w in enumerate(self.vocab)}
        V = max(len(self.vocab), 1)
        self.n_vocab = V
        self.w64 = words64(V)
        T = len(self.templates)
        self.lf_bits = np.zeros((T, self.w64), np.uint64)
        for i, lf in enumerate(lfs):
            self.lf_bits[i] = self.bits_of_ids([self.index[w] for w in lf])
        self.lf_size = np.array([len(lf) for lf in lfs], np.uint32)
        self.fields_set_size = np.array([len(set(t.fields_normalized())) for t in self.templates], np.uint32)
        slack = []
        for t in self.templates:
            if t.has_spdx_alt_segments():
                slack.append(5 * max(len(t.fields_normalized()), t.spdx_alt_segments()))
            else:
                slack.append(-1)
        self.length_slack = np.array(slack, np.int32)
        self.length = np.array([t.length() for t in self.templates], np.int32)
        self.is_cc = np.array([1 if getattr(t, 'creative_commons', lambda: False)() else 0
                               for t in self.templates], np.uint8)

    def bits_of_ids(self, ids: Iterable[int]) -> np.ndarray:
        row = np.zeros(self.w64, np.uint64)
        ids = np.fromiter(ids, dtype=np.int64)
        if ids.size:
            np.bitwise_or.at(row, ids >> 6, np.left_shift(np.uint64(1), (ids & 63).astype(np.uint64)))
        return row

    def intern(self, wordset) -> Tuple[np.ndarray, int]:
        ids = [self.index[w] for w in wordset if w in self.index]
        return self.bits_of_ids(ids), len(wordset)

    def intern_files(self, files: Sequence) -> FileBatch:
        """``files`` items need ``wordset()``, ``length()`` and ``potential_false_positive()``."""
        n = len(files)
        bits = np.zeros((n, self.w64), np.uint64)
        wf = np.zeros(n, np.uint32)
        ln = np.zeros(n, np.int32)
        cc = np.zeros(n, np.uint8)
        for i, f in enumerate(files):
            ws = f.wordset() or frozenset()
            bits[i], wf[i] = self.intern(ws)
            ln[i] = f.length()
            cc[i] = 1 if getattr(f, 'potential_false_positive', lambda: False)() else 0
        return FileBatch(bits, wf, ln, cc)
