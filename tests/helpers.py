"""Shared test helpers: seeded candidate files in normalized space + oracle comparison."""
from __future__ import annotations

import random
from typing import List, Sequence

import numpy as np

from licensee_amd.synth import IPSUM_WORDS
from oracle import dice_oracle as O

# the reference's filler list (spec/fixtures/ipsum.txt via licensee_amd/data/ipsum.json)
IPSUM = IPSUM_WORDS


class NormFile:
    """A candidate file given directly as normalized text (the Dice input space)."""

    def __init__(self, text: str, cc: bool = False):
        self.text = text
        self.cc = cc
        self._of = O.OracleFile(text)

    def wordset(self):
        return self._of.wordset

    def length(self):
        return len(self.text)

    def potential_false_positive(self):
        return self.cc

    @property
    def oracle(self):
        return self._of


def perturb(words: List[str], rng: random.Random, inserts: int, drop_frac: float) -> List[str]:
    out = [w for w in words if rng.random() >= drop_frac]
    for _ in range(inserts):
        out.insert(rng.randrange(len(out) + 1), rng.choice(IPSUM))
    return out


def make_files(templates: Sequence, n: int, seed: int, cc_rate: float = 0.05) -> List[NormFile]:
    """Files derived from random templates: 0-5 / 75 inserted ipsum words (spec_helper.rb:82-91,
    vendored_license_spec.rb:41), 0-5% dropped words, a few mixtures and empties."""
    rng = random.Random(seed)
    files = []
    for i in range(n):
        kind = rng.random()
        base = templates[rng.randrange(len(templates))].content_normalized().split(' ')
        if kind < 0.02:
            words = []
        elif kind < 0.06:
            other = templates[rng.randrange(len(templates))].content_normalized().split(' ')
            words = base + other
        elif kind < 0.5:
            words = perturb(base, rng, rng.randint(0, 5), 0.0)
        elif kind < 0.9:
            words = perturb(base, rng, rng.randint(0, 5), rng.random() * 0.05)
        else:
            words = perturb(base, rng, 75, 0.0)
        files.append(NormFile(' '.join(words), cc=rng.random() < cc_rate))
    return files


def oracle_templates(templates) -> List[O.OracleTemplate]:
    return [O.OracleTemplate(l.key, l.content_normalized(), l.spdx_alt_segments()) for l in templates]


class ArrayCorpus:
    """Per-template constants given directly as arrays (the ``dice_templates`` fields), for
    corpora no License list produces -- e.g. one outside the sparse program's fast envelope."""

    def __init__(self, lf_bits, lf_size, fields_set_size, length_slack, length, is_cc, n_vocab):
        self.lf_bits = np.ascontiguousarray(lf_bits, np.uint64)
        self.lf_size = np.ascontiguousarray(lf_size, np.uint32)
        self.fields_set_size = np.ascontiguousarray(fields_set_size, np.uint32)
        self.length_slack = np.ascontiguousarray(length_slack, np.int32)
        self.length = np.ascontiguousarray(length, np.int32)
        self.is_cc = np.ascontiguousarray(is_cc, np.uint8)
        self.n_vocab = int(n_vocab)
        self.w64 = (self.n_vocab + 63) // 64

    @classmethod
    def of(cls, corpus):
        return cls(corpus.lf_bits.copy(), corpus.lf_size.copy(), corpus.fields_set_size.copy(),
                   corpus.length_slack.copy(), corpus.length.copy(), corpus.is_cc.copy(), corpus.n_vocab)

    def arrays(self):
        return (self.lf_bits, self.lf_size, self.fields_set_size, self.length_slack, self.length, self.is_cc)


def outside_fast_envelope(corpus) -> ArrayCorpus:
    """The corpus with three templates moved outside ``corpus_in_fast_envelope``
    (dice_program.cpp): |Lf| - |Fld| = 1 (200 |Lf| >= 1024 base: scores may reach 200), and a
    template length >= 2^20 characters. The formula is unchanged (content_helper.rb:128-133)."""
    c = ArrayCorpus.of(corpus)
    order = np.argsort(-c.lf_size.astype(np.int64), kind='stable')
    for j in order[:2]:
        c.fields_set_size[j] = c.lf_size[j] - 1
    c.length[order[2]] = (1 << 20) + 12345
    return c


def widen_lanes(fb, seed: int, frac: float = 0.15):
    """Move a fraction of the files outside the fast envelope (|W_F| >= 2^20 and/or
    len_F >= 2^21, as a file with a million out-of-vocabulary words would have), scattered so
    most 64-file waves mix fast and slow lanes. Values stay where the int32 denominator
    base + |W_F| + adj/4 cannot overflow. Returns the modified copy and the changed indices."""
    from licensee_amd._native import FileBatch
    rng = np.random.default_rng(seed)
    n = fb.n
    idx = np.nonzero(rng.random(n) < frac)[0]
    wf = fb.wordset_size.copy()
    ln = fb.length.copy()
    kind = rng.integers(0, 3, idx.size)
    big_wf = (1 << 20) + rng.integers(0, 1 << 24, idx.size)
    big_len = (1 << 21) + rng.integers(0, 1 << 26, idx.size)
    wf[idx] = np.where(kind != 1, big_wf, wf[idx]).astype(np.uint32)
    ln[idx] = np.where(kind != 0, big_len, ln[idx]).astype(np.int32)
    return FileBatch(fb.bits.copy(), wf, ln, fb.cc_false_positive.copy()), idx
