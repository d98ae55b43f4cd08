"""Shared test helpers: seeded candidate files in normalized space + oracle comparison."""
from __future__ import annotations

import random
from typing import List, Sequence

from oracle import dice_oracle as O

IPSUM = ('lorem ipsum dolor sit amet consectetur adipiscing elit sed do eiusmod tempor incididunt ut '
         'labore et dolore magna aliqua enim ad minim veniam quis nostrud exercitation ullamco laboris '
         'nisi aliquip ex ea commodo consequat duis aute irure in reprehenderit voluptate velit esse '
         'cillum fugiat nulla pariatur excepteur sint occaecat cupidatat non proident sunt culpa qui '
         "officia deserunt mollit anim id est laborum software license's licensor's").split()


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
