"""ORACLE -- test infrastructure only. CPU restatement of licensee's Dice scoring.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module; the product path (``licensee_amd``) never does and has no CPU
fallback. This is the checker, never the thing measured or shipped.

It restates, over plain Python sets of word *strings* (mirroring Ruby ``Set``):

    wordset scan            lib/licensee/content_helper.rb:108-110
    fields_normalized(_set) lib/licensee/content_helper.rb:328-335, license_field.rb:50
    wordset_fieldless       lib/licensee/content_helper.rb:323-325
    similarity              lib/licensee/content_helper.rb:128-133  (Set#& then Float/Integer)
    variation_adjusted_...  lib/licensee/content_helper.rb:337-347
    potential_matches       lib/licensee/matchers/dice.rb:23-31 (CC filter, license_file.rb:63-65,80-82)
    matches_by_similarity   lib/licensee/matchers/dice.rb:34-41 (sort_by.reverse)
    matches / match         lib/licensee/matchers/dice.rb:8-14,44-48
    confidence              lib/licensee/matchers/dice.rb:51-53 (Integer 0 when no match)

Inputs are *normalized* texts (``content_normalized``). Normalization itself is pinned
directly by the reference goldens (license-hashes.json, fixtures.yml) in
tests/test_normalize.py, so the oracle starts from normalized strings.

Parity pinning: ``spec/licensee/matchers/dice_matcher_spec.rb:23-31`` golden floats
(100.0, 94.56967213114754, 26.821370750134918) and the 19 ``matcher: dice`` rows of
``spec/fixtures/fixtures.yml`` -- see tests/test_oracle.py.

Tie rule (parity-unpinned, SURVEY.md §7 hard part 2): Ruby's ``sort_by`` is not stable;
this oracle uses a stable ascending sort followed by ``reverse`` -- among exactly equal
scores the template later in key order ranks first. The HIP kernels implement the same rule.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import FrozenSet, List, Optional, Sequence, Tuple

WORD_RE = re.compile(r"(?:[A-Za-z0-9_/-](?:'s|(?<=s)')?)+")               # content_helper.rb:109
FIELD_RE = re.compile(r'\[(fullname|login|email|project|description|year|projecturl)\]')  # license_field.rb:50
CC_FALSE_POSITIVE_RE = re.compile(r'^(creative commons )?Attribution-(NonCommercial|NoDerivatives)',
                                  re.I | re.M)                              # license_file.rb:63-65
DEFAULT_THRESHOLD = 98                                                      # licensee.rb:21


@dataclass(frozen=True)
class OracleTemplate:
    key: str
    normalized: str
    alt_segments: int
    wordset: FrozenSet[str] = field(init=False)
    fields: Tuple[str, ...] = field(init=False)
    fieldless: FrozenSet[str] = field(init=False)

    def __post_init__(self):
        ws = frozenset(WORD_RE.findall(self.normalized))
        flds = tuple(FIELD_RE.findall(self.normalized))
        object.__setattr__(self, 'wordset', ws)
        object.__setattr__(self, 'fields', flds)
        object.__setattr__(self, 'fieldless', ws - frozenset(flds))

    @property
    def length(self) -> int:
        return len(self.normalized)

    @property
    def is_cc(self) -> bool:
        return self.key.startswith('cc-')                                   # license.rb:209-212


@dataclass(frozen=True)
class OracleFile:
    normalized: str
    raw_stripped: str = ''     # content.strip, for potential_false_positive?
    wordset: FrozenSet[str] = field(init=False)

    def __post_init__(self):
        object.__setattr__(self, 'wordset', frozenset(WORD_RE.findall(self.normalized)))

    @property
    def length(self) -> int:
        return len(self.normalized)

    @property
    def potential_false_positive(self) -> bool:
        return CC_FALSE_POSITIVE_RE.search(self.raw_stripped) is not None


def overlap(template: OracleTemplate, wordset: FrozenSet[str]) -> int:
    """``(wordset_fieldless & other.wordset).size`` -- Set#& iterates the smaller set."""
    a, b = template.fieldless, wordset
    small, big = (a, b) if len(a) <= len(b) else (b, a)
    return sum(1 for w in small if w in big)


def adjusted_delta(template: OracleTemplate, file_length: int) -> int:
    """content_helper.rb:337-347 with License self (spdx_alt_segments present)."""
    delta = abs(template.length - file_length)
    adjusted = delta - max(len(template.fields), template.alt_segments) * 5
    return adjusted if adjusted > 0 else 0


def denominator(template: OracleTemplate, wf_size: int, file_length: int) -> int:
    total = len(template.fieldless) + wf_size - len(set(template.fields))
    return total + adjusted_delta(template, file_length) // 4


def similarity_parts(template: OracleTemplate, f: OracleFile) -> Tuple[int, int, float]:
    ov = overlap(template, f.wordset)
    den = denominator(template, len(f.wordset), f.length)
    return ov, den, (ov * 200.0) / den


def similarity(template: OracleTemplate, f: OracleFile) -> float:
    return similarity_parts(template, f)[2]


def potential_matches(templates: Sequence[OracleTemplate], f: OracleFile) -> List[int]:
    fp = f.potential_false_positive
    return [i for i, t in enumerate(templates) if not (t.is_cc and fp)]


def matches_by_similarity(templates: Sequence[OracleTemplate], f: OracleFile,
                          cc_fp: Optional[bool] = None) -> List[Tuple[int, float]]:
    """dice.rb:34-41. ``templates`` must be in ``License.all`` key order."""
    fp = f.potential_false_positive if cc_fp is None else cc_fp
    scored = [(i, similarity(t, f)) for i, t in enumerate(templates) if not (t.is_cc and fp)]
    scored.sort(key=lambda p: p[1])          # stable ascending ...
    scored.reverse()                         # ... reversed: later key first among ties
    return scored


def match(templates: Sequence[OracleTemplate], f: OracleFile, threshold=DEFAULT_THRESHOLD,
          cc_fp: Optional[bool] = None) -> Tuple[int, object]:
    """Returns (template index or -1, confidence) -- dice.rb:8-14,44-53."""
    ms = [p for p in matches_by_similarity(templates, f, cc_fp) if p[1] >= threshold]
    if not ms:
        return -1, 0
    return ms[0]


def best_argmax(ov_den: Sequence[Tuple[int, int]], allowed: Sequence[bool]) -> int:
    """Exact-rational argmax with the oracle tie rule (later index wins on equality)."""
    best = -1
    for i, (ov, den) in enumerate(ov_den):
        if not allowed[i]:
            continue
        if best < 0 or (ov * 200.0) / den >= (ov_den[best][0] * 200.0) / ov_den[best][1]:
            best = i
    return best
