"""Dice scoring engine: the process-wide device-resident template corpus and the batch API.

Mirrors what the reference memoizes per process (``License.all`` @all, license.rb:21, and
the ContentHelper ``@x ||=`` memos) with one ``dice_ctx`` per device. Everything that
scores goes through the HIP library (``_native.Scorer``); there is no CPU path.

    Dice#matches_by_similarity       lib/licensee/matchers/dice.rb:34-41
    Dice#match / #confidence         dice.rb:8-14,51-53 (batch form: ``match_files``)
    detect's licenses_by_similarity  commands/detect.rb:55-64,93-98 (``closest_files``)
    License#similarity(file)         content_helper.rb:128-133 (``pair_similarity``)
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

from . import config
from ._native import FileBatch, Scorer
from .corpus import TemplateCorpus
from .license import License


class DiceEngine:
    def __init__(self, templates: Optional[Sequence[License]] = None, device: int = 0):
        self.templates = list(templates) if templates is not None else License.all(hidden=True, pseudo=False)
        # key order positions (License objects); any other ContentHelper self (pair_similarity)
        # has no key and is only addressed by index
        self.position = {getattr(t, 'key', f'#{i}'): i for i, t in enumerate(self.templates)}
        self.corpus = TemplateCorpus(self.templates)
        c = self.corpus
        self.scorer = Scorer(c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc,
                             n_vocab=c.n_vocab, device=device)

    def intern(self, files: Sequence) -> FileBatch:
        return self.corpus.intern_files(files)

    def score_row(self, f) -> Tuple[List[int], List[float]]:
        ov, score, _, _ = self.scorer.matrix(self.intern([f]), 0)
        return ov[0].tolist(), score[0].tolist()

    def matches_by_similarity(self, f, potential: Sequence[License]) -> List[Tuple[License, float]]:
        _, scores = self.score_row(f)
        pairs = [(lic, scores[self.position[lic.key]]) for lic in potential]
        pairs.sort(key=lambda p: p[1])   # stable ascending, then reverse (dice.rb:39):
        pairs.reverse()                  # later key first among exact ties
        return pairs

    def licenses_by_similarity(self, f) -> List[Tuple[License, float]]:
        """The CLI's ranking (commands/detect.rb:93-98): every template, no CC filter."""
        return self.matches_by_similarity(f, self.templates)

    def closest_files(self, files: Sequence, k: int = 3) -> List[List[Tuple[License, float]]]:
        """Batched ``licenses_by_similarity(f)[0...k]`` (detect.rb:55-64, "Closest non-matching
        licenses") from the matrix kernel's top-k with the CC filter off."""
        fb = self.intern(files)
        fb.cc_false_positive[:] = 0
        _, _, idx, score = self.scorer.matrix(fb, k)
        return [[(self.templates[t], s) for t, s in zip(ri.tolist(), rs.tolist()) if t >= 0]
                for ri, rs in zip(idx, score)]

    def match_files(self, files: Sequence, threshold=None):
        """Batched ``Dice#match``/``#confidence``: list of (License or None, confidence)."""
        thr = config.confidence_threshold() if threshold is None else threshold
        best, _, score = self.scorer.match(self.intern(files), float(thr), confidence=True)
        return [(self.templates[b], s) if b >= 0 else (None, 0) for b, s in zip(best.tolist(), score.tolist())]


_engine: Optional[DiceEngine] = None


def default_engine() -> DiceEngine:
    global _engine
    if _engine is None:
        _engine = DiceEngine()
    return _engine


def reset_default_engine():
    global _engine
    if _engine is not None:
        _engine.scorer.close()
    _engine = None


def pair_similarity(a, b) -> float:
    """``a.similarity(b)`` for any two ContentHelper objects, scored on the GPU.

    A License in the default corpus reuses the resident context; any other ``a`` gets a
    one-template context (its own vocabulary, the simple length delta when it is not a
    License -- content_helper.rb:343)."""
    if isinstance(a, License) and not a.pseudo_license():
        eng = default_engine()
        if a.key in eng.position:
            _, row = eng.score_row(b)
            return row[eng.position[a.key]]
    eng = DiceEngine([a])
    try:
        _, row = eng.score_row(b)
        return row[0]
    finally:
        eng.scorer.close()


def precompile_default() -> str:
    """Build step: compile + cache the sparse program for the vendored corpus (no device)."""
    import ctypes

    from . import _native
    lib = _native.load_library()
    c = TemplateCorpus(License.all(hidden=True, pseudo=False))
    keep = [c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc]
    t = _native._Templates(len(c.lf_size), c.n_vocab, *[k.ctypes.data for k in keep])
    path = ctypes.create_string_buffer(1024)
    _native._check(lib.dice_precompile(ctypes.byref(t), path, 1024))
    return path.value.decode()
