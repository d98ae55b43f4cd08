"""Matchers on the LicenseFile path: Copyright and Exact stay on the CPU (north star);
Dice scores on the GPU through ``licensee_amd.dice``.

    Matcher base / potential_matches   lib/licensee/matchers/matcher.rb:11-31
    Copyright                          lib/licensee/matchers/copyright.rb:8-23
    Exact                              lib/licensee/matchers/exact.rb:6-16
    Dice                               lib/licensee/matchers/dice.rb:8-59
"""
from __future__ import annotations

from typing import List, Optional, Tuple

from . import config
from .content_helper import COPYRIGHT_MATCH_REGEX, ruby_strip
from .license import License


class Matcher:
    def __init__(self, file):
        self.file = file

    @property
    def name(self) -> str:
        return type(self).__name__.lower()

    def potential_matches(self) -> List[License]:
        return License.all(hidden=True, pseudo=False)

    def to_h(self):
        return {'name': self.name, 'confidence': self.confidence()}


class Copyright(Matcher):
    def match(self) -> Optional[License]:
        if COPYRIGHT_MATCH_REGEX.search(ruby_strip(self.file.content)):
            return License.find('no-license')
        return None

    def confidence(self):
        return 100


class Exact(Matcher):
    def match(self) -> Optional[License]:
        if not hasattr(self, '_match'):
            ws = self.file.wordset()
            self._match = next((l for l in self.potential_matches() if l.wordset() == ws), None)
        return self._match

    def confidence(self):
        return 100


class Dice(Matcher):
    """GPU-scored. ``matches_by_similarity`` comes from the HIP similarity-matrix kernel."""

    def potential_matches(self) -> List[License]:
        if not hasattr(self, '_potential'):
            fp = self.file.potential_false_positive()
            # dice.rb:28 `license.wordset` excludes only nil: an empty Set is truthy in Ruby
            self._potential = [l for l in super().potential_matches()
                               if not (l.creative_commons() and fp) and l.wordset() is not None]
        return self._potential

    potential_licenses = potential_matches

    def matches_by_similarity(self) -> List[Tuple[License, float]]:
        if not hasattr(self, '_mbs'):
            from .dice import default_engine
            self._mbs = default_engine().matches_by_similarity(self.file, self.potential_matches())
        return self._mbs

    licenses_by_similarity = matches_by_similarity

    def matches(self) -> List[Tuple[License, float]]:
        thr = config.confidence_threshold()
        return [m for m in self.matches_by_similarity() if m[1] >= thr]

    def match(self) -> Optional[License]:
        ms = self.matches()
        return ms[0][0] if ms else None

    def confidence(self):
        ms = self.matches()
        return ms[0][1] if ms else 0
