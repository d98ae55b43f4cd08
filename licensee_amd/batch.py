"""Batched LicenseFile#license / #confidence / matcher over many files.

The reference evaluates ``[Copyright, Exact, Dice].map(new).find(&:match)`` per file
(license_file.rb:67-69, project_file.rb:69-80) and falls back to ``License 'other'``
(license_file.rb:92-98). Here the whole chain runs in bulk:

  host (liblicensee_host.so, threads): decode, normalize, intern, Copyright, Exact
  GPU  (liblicensee_dice.so):          Dice#match / #confidence for the files left

Results equal the per-file Python chain (tests/test_gpu_golden.py::test_batch_chain).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence, Union

from . import config
from .license import License


@dataclass
class Detection:
    license: License            # matched License, or License 'other'
    matcher: Optional[str]      # 'copyright' | 'exact' | 'dice' | None
    confidence: object          # 100 (copyright/exact), Float (dice), None (no matcher)


class BatchDetector:
    """One resident template corpus on the device + one native host context.

    ``engine`` defaults to the process-wide :func:`dice.default_engine` (the vendored
    corpus); pass a :class:`dice.DiceEngine` to use another corpus or device."""

    def __init__(self, engine=None, nthreads: int = 8):
        from .dice import default_engine
        from .native_host import HostPrep
        self.engine = engine if engine is not None else default_engine()
        self.host = HostPrep(self.engine.corpus)
        self.nthreads = nthreads

    def detect(self, contents: Sequence[Union[str, bytes]], filenames: Optional[Sequence[str]] = None,
               threshold=None) -> List[Detection]:
        thr = config.confidence_threshold() if threshold is None else threshold
        fb, copyright, exact, _ = self.host.prep_files(contents, filenames, nthreads=self.nthreads)
        best, _, score = self.engine.scorer.match(fb, float(thr))
        templates = self.engine.templates
        no_license, other = License.find('no-license'), License.find('other')
        out = []
        for i in range(len(contents)):
            if copyright[i]:
                out.append(Detection(no_license, 'copyright', 100))
            elif exact[i] >= 0:
                out.append(Detection(templates[exact[i]], 'exact', 100))
            elif best[i] >= 0:
                out.append(Detection(templates[best[i]], 'dice', float(score[i])))
            else:
                out.append(Detection(other, None, None))
        return out
