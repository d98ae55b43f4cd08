"""Batched LicenseFile#license / #confidence / matcher over many files.

The reference evaluates ``[Copyright, Exact, Dice].map(new).find(&:match)`` per file
(license_file.rb:67-69, project_file.rb:69-80) and falls back to ``License 'other'``
(license_file.rb:92-98). Here the whole chain runs in bulk:

  host (liblicensee_host.so, threads): decode, content_normalized, Copyright, the CC flag
  GPU  (liblicensee_dice.so):          the wordset scan + vocabulary bitsets + field-word
                                       masks (dice_batch_upload_text, content_helper.rb:108-110),
                                       Exact#match (dice_batch_exact: |W_F| == |W_t| and
                                       W_t ⊆ W_F, exact.rb:6-12) and Dice#match / #confidence
                                       on the same resident batch
(``wordset_on='host'`` scans and interns in the host threads instead, the round-5 split;
``exact_on='host'`` keeps Exact in the host threads too, the round-2 split.)

Results equal the per-file Python chain (tests/test_gpu_golden.py::test_batch_chain).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Iterable, Iterator, List, Optional, Sequence, Tuple, Union

from . import config
from .license import License


@dataclass(slots=True)
class Detection:
    license: License            # matched License, or License 'other'
    matcher: Optional[str]      # 'copyright' | 'exact' | 'dice' | None
    confidence: object          # 100 (copyright/exact), Float (dice), None (no matcher)


class BatchDetector:
    """One resident template corpus on the device + one native host context.

    ``engine`` defaults to the process-wide :func:`dice.default_engine` (the vendored
    corpus); pass a :class:`dice.DiceEngine` to use another corpus or device."""

    def __init__(self, engine=None, nthreads: int = 8, exact_on: str = 'device', wordset_on: str = 'device'):
        from .dice import default_engine
        from .native_host import HostPrep
        if exact_on not in ('device', 'host'):
            raise ValueError("exact_on is 'device' or 'host'")
        if wordset_on not in ('device', 'host'):
            raise ValueError("wordset_on is 'device' or 'host'")
        self.engine = engine if engine is not None else default_engine()
        self.host = HostPrep(self.engine.corpus)
        self.nthreads = nthreads
        self.exact_on = exact_on if self.host.field_need is not None else 'host'
        # the device scan reports the non-vocabulary field words as mask bits for device Exact
        self.wordset_on = wordset_on if self.exact_on == 'device' else 'host'
        self._batch = None          # one device batch, reused by every detect() and grown on demand
        self._pinned = [None, None]  # page-locked text buffers: batch k uploads from one while k + 1 fills the other
        self._turn = 0
        if self.exact_on == 'device':
            self.engine.scorer.exact_setup(*exact_tables(self.engine.corpus, self.host))
        if self.wordset_on == 'device':
            self.engine.scorer.vocab_setup(self.engine.corpus.vocab, self.host.nv_fields)

    def _device_batch(self, n: int):
        if self._batch is None or self._batch.capacity < n:
            if self._batch is not None:
                self._batch.close()
            cap = max(n, 64) if self._batch is None else max(n, 2 * self._batch.capacity)
            self._batch = self.engine.scorer.batch(cap)
        return self._batch

    def close(self):
        if self._batch is not None:
            self._batch.close()
            self._batch = None
        for i, p in enumerate(self._pinned):
            if p is not None:
                p.close()
                self._pinned[i] = None

    def _text_buffer(self, nbytes: int):
        """The next page-locked text buffer (alternating, grown on demand)."""
        from ._native import PinnedBuffer
        i = self._turn
        self._turn ^= 1
        p = self._pinned[i]
        if p is None or p.nbytes < nbytes:
            if p is not None:
                p.close()
            p = self._pinned[i] = PinnedBuffer(max(nbytes, 2 * p.nbytes if p is not None else nbytes))
        return p.array

    def detect(self, contents: Sequence[Union[str, bytes]], filenames: Optional[Sequence[str]] = None,
               threshold=None) -> List[Detection]:
        thr = config.confidence_threshold() if threshold is None else threshold
        return self._score(self._prep(contents, filenames), thr)

    def detect_stream(self, batches: Iterable[Tuple[Sequence[Union[str, bytes]], Optional[Sequence[str]]]],
                      threshold=None) -> Iterator[List[Detection]]:
        """detect() over a stream of (contents, filenames) batches as a two-stage pipeline: the
        native host threads prepare batch k + 1 (decode, normalize, intern, Copyright) while batch
        k is uploaded, matched on the device and turned into Detections. Yields one list per batch,
        in order, each equal to detect() of that batch."""
        from concurrent.futures import ThreadPoolExecutor
        thr = config.confidence_threshold() if threshold is None else threshold
        it = iter(batches)
        with ThreadPoolExecutor(1) as ex:
            nxt = next(it, None)
            fut = ex.submit(self._prep, *nxt) if nxt is not None else None
            while fut is not None:
                prepped = fut.result()
                nxt = next(it, None)
                fut = ex.submit(self._prep, *nxt) if nxt is not None else None
                yield self._score(prepped, thr)

    def _prep(self, contents, filenames=None):
        """Host stage (liblicensee_host.so threads; ctypes releases the GIL during the call)."""
        if self.wordset_on == 'device':
            return ('text', self.host.normalize_files(contents, filenames, nthreads=self.nthreads,
                                                      out=self._text_buffer), contents, filenames)
        field_masks = self.exact_on == 'device'
        fb, copyright, third, _ = self.host.prep_files(contents, filenames, nthreads=self.nthreads,
                                                       field_masks=field_masks)
        return fb, copyright, third

    def _score_text(self, prepped, thr):
        """Device stage of wordset_on='device': upload the normalized texts (the device scans and
        interns the wordsets), patch the rare files whose distinct non-vocabulary words overflow
        the device set with host-prepared rows, then Exact + Dice#match/#confidence."""
        import numpy as np
        _, (text, off, tl, ln, cc, copyright, _), contents, filenames = prepped
        n = len(off)
        b = self._device_batch(max(n, 1))
        st = b.upload_text(text, off, tl, ln, cc)
        over = np.nonzero(st)[0]
        if over.size:
            sub = [contents[i] for i in over]
            sfn = [filenames[i] for i in over] if filenames is not None else None
            fb, _, fm, _ = self.host.prep_files(sub, sfn, nthreads=self.nthreads, field_masks=True)
            b.set_rows(over, fb.bits, fb.wordset_size, fm)
        b.exact(None)
        b.match(float(thr), confidence=True)
        exact = b.download_exact()
        best, _, score = b.download_match()
        return copyright, exact, best, score

    def _score(self, prepped, thr) -> List[Detection]:
        """Device stage: Exact (device) + Dice#match/#confidence, then the matcher chain's order."""
        if prepped[0] == 'text':
            copyright, exact, best, score = self._score_text(prepped, thr)
            return self._detections(copyright, exact, best, score)
        fb, copyright, third = prepped
        if self.exact_on == 'device':
            b = self._device_batch(max(fb.n, 1))
            b.upload(fb)
            b.exact(third)
            b.match(float(thr), confidence=True)
            exact = b.download_exact()
            best, _, score = b.download_match()
        else:
            exact = third
            best, _, score = self.engine.scorer.match(fb, float(thr), confidence=True)
        return self._detections(copyright, exact, best, score)

    def _detections(self, copyright, exact, best, score) -> List[Detection]:
        templates = self.engine.templates
        no_license, other = License.find('no-license'), License.find('other')
        # the matcher chain's order per file (Copyright, Exact, Dice, else 'other'), over Python lists
        # (numpy scalar indexing per file cost as much as the host preparation of the next batch);
        # the cyclic collector paused while the batch's objects are made (they hold no cycles, and
        # in a process with a large heap its passes cost more than the objects themselves)
        import gc
        paused = gc.isenabled()
        gc.disable()
        try:
            return [Detection(no_license, 'copyright', 100) if c else
                    Detection(templates[e], 'exact', 100) if e >= 0 else
                    Detection(templates[bi], 'dice', sc) if bi >= 0 else
                    Detection(other, None, None)
                    for c, e, bi, sc in zip(copyright.tolist(), exact.tolist(), best.tolist(), score.tolist())]
        finally:
            if paused:
                gc.enable()


def exact_tables(corpus, host):
    """dice_exact_setup's tables for a TemplateCorpus: |wordset| per template, its field words
    that are vocabulary words as bitsets, the others as bits of ``host.nv_fields``
    (content_helper.rb:323-335: wordset = wordset_fieldless + the field words)."""
    import numpy as np
    T = len(corpus.templates)
    bits = np.zeros((T, corpus.w64), np.uint64)
    for t, tpl in enumerate(corpus.templates):
        for w in set(tpl.fields_normalized()):
            i = corpus.index.get(w)
            if i is not None:
                bits[t, i >> 6] |= np.uint64(1 << (i & 63))
    return host._ws, bits, host.field_need
