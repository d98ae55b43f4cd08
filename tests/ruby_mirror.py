"""Statement-for-statement Python restatement of the Ruby FFI binding in INTEGRATION.md §3
(`Licensee::GpuDice`), over the same C-ABI through ctypes (Ruby's FFI gem stands in as ctypes).

Ruby is not in this image, so the binding cannot run; this mirror runs its logic -- corpus
construction with first-seen vocabulary numbering, the n = 1 similarity-matrix call and the
stable-ascending-then-reversed ranking of `matches_by_similarity`, the batched `match`, and the
Copyright -> Exact -> GPU Dice `detect` chain -- so tests/test_gpu_ruby_mirror.py can check it
against the product path. Test infrastructure only.
"""
from __future__ import annotations

import ctypes

import numpy as np

from licensee_amd import _native
from licensee_amd.license import License


class Error(RuntimeError):
    pass


class GpuDice:
    """module Licensee::GpuDice"""
    _corpus = None

    @classmethod
    def corpus(cls):
        # def self.corpus; @corpus ||= Corpus.new; end
        if cls._corpus is None:
            cls._corpus = Corpus()
        return cls._corpus

    @classmethod
    def reset(cls):
        if cls._corpus is not None:
            cls._corpus.close()
        cls._corpus = None


def _u32(a):
    return np.ascontiguousarray(np.array(a if len(a) else [0], dtype=np.uint32))


def _i32(a):
    return np.ascontiguousarray(np.array(a if len(a) else [0], dtype=np.int32))


def _u8(a):
    return np.ascontiguousarray(np.array(a if len(a) else [0], dtype=np.uint8))


class Corpus:
    """class Licensee::GpuDice::Corpus"""

    def __init__(self, licenses=None, device=0):
        lib = _native.load_library()
        if licenses is None:
            licenses = License.all(hidden=True, pseudo=False)   # Licensee.licenses(hidden: true, psuedo: false)
        self.licenses = list(licenses)
        self.index = {l.key: i for i, l in enumerate(self.licenses)}
        # @vocab: first-seen numbering of the templates' wordset_fieldless
        self.vocab = {}
        for l in self.licenses:
            for w in sorted(l.wordset_fieldless()):   # Ruby Set iterates in insertion order; any order works
                if w not in self.vocab:
                    self.vocab[w] = len(self.vocab)
        self.w64 = lib.dice_words64(max(len(self.vocab), 1))
        t = len(self.licenses)
        bits = np.zeros(t * self.w64, np.uint64)
        for i, l in enumerate(self.licenses):
            self._put_bits(bits, i, l.wordset_fieldless())
        self._keep = [bits,
                      _u32([len(l.wordset_fieldless()) for l in self.licenses]),
                      _u32([len(l.fields_normalized_set()) for l in self.licenses]),
                      _i32([5 * max(len(l.fields_normalized()), l.spdx_alt_segments()) for l in self.licenses]),
                      _i32([l.length() for l in self.licenses]),
                      _u8([1 if l.creative_commons() else 0 for l in self.licenses])]
        tpl = _native._Templates(t, max(len(self.vocab), 1), *[a.ctypes.data for a in self._keep])
        ctx = ctypes.c_void_p()
        self._check(lib.dice_create(ctypes.byref(tpl), device, ctypes.byref(ctx)))
        self.ctx = ctx
        self._setup_exact()

    def close(self):
        if self.ctx:
            _native.load_library().dice_destroy(self.ctx)
        self.ctx = None

    def matches_by_similarity(self, file, potential):
        scores = self.similarity_rows([file])[0]
        ranked = []
        for license in potential:
            if license.key not in self.index:
                raise Error(f'{license.key} is not in the GPU corpus')
            i = self.index[license.key]
            ranked.append((license, scores[i], i))
        # ranked.sort_by { |_, score, i| [score, i] }.reverse
        ranked.sort(key=lambda r: (r[1], r[2]))
        ranked.reverse()
        return [(license, score) for license, score, _ in ranked]

    def similarity_rows(self, files):
        n = len(files)
        t = len(self.licenses)
        if n == 0:
            return []
        score = np.empty(n * t, np.float64)
        fs = self._files_struct(files)
        self._check(_native.load_library().dice_similarity_matrix(self.ctx, ctypes.byref(fs), None,
                                                                   score.ctypes.data, 0, None, None))
        return [list(score[i * t:(i + 1) * t]) for i in range(n)]

    def match(self, files, threshold=98):
        n = len(files)
        if n == 0:
            return []
        best = np.empty(n, np.int32)
        score = np.empty(n, np.float64)
        fs = self._files_struct(files)
        self._check(_native.load_library().dice_match(self.ctx, ctypes.byref(fs), float(threshold),
                                                      best.ctypes.data, None, score.ctypes.data))
        return [(self.licenses[b], float(s)) if b >= 0 else (None, 0) for b, s in zip(best, score)]

    def exact(self, files):
        n = len(files)
        if n == 0:
            return []
        out = np.empty(n, np.int32)
        fmask = np.array([self._field_mask(f.wordset() or ()) for f in files], np.uint64)
        fs = self._files_struct(files)
        self._check(_native.load_library().dice_exact(self.ctx, ctypes.byref(fs), fmask.ctypes.data,
                                                      out.ctypes.data))
        return [self.licenses[i] if i >= 0 else None for i in out]

    def detect(self, license_files, threshold=98):
        from licensee_amd.matchers import Copyright
        out = [None] * len(license_files)
        rest = []
        for i, f in enumerate(license_files):
            m = Copyright(f)
            if m.match() is not None:
                out[i] = (m.match(), m.confidence(), m.name)
            else:
                rest.append(i)
        files = [license_files[i] for i in rest]
        exact = self.exact(files)
        for j, (license, confidence) in enumerate(self.match(files, threshold)):
            if exact[j] is not None:
                out[rest[j]] = (exact[j], 100, 'exact')
            elif license is not None:
                out[rest[j]] = (license, confidence, 'dice')
            else:
                out[rest[j]] = (License.find('other'), None, None)
        return out

    def _setup_exact(self):
        self.fields = {}
        t = len(self.licenses)
        fbits = np.zeros(t * self.w64, np.uint64)
        need = [0] * t
        for i, l in enumerate(self.licenses):
            words = l.fields_normalized_set()
            self._put_bits(fbits, i, words)
            for w in sorted(words):   # Ruby Set order is insertion order; any numbering works
                if w in self.vocab:
                    continue
                k = self.fields.setdefault(w, len(self.fields))
                if k >= 64:
                    raise Error('more than 64 field words outside the vocabulary')
                need[i] |= 1 << k
        needp = np.array(need, np.uint64)
        self._exact_keep = [fbits, needp]
        ws = _u32([len(l.wordset()) for l in self.licenses])
        self._exact_keep.append(ws)
        self._check(_native.load_library().dice_exact_setup(self.ctx, ws.ctypes.data, fbits.ctypes.data,
                                                            needp.ctypes.data))

    def _field_mask(self, words):
        return sum(1 << self.fields[w] for w in words if w in self.fields)

    def _files_struct(self, files):
        n = len(files)
        bits = np.zeros(max(n, 1) * self.w64, np.uint64)
        for i, f in enumerate(files):
            self._put_bits(bits, i, f.wordset() or ())
        ws = _u32([len(f.wordset() or ()) for f in files])
        ln = _i32([f.length() for f in files])
        cc = _u8([1 if getattr(f, 'potential_false_positive', lambda: False)() else 0 for f in files])
        self._files_keep = [bits, ws, ln, cc]
        return _native._Files(n, bits.ctypes.data, ws.ctypes.data, ln.ctypes.data, cc.ctypes.data)

    def _put_bits(self, arr, row, words):
        base = row * self.w64
        for w in words:
            i = self.vocab.get(w)
            if i is not None:
                arr[base + (i >> 6)] |= np.uint64(1) << np.uint64(i & 63)

    @staticmethod
    def _check(rc):
        if rc != 0:
            raise Error(f'dice error {rc}: {_native.load_library().dice_last_error().decode()}')
