"""Synthetic perturbed-license corpus (measurement harness input) -- ctypes front end of
csrc/synth.cpp. See that file for the perturbation recipe and its reference anchors.

The generator works in normalized space: each template's ``content_normalized`` is split
into space-separated tokens, each token is mapped once to its scan words
(content_helper.rb:109) as extended word ids -- vocabulary ids first, out-of-vocabulary
ids after -- and the C++ side composes files from token ids.
"""
from __future__ import annotations

import ctypes
import json
import os
from typing import List, Optional, Sequence

import numpy as np

from ._native import FileBatch
from .content_helper import WORDSET_REGEX
from .corpus import TemplateCorpus

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'lib', 'liblicensee_synth.so')

# Filler words: the reference's own list, spec/fixtures/ipsum.txt (924 words, repeats kept so
# the draw weights match add_random_words, spec_helper.rb:82-91), vendored lowercased as
# data/ipsum.json by tools/vendor_templates.py.
IPSUM_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'data', 'ipsum.json')
with open(IPSUM_PATH, encoding='utf-8') as _fh:
    IPSUM_WORDS = tuple(json.load(_fh)['words'])


class _Spec(ctypes.Structure):
    _fields_ = [('n_tokens', ctypes.c_int32), ('tok_len', ctypes.c_void_p),
                ('tok_word_off', ctypes.c_void_p), ('tok_words', ctypes.c_void_p),
                ('n_templates', ctypes.c_int32), ('tpl_off', ctypes.c_void_p),
                ('tpl_tokens', ctypes.c_void_p), ('n_ipsum', ctypes.c_int32),
                ('ipsum_tokens', ctypes.c_void_p), ('n_vocab', ctypes.c_int32),
                ('n_ext', ctypes.c_int32), ('profile', ctypes.c_int32)]


_lib = None


def _load():
    global _lib
    if _lib is None:
        l = ctypes.CDLL(LIB_PATH)
        vp = ctypes.c_void_p
        l.synth_generate.restype = ctypes.c_int
        l.synth_generate.argtypes = [vp, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32,
                                     vp, vp, vp, vp, vp]
        l.synth_tokens.restype = ctypes.c_int64
        l.synth_tokens.argtypes = [vp, ctypes.c_uint64, ctypes.c_int64, vp, ctypes.c_int64, vp, vp]
        _lib = l
    return _lib


class SyntheticCorpus:
    def __init__(self, corpus: TemplateCorpus, texts: Optional[Sequence[str]] = None, profile: int = 0,
                 ipsum: Sequence[str] = IPSUM_WORDS):
        self.corpus = corpus
        texts = list(texts) if texts is not None else [t.content_normalized() for t in corpus.templates]
        self.tokens: List[str] = []
        tok_id = {}
        ext = dict(corpus.index)
        tok_len, tok_off, tok_words = [], [0], []

        def token(s: str) -> int:
            if s in tok_id:
                return tok_id[s]
            tok_id[s] = len(self.tokens)
            self.tokens.append(s)
            tok_len.append(len(s))
            for w in dict.fromkeys(WORDSET_REGEX.findall(s)):
                if w not in ext:
                    ext[w] = len(ext)
                tok_words.append(ext[w])
            tok_off.append(len(tok_words))
            return tok_id[s]

        tpl_off, tpl_tokens = [0], []
        for text in texts:
            tpl_tokens.extend(token(s) for s in (text.split(' ') if text else []))
            tpl_off.append(len(tpl_tokens))
        ipsum_ids = [token(w) for w in ipsum]
        self.ext_words = ext
        self._arrays = [np.array(tok_len, np.int32), np.array(tok_off, np.int32),
                        np.array(tok_words if tok_words else [0], np.int32), np.array(tpl_off, np.int64),
                        np.array(tpl_tokens if tpl_tokens else [0], np.int32), np.array(ipsum_ids, np.int32)]
        a = self._arrays
        self._spec = _Spec(len(self.tokens), a[0].ctypes.data, a[1].ctypes.data, a[2].ctypes.data,
                           len(texts), a[3].ctypes.data, a[4].ctypes.data, len(ipsum_ids), a[5].ctypes.data,
                           corpus.n_vocab, max(len(ext), corpus.n_vocab), profile)

    def generate(self, first: int, n: int, seed: int = 20250202, nthreads: int = 8, with_source: bool = False):
        w64 = self.corpus.w64
        bits = np.empty((n, w64), np.uint64)
        wf = np.empty(n, np.uint32)
        ln = np.empty(n, np.int32)
        cc = np.empty(n, np.uint8)
        src = np.empty(n, np.int32) if with_source else None
        rc = _load().synth_generate(ctypes.byref(self._spec), seed, first, n, nthreads, bits.ctypes.data,
                                    wf.ctypes.data, ln.ctypes.data, cc.ctypes.data,
                                    None if src is None else src.ctypes.data)
        if rc:
            raise RuntimeError('synth_generate failed')
        fb = FileBatch(bits, wf, ln, cc)
        return (fb, src) if with_source else fb

    def text(self, index: int, seed: int = 20250202):
        """Replay file ``index`` as normalized text (tests)."""
        cap = 1 << 16
        while True:
            out = np.empty(cap, np.int32)
            cc = ctypes.c_uint8()
            src = ctypes.c_int32()
            n = _load().synth_tokens(ctypes.byref(self._spec), seed, index, out.ctypes.data, cap,
                                     ctypes.byref(cc), ctypes.byref(src))
            if n <= cap:
                return ' '.join(self.tokens[t] for t in out[:n]), bool(cc.value), src.value
            cap = int(n)
