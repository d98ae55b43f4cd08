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

import ctypes
import hashlib
import os
import struct
import sys
from typing import Dict, Iterable, List, Sequence, Tuple

import numpy as np

from ._native import FileBatch, words64

_HOST_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'lib', 'liblicensee_host.so')
_CACHE_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'lib', 'cache')
_PACK_VERSION = 2
_packed: Dict[str, np.ndarray] = {}


def vocabulary_order(members: Dict[str, List[int]], n_templates: int) -> List[str]:
    """Deterministic vocabulary order for the device bitsets.

    Words with the same template-membership signature form a group. For T <= 64 (the
    sparse-program regime) groups are chained greedily by nearest Hamming distance between
    signatures, starting from the most widely shared group, so each template's words land in
    few 32-bit dwords (1547 -> 1352 program entries on the 47 vendored templates). Larger
    corpora use the dense kernel, where order does not matter: signature-lexicographic."""
    if n_templates > 64:
        return sorted(members, key=lambda w: (tuple(members[w]), w))
    groups: Dict[int, List[str]] = {}
    for w, ts in members.items():
        groups.setdefault(sum(1 << t for t in ts), []).append(w)
    sigs = np.array(sorted(groups), dtype=np.uint64)
    sizes = np.array([len(groups[int(g)]) for g in sigs], dtype=np.int64)
    pop = np.array([bin(int(g)).count('1') for g in sigs], dtype=np.int64)
    left = np.ones(len(sigs), dtype=bool)
    cur = int(np.lexsort((np.arange(len(sigs)), -sizes, -pop))[0])
    chain = [cur]
    left[cur] = False
    lut = np.array([bin(i).count('1') for i in range(256)], dtype=np.int64)
    for _ in range(len(sigs) - 1):
        x = (sigs ^ sigs[cur]).view(np.uint8).reshape(-1, 8)
        ham = lut[x].sum(axis=1)
        ham[~left] = 1 << 40
        # nearest signature; ties: larger group, then smaller signature value (deterministic)
        cand = np.nonzero(ham == ham.min())[0]
        cur = int(cand[np.lexsort((sigs[cand], -sizes[cand]))[0]])
        chain.append(cur)
        left[cur] = False
    return [w for g in chain for w in sorted(groups[int(sigs[g])])]


def _pack_budget(n_vocab: int, n_templates: int) -> int:
    """Default local-search attempts: ~3 s for the 47 vendored templates, ~15 s for ~600."""
    return n_vocab * (10000 if n_templates <= 64 else 2000)


def _pack_lib():
    try:
        lib = ctypes.CDLL(_HOST_LIB)
    except OSError:
        return None
    fn = lib.lh_vocab_pack
    fn.restype = ctypes.c_int64
    vp = ctypes.c_void_p
    fn.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp, ctypes.c_int32, ctypes.c_int64,
                   ctypes.c_uint64, vp]
    return fn


def _signatures(order: List[str], members: Dict[str, List[int]], n_templates: int) -> np.ndarray:
    W = (n_templates + 63) // 64
    sig = np.zeros((len(order), W), np.uint64)
    for i, w in enumerate(order):
        for t in members[w]:
            sig[i, t >> 6] |= np.uint64(1) << np.uint64(t & 63)
    return sig


def _cache_path(sig: np.ndarray, n_templates: int, bin_bits: int) -> str:
    key = hashlib.sha1(sig.tobytes() + struct.pack('<iiii', sig.shape[0], n_templates, bin_bits,
                                                   _PACK_VERSION)).hexdigest()[:20]
    return os.path.join(_CACHE_DIR, f'vocab_{key}.i32')


def _read_perm(path: str, V: int):
    if not os.path.exists(path):
        return None
    perm = np.fromfile(path, dtype=np.int32)
    if len(perm) != V or not np.array_equal(np.sort(perm), np.arange(V, dtype=np.int32)):
        return None
    return perm


def _write_perm(path: str, perm: np.ndarray):
    try:
        os.makedirs(_CACHE_DIR, exist_ok=True)
        tmp = f'{path}.{os.getpid()}'
        perm.tofile(tmp)
        os.replace(tmp, path)
    except OSError:
        pass


def pack_vocabulary(order: List[str], members: Dict[str, List[int]], n_templates: int,
                    iters: int = None) -> List[str]:
    """Re-pack ``order`` into device bins with the native local search (lh_vocab_pack).

    Bins are 32 words for the sparse program (T <= 64: cost = instruction pairs per
    (template, dword)) and 64 words for the LDS kernel (records per (template, u64)).
    Deterministic (fixed seed). The result is cached in-process and under lib/cache by a
    hash of the signatures; a cached order is used as is, so a longer build-time search
    (:func:`improve_packing`) serves every later run. Without the native host library the
    order is returned unchanged (scores never depend on the order)."""
    V = len(order)
    if V < 2 or n_templates < 2:   # one template: every word has the same signature
        return order
    sig = _signatures(order, members, n_templates)
    bin_bits = 32 if n_templates <= 64 else 64
    path = _cache_path(sig, n_templates, bin_bits)
    perm = _packed.get(path)
    if perm is None:
        perm = _read_perm(path, V)
    if perm is None:
        fn = _pack_lib()
        if fn is None:
            print(f'licensee_amd: {_HOST_LIB} missing, vocabulary left unpacked', file=sys.stderr)
            return order
        init = np.arange(V, dtype=np.int32)
        perm = np.empty(V, np.int32)
        budget = _pack_budget(V, n_templates) if iters is None else iters
        if fn(sig.ctypes.data, V, sig.shape[1], n_templates, init.ctypes.data, bin_bits, budget, 20250202,
              perm.ctypes.data) < 0:
            raise ValueError('lh_vocab_pack rejected the vocabulary')
        _write_perm(path, perm)
    _packed[path] = perm
    return [order[i] for i in perm]


# The postings kernel (T > 64, csrc/dice_post.hip) scores the first D <= 16 u64 words of the
# vocabulary as dense template masks and every later word through its postings list, whose
# expected cost per file grows with the square of the list length: its widest words belong in
# that prefix.
_POSTINGS_PREFIX = 16 * 64


def postings_prefix(order: List[str], members: Dict[str, List[int]]) -> List[str]:
    """``order`` with its _POSTINGS_PREFIX widest words moved to the front, widest first (ties:
    earlier in ``order``); the rest keep their relative order. Deterministic."""
    if len(order) <= _POSTINGS_PREFIX:
        return sorted(order, key=lambda w: -len(members[w]))   # stable: ties keep their order
    pos = {w: i for i, w in enumerate(order)}
    head = sorted(order, key=lambda w: (-len(members[w]), pos[w]))[:_POSTINGS_PREFIX]
    chosen = set(head)
    return head + [w for w in order if w not in chosen]


def improve_packing(templates: Sequence, iters_per_word: int) -> Tuple[int, int]:
    """Build step: continue the local search from the cached order of ``templates``' corpus
    with a larger budget and keep the result when it is cheaper. Returns (old, new) cost."""
    lfs = [t.wordset_fieldless() for t in templates]
    members: Dict[str, List[int]] = {}
    for i, lf in enumerate(lfs):
        for w in lf:
            members.setdefault(w, []).append(i)
    T = len(lfs)
    order = vocabulary_order(members, T)
    V = len(order)
    fn = _pack_lib()
    if fn is None or V < 2 or T < 2:
        return 0, 0
    pack_vocabulary(order, members, T)                  # make sure a cached order exists
    sig = _signatures(order, members, T)
    bin_bits = 32 if T <= 64 else 64
    path = _cache_path(sig, T, bin_bits)
    marker = f'{path}.improved{iters_per_word}'
    cur = _read_perm(path, V)
    if cur is None:
        cur = _packed[path]
    out = np.empty(V, np.int32)
    if os.path.exists(marker):                          # already searched with this budget
        c = fn(sig.ctypes.data, V, sig.shape[1], T, cur.ctypes.data, bin_bits, 0, 1, out.ctypes.data)
        return c, c
    old = fn(sig.ctypes.data, V, sig.shape[1], T, cur.ctypes.data, bin_bits, 0, 1, out.ctypes.data)
    new = fn(sig.ctypes.data, V, sig.shape[1], T, cur.ctypes.data, bin_bits, V * iters_per_word, 20250202,
             out.ctypes.data)
    if 0 <= new < old:
        _write_perm(path, out)
        _packed[path] = out
    try:
        open(marker, 'w').close()
    except OSError:
        pass
    return old, min(old, new) if new >= 0 else old


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
        self.vocab: List[str] = pack_vocabulary(vocabulary_order(members, len(lfs)), members, len(lfs))
        if len(lfs) > 64:
            self.vocab = postings_prefix(self.vocab, members)
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
