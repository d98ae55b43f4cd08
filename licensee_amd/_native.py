"""ctypes binding of the C-ABI in include/licensee_dice.h (liblicensee_dice.so).

This is the product's only scoring path: if the HIP library is missing or no gfx950
device is usable, calls raise -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'lib')
LIB_PATH = os.path.join(LIB_DIR, 'liblicensee_dice.so')

DICE_OK = 0
DICE_TOPK_MAX = 16

EXPORTED_SYMBOLS = (
    'dice_words64', 'dice_create', 'dice_destroy', 'dice_ctx_info', 'dice_match',
    'dice_similarity_matrix', 'dice_batch_create', 'dice_batch_destroy', 'dice_batch_upload',
    'dice_batch_match', 'dice_batch_matrix', 'dice_batch_download_match',
    'dice_batch_download_matrix', 'dice_batch_result_ptrs', 'dice_batch_bytes_per_file',
    'dice_last_error', 'dice_precompile', 'dice_program_source', 'dice_batch_stream_probe',
    'dice_match_sharded', 'dice_similarity_matrix_sharded', 'dice_batch_upload_ids', 'dice_last_gather_peer',
    'dice_batch_deferred',
    'dice_ctx_match_kernel', 'dice_exact_setup', 'dice_batch_exact', 'dice_batch_download_exact', 'dice_exact',
    'dice_match_confidence', 'dice_batch_match_confidence', 'dice_match_sharded_confidence',
    'dice_batch_scored_pairs', 'dice_vocab_setup', 'dice_batch_upload_text', 'dice_batch_set_rows',
    'dice_batch_download_rows', 'dice_host_alloc', 'dice_host_free',
)
DICE_GATHER_HOST = 0
DICE_GATHER_DEVICE = 1


class DiceError(RuntimeError):
    pass


class _Templates(ctypes.Structure):
    _fields_ = [('n_templates', ctypes.c_int32), ('n_vocab', ctypes.c_int32),
                ('lf_bits', ctypes.c_void_p), ('lf_size', ctypes.c_void_p),
                ('fields_set_size', ctypes.c_void_p), ('length_slack', ctypes.c_void_p),
                ('length', ctypes.c_void_p), ('is_cc', ctypes.c_void_p)]


class _Files(ctypes.Structure):
    _fields_ = [('n_files', ctypes.c_int64), ('bits', ctypes.c_void_p),
                ('wordset_size', ctypes.c_void_p), ('length', ctypes.c_void_p),
                ('cc_false_positive', ctypes.c_void_p)]


_lib = None


def hip_runtime_path() -> Optional[str]:
    """The HIP runtime this process should share: LICENSEE_DICE_HIP_RUNTIME if set ('' = none),
    else the copy torch ships (torch/lib/libamdhip64.so, soname libamdhip64.so.7) when torch is
    installed -- found without importing torch."""
    env = os.environ.get('LICENSEE_DICE_HIP_RUNTIME')
    if env is not None:
        return env or None
    import importlib.util
    try:
        spec = importlib.util.find_spec('torch')
    except (ImportError, ValueError):
        return None
    if spec is None or not spec.origin:
        return None
    p = os.path.join(os.path.dirname(spec.origin), 'lib', 'libamdhip64.so')
    return p if os.path.exists(p) else None


def elf_dynamic(path: str) -> Tuple[Optional[str], Tuple[str, ...]]:
    """(DT_SONAME, DT_NEEDED entries) of an ELF64 little-endian shared object, read from its
    program headers (PT_DYNAMIC, the string table's address mapped through PT_LOAD); (None, ())
    when the file is not such an object."""
    import struct
    try:
        with open(path, 'rb') as fh:
            hdr = fh.read(64)
            if len(hdr) < 64 or hdr[:4] != b'\x7fELF' or hdr[4] != 2 or hdr[5] != 1:
                return None, ()
            phoff, = struct.unpack_from('<Q', hdr, 0x20)
            phentsize, phnum = struct.unpack_from('<HH', hdr, 0x36)
            fh.seek(phoff)
            ph = fh.read(phentsize * phnum)
            loads, dyn = [], None
            for i in range(phnum):
                p_type, _, p_offset, p_vaddr, _, p_filesz, _, _ = struct.unpack_from('<IIQQQQQQ', ph, i * phentsize)
                if p_type == 1:
                    loads.append((p_vaddr, p_offset, p_filesz))
                elif p_type == 2:
                    dyn = (p_offset, p_filesz)
            if dyn is None:
                return None, ()
            fh.seek(dyn[0])
            raw = fh.read(dyn[1])
            ents = [struct.unpack_from('<qQ', raw, o) for o in range(0, len(raw) - 15, 16)]
            strtab = next((v for t, v in ents if t == 5), None)
            if strtab is None:
                return None, ()
            base = next((off + strtab - va for va, off, sz in loads if va <= strtab < va + sz), None)
            if base is None:
                return None, ()

            def string(o):
                fh.seek(base + o)
                s = fh.read(256)
                return s[:s.index(b'\0')].decode('utf-8', 'replace') if b'\0' in s else None
            soname = next((string(v) for t, v in ents if t == 14), None)
            needed = tuple(string(v) for t, v in ents if t == 1)
            return soname, tuple(x for x in needed if x)
    except (OSError, struct.error, ValueError):
        return None, ()


def needed_hip_soname(lib_path: str) -> Optional[str]:
    """The HIP runtime soname lib_path was linked against (libamdhip64.so.N), or None."""
    return next((x for x in elf_dynamic(lib_path)[1] if x.startswith('libamdhip64.so')), None)


def preload_decision(lib_path: str = LIB_PATH) -> Tuple[Optional[str], str]:
    """(runtime file to map first or None, reason). The candidate (hip_runtime_path) is mapped only
    when its DT_SONAME equals the soname lib_path needs: a torch built against another ROCm major
    ships libamdhip64.so.6, which the library would not bind to -- mapping it anyway would only put
    a second runtime beside the one the library loads (dice_create refuses that)."""
    p = hip_runtime_path()
    if not p:
        return None, 'no candidate runtime'
    want = needed_hip_soname(lib_path)
    have = elf_dynamic(p)[0]
    if want is None or have != want:
        return None, f'{p} has soname {have!r}, {os.path.basename(lib_path)} needs {want!r}: not preloaded'
    return p, f'{p} ({have})'


def _preload_hip_runtime(lib_path: str = LIB_PATH):
    """One HIP runtime per process. liblicensee_dice.so needs libamdhip64.so.7 by soname; if the
    runtime torch uses is mapped first, the library binds to it, and torch (imported before or
    after) keeps one runtime and one device view. Loaded the other way round, /opt/rocm's copy
    and torch's would both be mapped, and dice_create refuses that (dice_last_error names both).
    A candidate whose soname differs from the one the library needs is skipped (preload_decision)."""
    p, _ = preload_decision(lib_path)
    if p:
        ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load liblicensee_dice.so (raises if it was not built -- no fallback). LICENSEE_DICE_LIB
    names another build of the same library (A/B of compile-time kernel variants)."""
    global _lib
    path = os.environ.get('LICENSEE_DICE_LIB', path)
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise DiceError(f'{path} is missing: build it with `python -c "import __graft_entry__ as g; g.build()"`')
    _preload_hip_runtime(path)
    lib = ctypes.CDLL(path)
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    sig = {
        'dice_words64': (i32, [i32]),
        'dice_create': (ctypes.c_int, [ctypes.POINTER(_Templates), i32, ctypes.POINTER(vp)]),
        'dice_destroy': (None, [vp]),
        'dice_ctx_info': (ctypes.c_int, [vp, vp, vp, vp, vp]),
        'dice_ctx_match_kernel': (ctypes.c_int32, [vp]),
        'dice_match': (ctypes.c_int, [vp, ctypes.POINTER(_Files), ctypes.c_double, vp, vp, vp]),
        'dice_match_confidence': (ctypes.c_int, [vp, ctypes.POINTER(_Files), ctypes.c_double, vp, vp, vp]),
        'dice_similarity_matrix': (ctypes.c_int, [vp, ctypes.POINTER(_Files), vp, vp, i32, vp, vp]),
        'dice_batch_create': (ctypes.c_int, [vp, i64, ctypes.POINTER(vp)]),
        'dice_batch_destroy': (None, [vp]),
        'dice_batch_upload': (ctypes.c_int, [vp, ctypes.POINTER(_Files), vp]),
        'dice_batch_upload_ids': (ctypes.c_int, [vp, i64, vp, vp, i32, vp, vp, vp, vp]),
        'dice_batch_match': (ctypes.c_int, [vp, ctypes.c_double, vp]),
        'dice_batch_match_confidence': (ctypes.c_int, [vp, ctypes.c_double, vp]),
        'dice_batch_matrix': (ctypes.c_int, [vp, i32, vp]),
        'dice_batch_download_match': (ctypes.c_int, [vp, vp, vp, vp, vp]),
        'dice_batch_download_matrix': (ctypes.c_int, [vp, vp, vp, i32, vp, vp, vp]),
        'dice_batch_result_ptrs': (ctypes.c_int, [vp, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp)]),
        'dice_batch_bytes_per_file': (i64, [vp]),
        'dice_batch_stream_probe': (ctypes.c_int, [vp, vp]),
        'dice_last_error': (ctypes.c_char_p, []),
        'dice_match_sharded': (ctypes.c_int, [vp, i32, ctypes.POINTER(_Files), ctypes.c_double, i32, vp, vp, vp]),
        'dice_match_sharded_confidence': (ctypes.c_int, [vp, i32, ctypes.POINTER(_Files), ctypes.c_double, i32, vp, vp,
                                                         vp]),
        'dice_similarity_matrix_sharded': (ctypes.c_int, [vp, i32, ctypes.POINTER(_Files), i32, vp, vp, i32,
                                                          vp, vp]),
        'dice_last_gather_peer': (i32, []),
        'dice_batch_deferred': (ctypes.c_int, [vp, ctypes.POINTER(i64), vp]),
        'dice_batch_scored_pairs': (ctypes.c_int, [vp, ctypes.POINTER(i64), vp]),
        'dice_precompile': (ctypes.c_int, [ctypes.POINTER(_Templates), ctypes.c_char_p, i32]),
        'dice_program_source': (i64, [ctypes.POINTER(_Templates), ctypes.c_char_p, i64]),
        'dice_exact_setup': (ctypes.c_int, [vp, vp, vp, vp]),
        'dice_batch_exact': (ctypes.c_int, [vp, vp, vp]),
        'dice_batch_download_exact': (ctypes.c_int, [vp, vp, vp]),
        'dice_exact': (ctypes.c_int, [vp, ctypes.POINTER(_Files), vp, vp]),
        'dice_vocab_setup': (ctypes.c_int, [vp, i32, vp, i32, vp]),
        'dice_batch_upload_text': (ctypes.c_int, [vp, i64, vp, i64, vp, vp, vp, vp, vp, ctypes.POINTER(i64), vp]),
        'dice_batch_set_rows': (ctypes.c_int, [vp, i64, vp, vp, vp, vp, vp]),
        'dice_batch_download_rows': (ctypes.c_int, [vp, vp, vp, vp, vp]),
        'dice_host_alloc': (ctypes.c_int, [i64, ctypes.POINTER(vp)]),
        'dice_host_free': (None, [vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _check(rc: int):
    if rc != DICE_OK:
        msg = load_library().dice_last_error().decode('utf-8', 'replace')
        raise DiceError(f'dice error {rc}: {msg}')


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data


def words64(n_vocab: int) -> int:
    return (n_vocab + 63) // 64


@dataclass
class FileBatch:
    """Interned candidate files (host memory), the layout of ``dice_files``."""
    bits: np.ndarray            # [n, words64(V)] uint64
    wordset_size: np.ndarray    # [n] uint32
    length: np.ndarray          # [n] int32
    cc_false_positive: np.ndarray  # [n] uint8

    def __post_init__(self):
        self.bits = np.ascontiguousarray(self.bits, dtype=np.uint64)
        self.wordset_size = np.ascontiguousarray(self.wordset_size, dtype=np.uint32)
        self.length = np.ascontiguousarray(self.length, dtype=np.int32)
        self.cc_false_positive = np.ascontiguousarray(self.cc_false_positive, dtype=np.uint8)
        n = self.bits.shape[0]
        if not (self.wordset_size.shape == self.length.shape == self.cc_false_positive.shape == (n,)):
            raise ValueError('inconsistent FileBatch shapes')

    @property
    def n(self) -> int:
        return self.bits.shape[0]

    def _struct(self) -> _Files:
        return _Files(self.n, _ptr(self.bits), _ptr(self.wordset_size), _ptr(self.length),
                      _ptr(self.cc_false_positive))


def bits_to_ids(bits: np.ndarray, n_vocab: int, chunk: int = 16384):
    """Bitset rows [n, words64(V)] -> the id-list form of ``DeviceBatch.upload_ids``:
    (offsets [n+1] int64, ids uint16 when V <= 65536 else uint32), ids ascending per file."""
    bits = np.ascontiguousarray(bits, dtype=np.uint64)
    n = bits.shape[0]
    dt = np.uint16 if n_vocab <= 65536 else np.uint32
    counts = np.zeros(n, np.int64)
    parts = []
    for a in range(0, n, chunk):
        blk = np.unpackbits(bits[a:a + chunk].view(np.uint8), axis=1, bitorder='little')[:, :n_vocab]
        r, col = np.nonzero(blk)
        counts[a:a + blk.shape[0]] = np.bincount(r, minlength=blk.shape[0])
        parts.append(col.astype(dt))
    offsets = np.zeros(n + 1, np.int64)
    np.cumsum(counts, out=offsets[1:])
    return offsets, (np.concatenate(parts) if parts else np.zeros(0, dt))


class Scorer:
    """Owns a ``dice_ctx``: one template corpus resident on one gfx950 device."""

    def __init__(self, lf_bits: np.ndarray, lf_size, fields_set_size, length_slack, length, is_cc,
                 n_vocab: int, device: int = 0):
        lib = load_library()
        self._keep = [np.ascontiguousarray(lf_bits, dtype=np.uint64),
                      np.ascontiguousarray(lf_size, dtype=np.uint32),
                      np.ascontiguousarray(fields_set_size, dtype=np.uint32),
                      np.ascontiguousarray(length_slack, dtype=np.int32),
                      np.ascontiguousarray(length, dtype=np.int32),
                      np.ascontiguousarray(is_cc, dtype=np.uint8)]
        T = self._keep[1].shape[0]
        if self._keep[0].shape != (T, words64(n_vocab)):
            raise ValueError('lf_bits must be [T, words64(V)]')
        self.n_templates, self.n_vocab, self.device = T, n_vocab, device
        tpl = _Templates(T, n_vocab, *[_ptr(a) for a in self._keep])
        ctx = ctypes.c_void_p()
        _check(lib.dice_create(ctypes.byref(tpl), device, ctypes.byref(ctx)))
        self._ctx = ctx

    def close(self):
        if getattr(self, '_ctx', None):
            load_library().dice_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self) -> Tuple[int, int, int, int]:
        vals = [ctypes.c_int32() for _ in range(4)]
        _check(load_library().dice_ctx_info(self._ctx, *[ctypes.byref(v) for v in vals]))
        return tuple(v.value for v in vals)

    def match_kernel(self) -> int:
        """Kernel Dice#match runs on: 0 dense, 1 sparse program, 2 LDS records, 3 postings,
        4 bound-pruned (dice_prune.hip)."""
        return int(load_library().dice_ctx_match_kernel(self._ctx))

    def match(self, files: FileBatch, threshold: float, confidence: bool = False):
        """(best, overlap, score) per file. confidence=False: score/overlap of the top-ranked
        template even when it misses the threshold (dice_match); True: Dice#confidence, 0 for a
        file without a match (dice_match_confidence, dice.rb:51-53)."""
        n = files.n
        best = np.empty(n, np.int32)
        ov = np.empty(n, np.uint32)
        score = np.empty(n, np.float64)
        if n:
            st = files._struct()
            lib = load_library()
            fn = lib.dice_match_confidence if confidence else lib.dice_match
            _check(fn(self._ctx, ctypes.byref(st), float(threshold), _ptr(best), _ptr(ov), _ptr(score)))
        return best, ov, score

    def matrix(self, files: FileBatch, k: int = 0):
        n, T = files.n, self.n_templates
        ov = np.empty((n, T), np.uint32)
        score = np.empty((n, T), np.float64)
        tki = np.empty((n, max(k, 0)), np.int32)
        tks = np.empty((n, max(k, 0)), np.float64)
        if n:
            st = files._struct()
            _check(load_library().dice_similarity_matrix(self._ctx, ctypes.byref(st), _ptr(ov), _ptr(score), k,
                                                         _ptr(tki) if k else None, _ptr(tks) if k else None))
        return ov, score, tki, tks

    def batch(self, capacity: int) -> 'DeviceBatch':
        return DeviceBatch(self, capacity)

    def exact_setup(self, wordset_size, field_bits: Optional[np.ndarray] = None,
                    field_need: Optional[np.ndarray] = None):
        """Exact#match tables (exact.rb:6-12): |wordset| per template, the field words that are
        vocabulary words as [T, words64(V)] bits, the others as [T] uint64 need masks."""
        T = self.n_templates
        ws = np.ascontiguousarray(wordset_size, dtype=np.uint32)
        fb = None if field_bits is None else np.ascontiguousarray(field_bits, dtype=np.uint64)
        fn = None if field_need is None else np.ascontiguousarray(field_need, dtype=np.uint64)
        if ws.shape != (T,) or (fb is not None and fb.shape != (T, words64(self.n_vocab))) or \
                (fn is not None and fn.shape != (T,)):
            raise ValueError('exact tables: wordset_size [T], field_bits [T, words64(V)], field_need [T]')
        _check(load_library().dice_exact_setup(self._ctx, _ptr(ws), _ptr(fb), _ptr(fn)))

    def vocab_setup(self, words, extra=()):
        """The device wordset scan's tables (``dice_vocab_setup``): the vocabulary words in id
        order and up to 64 extra words (template field words outside the vocabulary), ASCII."""
        enc = [w.encode('ascii') for w in words]
        ext = [w.encode('ascii') for w in extra]
        wa = (ctypes.c_char_p * max(len(enc), 1))(*enc)
        ea = (ctypes.c_char_p * max(len(ext), 1))(*ext)
        _check(load_library().dice_vocab_setup(self._ctx, len(enc), ctypes.cast(wa, ctypes.c_void_p),
                                               len(ext), ctypes.cast(ea, ctypes.c_void_p)))

    def exact(self, files: FileBatch, field_mask: Optional[np.ndarray] = None) -> np.ndarray:
        """Exact#match per file on the device: template index or -1."""
        out = np.empty(files.n, np.int32)
        if files.n:
            fm = None if field_mask is None else np.ascontiguousarray(field_mask, dtype=np.uint64)
            if fm is not None and fm.shape != (files.n,):
                raise ValueError('field_mask must be [n]')
            st = files._struct()
            _check(load_library().dice_exact(self._ctx, ctypes.byref(st), _ptr(fm), _ptr(out)))
        return out


class PinnedBuffer:
    """Page-locked host bytes (``dice_host_alloc``) viewed as a uint8 numpy array."""

    def __init__(self, nbytes: int):
        p = ctypes.c_void_p()
        _check(load_library().dice_host_alloc(int(nbytes), ctypes.byref(p)))
        self._p = p
        self.nbytes = int(nbytes)
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * max(self.nbytes, 1)).from_address(p.value))[:self.nbytes]

    def close(self):
        if getattr(self, '_p', None):
            self.array = None
            load_library().dice_host_free(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceBatch:
    """A device-resident batch (``dice_batch``): upload once, score many times."""

    def __init__(self, scorer: Scorer, capacity: int):
        self.scorer = scorer
        b = ctypes.c_void_p()
        _check(load_library().dice_batch_create(scorer._ctx, int(capacity), ctypes.byref(b)))
        self._b = b
        self.capacity = int(capacity)
        self.n = 0

    def close(self):
        if getattr(self, '_b', None):
            load_library().dice_batch_destroy(self._b)
            self._b = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, files: FileBatch, stream: int = 0):
        st = files._struct()
        _check(load_library().dice_batch_upload(self._b, ctypes.byref(st), stream or None))
        self.n = files.n

    def upload_ids(self, offsets: np.ndarray, ids: np.ndarray, wordset_size, length, cc_false_positive,
                   stream: int = 0):
        """Upload files as word-id lists (CSR: file i = ids[offsets[i]:offsets[i+1]], uint16 or
        uint32); the bitsets are built on the device (``dice_batch_upload_ids``)."""
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        ids = np.ascontiguousarray(ids)
        if ids.dtype not in (np.uint16, np.uint32):
            raise ValueError('ids must be uint16 or uint32')
        wf = np.ascontiguousarray(wordset_size, dtype=np.uint32)
        ln = np.ascontiguousarray(length, dtype=np.int32)
        cc = np.ascontiguousarray(cc_false_positive, dtype=np.uint8)
        n = offsets.shape[0] - 1
        if n < 0 or not (wf.shape == ln.shape == cc.shape == (n,)):
            raise ValueError('inconsistent id-list shapes')
        if n and offsets[-1] > ids.shape[0]:
            raise ValueError('offsets run past the id list')
        _check(load_library().dice_batch_upload_ids(self._b, n, _ptr(offsets), _ptr(ids) if ids.size else None,
                                                    ids.dtype.itemsize, _ptr(wf), _ptr(ln), _ptr(cc),
                                                    stream or None))
        self.n = n

    def upload_text(self, text: np.ndarray, offsets, text_len, length, cc_false_positive, stream: int = 0):
        """Upload normalized texts (``dice_batch_upload_text``: uint8 ``text``, file i at
        ``text[offsets[i]:offsets[i] + text_len[i]]``, 16-byte aligned offsets); the device scans
        the wordsets. Returns the [n] status array (1 = too many distinct words outside the
        vocabulary for the device set: send that file with :meth:`set_rows`)."""
        text = np.ascontiguousarray(text, dtype=np.uint8)
        off = np.ascontiguousarray(offsets, dtype=np.int64)
        tl = np.ascontiguousarray(text_len, dtype=np.int32)
        ln = np.ascontiguousarray(length, dtype=np.int32)
        cc = np.ascontiguousarray(cc_false_positive, dtype=np.uint8)
        n = off.shape[0]
        if not (tl.shape == ln.shape == cc.shape == (n,)):
            raise ValueError('inconsistent text-upload shapes')
        st = np.zeros(n, np.uint8)
        nov = ctypes.c_int64(0)
        _check(load_library().dice_batch_upload_text(self._b, n, _ptr(text), int(text.shape[0]), _ptr(off), _ptr(tl),
                                                     _ptr(ln), _ptr(cc), _ptr(st), ctypes.byref(nov), stream or None))
        self.n = n
        return st

    def set_rows(self, index, bits, wordset_size, field_mask=None, stream: int = 0):
        """Overwrite rows / |W_F| / field masks of the resident files ``index`` (``dice_batch_set_rows``)."""
        idx = np.ascontiguousarray(index, dtype=np.int64)
        b = np.ascontiguousarray(bits, dtype=np.uint64)
        wf = np.ascontiguousarray(wordset_size, dtype=np.uint32)
        fm = None if field_mask is None else np.ascontiguousarray(field_mask, dtype=np.uint64)
        k = idx.shape[0]
        if b.shape != (k, words64(self.scorer.n_vocab)) or wf.shape != (k,) or (fm is not None and fm.shape != (k,)):
            raise ValueError('set_rows: index [k], bits [k, words64(V)], wordset_size [k], field_mask [k]')
        _check(load_library().dice_batch_set_rows(self._b, k, _ptr(idx), _ptr(b), _ptr(wf), _ptr(fm), stream or None))

    def download_rows(self, stream: int = 0):
        """The resident rows [n, words64(V)], |W_F| [n] and field masks [n] (``dice_batch_download_rows``)."""
        n = self.n
        bits = np.empty((n, words64(self.scorer.n_vocab)), np.uint64)
        wf = np.empty(n, np.uint32)
        fm = np.empty(n, np.uint64)
        _check(load_library().dice_batch_download_rows(self._b, _ptr(bits), _ptr(wf), _ptr(fm), stream or None))
        return bits, wf, fm

    def match(self, threshold: float, stream: int = 0, confidence: bool = False):
        lib = load_library()
        fn = lib.dice_batch_match_confidence if confidence else lib.dice_batch_match
        _check(fn(self._b, float(threshold), stream or None))

    def matrix(self, k: int, stream: int = 0):
        _check(load_library().dice_batch_matrix(self._b, int(k), stream or None))
        self.k = int(k)

    def download_match(self, stream: int = 0):
        n = self.n
        best = np.empty(n, np.int32)
        ov = np.empty(n, np.uint32)
        score = np.empty(n, np.float64)
        _check(load_library().dice_batch_download_match(self._b, _ptr(best), _ptr(ov), _ptr(score), stream or None))
        return best, ov, score

    def download_matrix(self, k: Optional[int] = None, stream: int = 0):
        """Matrix results of the last :meth:`matrix` call; the top-k arrays are [n][k] with
        that call's k (a different ``k`` raises, as the C-ABI returns DICE_E_ARG)."""
        n, T = self.n, self.scorer.n_templates
        k = getattr(self, 'k', 0) if k is None else int(k)
        ov = np.empty((n, T), np.uint32)
        score = np.empty((n, T), np.float64)
        tki = np.empty((n, k), np.int32)
        tks = np.empty((n, k), np.float64)
        _check(load_library().dice_batch_download_matrix(self._b, _ptr(ov), _ptr(score), k,
                                                         _ptr(tki) if k else None, _ptr(tks) if k else None,
                                                         stream or None))
        return ov, score, tki, tks

    def exact(self, field_mask: Optional[np.ndarray] = None, stream: int = 0):
        """Exact#match of the resident files (asynchronous; ``field_mask`` [n] uint64 or None)."""
        fm = None if field_mask is None else np.ascontiguousarray(field_mask, dtype=np.uint64)
        if fm is not None and fm.shape != (self.n,):
            raise ValueError('field_mask must be [n]')
        self._fm = fm   # the H2D copy may still read it after the call returns
        _check(load_library().dice_batch_exact(self._b, _ptr(fm), stream or None))

    def download_exact(self, stream: int = 0) -> np.ndarray:
        out = np.empty(self.n, np.int32)
        _check(load_library().dice_batch_download_exact(self._b, _ptr(out), stream or None))
        return out

    def deferred(self, stream: int = 0) -> int:
        """Files the bound-pruned kernel handed to the postings kernels in the last match."""
        v = ctypes.c_int64(0)
        _check(load_library().dice_batch_deferred(self._b, ctypes.byref(v), ctypes.c_void_p(stream) if stream else None))
        return int(v.value)

    def scored_pairs(self, stream: int = 0) -> int:
        """(file, template) pairs the last match call scored exactly (dice_batch_scored_pairs)."""
        v = ctypes.c_int64(0)
        _check(load_library().dice_batch_scored_pairs(self._b, ctypes.byref(v),
                                                      ctypes.c_void_p(stream) if stream else None))
        return int(v.value)

    def result_ptrs(self):
        p = [ctypes.c_void_p() for _ in range(3)]
        _check(load_library().dice_batch_result_ptrs(self._b, *[ctypes.byref(x) for x in p]))
        return tuple(x.value for x in p)

    def stream_probe(self, stream: int = 0):
        _check(load_library().dice_batch_stream_probe(self._b, stream or None))

    def bytes_per_file(self) -> int:
        return int(load_library().dice_batch_bytes_per_file(self._b))


def _ctx_array(scorers):
    scorers = list(scorers)
    if not scorers:
        raise ValueError('need at least one Scorer')
    arr = (ctypes.c_void_p * len(scorers))(*[sc._ctx.value for sc in scorers])
    return arr, len(scorers), scorers[0].n_templates


def match_sharded(scorers, files: FileBatch, threshold: float, gather: int = DICE_GATHER_HOST,
                  confidence: bool = False, out=None):
    """``dice_match_sharded`` (``dice_match_sharded_confidence`` with confidence=True): the files
    split into contiguous shards, one per Scorer (each on its own device, host thread and stream),
    results gathered on the host or on the first Scorer's device. Every Scorer must hold the same
    corpus. ``out``: optional (best int32, overlap uint32, score float64) [n] arrays to fill (e.g.
    page-locked buffers, which the gathers copy into directly)."""
    arr, n_ctx, _ = _ctx_array(scorers)
    n = files.n
    if out is not None:
        best, ov, score = out
        if not (best.dtype == np.int32 and ov.dtype == np.uint32 and score.dtype == np.float64 and
                best.shape == ov.shape == score.shape == (n,) and all(a.flags.c_contiguous for a in out)):
            raise ValueError('out must be contiguous [n] int32 / uint32 / float64 arrays')
    else:
        best = np.empty(n, np.int32)
        ov = np.empty(n, np.uint32)
        score = np.empty(n, np.float64)
    if n:
        st = files._struct()
        lib = load_library()
        fn = lib.dice_match_sharded_confidence if confidence else lib.dice_match_sharded
        _check(fn(arr, n_ctx, ctypes.byref(st), float(threshold), int(gather), _ptr(best), _ptr(ov), _ptr(score)))
    return best, ov, score


def last_gather_peer() -> int:
    """``dice_last_gather_peer``: 1 when the last sharded call's device gather wrote every remote
    shard through peer access, 0 when some went through a staged copy, -1 when no peer path was
    exercised (a host gather, or every context on the first context's device)."""
    return int(load_library().dice_last_gather_peer())


def matrix_sharded(scorers, files: FileBatch, k: int = 0, gather: int = DICE_GATHER_HOST):
    """``dice_similarity_matrix_sharded``: full [n][T] matrix + [n][k] top-k, sharded."""
    arr, n_ctx, T = _ctx_array(scorers)
    n = files.n
    ov = np.empty((n, T), np.uint32)
    score = np.empty((n, T), np.float64)
    tki = np.empty((n, max(k, 0)), np.int32)
    tks = np.empty((n, max(k, 0)), np.float64)
    if n:
        st = files._struct()
        _check(load_library().dice_similarity_matrix_sharded(arr, n_ctx, ctypes.byref(st), int(gather), _ptr(ov),
                                                             _ptr(score), int(k), _ptr(tki) if k else None,
                                                             _ptr(tks) if k else None))
    return ov, score, tki, tks
