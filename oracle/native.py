"""ORACLE -- test infrastructure only. ctypes wrapper of oracle/libdice_oracle.so (dice_ref.c).

Used by tests/ (large-scale parity through size-independent checks) and by bench.py's
``cpu_baseline`` leg; never by the product.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, 'libdice_oracle.so')
_lib = None


def lib():
    global _lib
    if _lib is None:
        l = ctypes.CDLL(LIB)
        vp = ctypes.c_void_p
        l.oracle_create.restype = vp
        l.oracle_create.argtypes = [ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp, vp, vp]
        l.oracle_destroy.argtypes = [vp]
        l.oracle_match.restype = ctypes.c_int
        l.oracle_match.argtypes = [vp, ctypes.c_int64, ctypes.c_int, vp, vp, vp, vp, vp, vp,
                                   ctypes.c_double, ctypes.c_int, vp, vp, vp]
        l.oracle_matrix.restype = ctypes.c_int
        l.oracle_matrix.argtypes = [vp, ctypes.c_int64, vp, vp, vp, vp, vp, ctypes.c_int, vp, vp]
        _lib = l
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


def bits_to_csr(bits: np.ndarray, n_vocab: int):
    """[n, w64] uint64 bitsets -> (offsets int64[n+1], ids int32) of set bits."""
    n = bits.shape[0]
    unpacked = np.unpackbits(bits.view(np.uint8).reshape(n, -1), axis=1, bitorder='little')[:, :n_vocab]
    rows, cols = np.nonzero(unpacked)
    off = np.zeros(n + 1, np.int64)
    np.add.at(off, rows + 1, 1)
    return np.cumsum(off), cols.astype(np.int32)


class OracleScorer:
    def __init__(self, lf_bits, lf_size, fields_set_size, length_slack, length, is_cc, n_vocab):
        off, ids = bits_to_csr(np.ascontiguousarray(lf_bits, np.uint64), n_vocab)
        self._keep = [off.astype(np.int32), ids, np.ascontiguousarray(fields_set_size, np.uint32),
                      np.ascontiguousarray(length_slack, np.int32), np.ascontiguousarray(length, np.int32),
                      np.ascontiguousarray(is_cc, np.uint8)]
        self.T = lf_bits.shape[0]
        self.V = n_vocab
        self._c = lib().oracle_create(self.T, n_vocab, *[_p(a) for a in self._keep])
        if not self._c:
            raise MemoryError('oracle_create failed')

    def __del__(self):
        if getattr(self, '_c', None):
            lib().oracle_destroy(self._c)
            self._c = None

    def match(self, bits, wf, lenf, ccfp, thr, nthreads=1, mode=0, csr=None):
        n = bits.shape[0]
        best = np.empty(n, np.int32)
        ov = np.empty(n, np.uint32)
        score = np.empty(n, np.float64)
        off, ids = csr if csr is not None else ((None, None) if mode == 1 else bits_to_csr(bits, self.V))
        rc = lib().oracle_match(self._c, n, mode, _p(off), _p(ids), _p(np.ascontiguousarray(bits)),
                                _p(wf), _p(lenf), _p(ccfp), float(thr), int(nthreads),
                                _p(best), _p(ov), _p(score))
        if rc:
            raise RuntimeError('oracle_match failed')
        return best, ov, score

    def matrix(self, bits, wf, lenf, ccfp, nthreads=1):
        n = bits.shape[0]
        off, ids = bits_to_csr(bits, self.V)
        mov = np.empty((n, self.T), np.uint32)
        msc = np.empty((n, self.T), np.float64)
        rc = lib().oracle_matrix(self._c, n, _p(off), _p(ids), _p(wf), _p(lenf), _p(ccfp), int(nthreads),
                                 _p(mov), _p(msc))
        if rc:
            raise RuntimeError('oracle_matrix failed')
        return mov, msc
