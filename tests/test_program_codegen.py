"""CPU test of the generated sparse-program kernels (csrc/dice_program.cpp).

The HIP source the library generates for a corpus is compiled for the HOST with g++ under a
small shim (tests/codegen/host_shim.h) and run lane by lane; results must equal the C
oracle bit-for-bit. This checks the code generator (entry list, baked-in constants, CC
masks, argmax / top-k epilogues, fast/slow compare paths) without a GPU.
"""
import ctypes
import os
import shutil
import subprocess

import numpy as np
import pytest

from tests.helpers import NormFile, make_files

HERE = os.path.dirname(os.path.abspath(__file__))


def tile_pack(bits: np.ndarray, wq: int, qperm=None) -> np.ndarray:
    """Row-major [n][w64] uint64 -> tile layout [n_tiles][wq][64] of 4 x uint32; with ``qperm``
    tile slot i holds vocabulary quad qperm[i] (dice_pack_tiles)."""
    n, w64 = bits.shape
    nt = (n + 63) // 64
    d32 = np.zeros((nt * 64, wq * 4), np.uint32)
    d32[:n, :w64 * 2] = bits.view(np.uint32).reshape(n, w64 * 2)
    t = d32.reshape(nt, 64, wq, 4)
    if qperm is not None:
        t = t[:, :, np.asarray(qperm, np.int64), :]
    return np.ascontiguousarray(t.transpose(0, 2, 1, 3))


def source_qperm(src: str):
    """The tile permutation a generated program declares (`// QPERM ...`), or None (identity)."""
    for line in src.splitlines():
        if line.startswith('// QPERM'):
            q = [int(x) for x in line.split()[2:]]
            return q or None
    return None


def _templates_struct(corpus):
    from licensee_amd import _native
    keep = [np.ascontiguousarray(x) for x in (corpus.lf_bits, corpus.lf_size, corpus.fields_set_size,
                                              corpus.length_slack, corpus.length, corpus.is_cc)]
    return keep, _native._Templates(len(corpus.lf_size), corpus.n_vocab, *[k.ctypes.data for k in keep])


def generated_source(corpus) -> str:
    from licensee_amd import _native
    lib = _native.load_library()
    keep, t = _templates_struct(corpus)
    n = lib.dice_program_source(ctypes.byref(t), None, 0)
    buf = ctypes.create_string_buffer(n + 1)
    lib.dice_program_source(ctypes.byref(t), buf, n + 1)
    return buf.value.decode()


def run_host(corpus, fb, k, tmp_path, with_votes=False):
    """Run the generated kernels on the host; with ``with_votes`` also return the number of
    64-file waves of the match kernel whose wave-wide vote chose the IEEE slow path."""
    src = generated_source(corpus)
    d = str(tmp_path)
    with open(os.path.join(d, 'prog.inc'), 'w') as fh:
        fh.write(src)
    shutil.copy(os.path.join(HERE, 'codegen', 'host_shim.h'), d)
    exe = os.path.join(d, 'drv')
    subprocess.run(['g++', '-O1', '-std=c++17', '-w', '-I', d, '-o', exe, os.path.join(HERE, 'codegen', 'driver.cpp')],
                   check=True)
    wq = (corpus.w64 + 1) // 2
    n = fb.n
    npad = ((n + 63) // 64) * 64
    qperm = source_qperm(src)
    assert qperm is None or sorted(qperm) == list(range(wq))
    tile_pack(fb.bits, wq, qperm).tofile(os.path.join(d, 'tiles.bin'))
    for name, arr, dt in (('wf', fb.wordset_size, np.uint32), ('len', fb.length, np.int32),
                          ('cc', fb.cc_false_positive, np.uint8)):
        pad = np.zeros(npad, dt)
        pad[:n] = arr
        pad.tofile(os.path.join(d, name + '.bin'))
    out = subprocess.run([exe, d, str(n), str(k)], check=True, capture_output=True, text=True).stdout
    slow_waves = int(out.split('slow_waves ')[1].split()[0])
    T = corpus.lf_bits.shape[0]
    rd = lambda name, dt: np.fromfile(os.path.join(d, name), dt)
    res = (rd('best.out', np.int32), rd('ov.out', np.uint32), rd('score.out', np.float64),
            # device matrix layout is template-major: [T][n] and [k][n]
            rd('mov.out', np.uint32).reshape(T, n).T, rd('msc.out', np.float64).reshape(T, n).T,
           rd('tki.out', np.int32).reshape(max(k, 1), n)[:k].T, rd('tks.out', np.float64).reshape(max(k, 1), n)[:k].T)
    return res + (slow_waves,) if with_votes else res


@pytest.mark.skipif(shutil.which('g++') is None, reason='needs g++')
@pytest.mark.parametrize('k', [3, 5])
def test_generated_program_matches_oracle(tmp_path, k):
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.license import License
    from oracle import dice_oracle as O
    from oracle.native import OracleScorer
    from tests.helpers import oracle_templates

    templates = License.all(hidden=True, pseudo=False)
    corpus = TemplateCorpus(templates)
    files = make_files(templates, 600, 21) + [NormFile(''), NormFile('x' * 10, cc=True)]
    fb = corpus.intern_files(files)
    best, ov, score, mov, msc, tki, tks = run_host(corpus, fb, k, tmp_path)
    orc = OracleScorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack,
                       corpus.length, corpus.is_cc, corpus.n_vocab)
    eb, eo, es = orc.match(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, 98.0)
    assert np.array_equal(best, eb) and np.array_equal(ov, eo) and np.array_equal(score, es)
    emov, emsc = orc.matrix(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive)
    assert np.array_equal(mov, emov) and np.array_equal(msc, emsc)
    otpl = oracle_templates(templates)
    for i, f in enumerate(files):
        ranked = O.matches_by_similarity(otpl, f.oracle, cc_fp=f.cc)[:k]
        assert tki[i].tolist() == [r[0] for r in ranked] + [-1] * (k - len(ranked)), i
        assert tks[i, :len(ranked)].tolist() == [r[1] for r in ranked], i


@pytest.mark.skipif(shutil.which('g++') is None, reason='needs g++')
def test_exact_ties_later_key_wins(tmp_path, monkeypatch):
    """Corpus with byte-identical templates under later keys: every file ties between a template
    and its clone, and the clone (later in key order) must rank first (dice.rb:39, stable sort +
    reverse), in the argmax and in the top-k."""
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.license import License
    from oracle.native import OracleScorer
    base = [License.find(k) for k in ('apache-2.0', 'bsd-2-clause', 'isc', 'mit', 'mpl-2.0', 'unlicense')]
    clones = [License('zz-' + l.key, {'title': l.title}, content_normalized=l.content_normalized(),
                      alt_segments=l.spdx_alt_segments()) for l in base]
    templates = sorted(base + clones, key=lambda l: l.key)
    corpus = TemplateCorpus(templates)
    files = make_files(templates, 300, 5) + [NormFile('')]
    fb = corpus.intern_files(files)
    best, ov, score, mov, msc, tki, tks = run_host(corpus, fb, 3, tmp_path)
    orc = OracleScorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack,
                       corpus.length, corpus.is_cc, corpus.n_vocab)
    eb, eo, es = orc.match(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, 98.0)
    assert np.array_equal(best, eb) and np.array_equal(ov, eo) and np.array_equal(score, es)
    keys = [t.key for t in templates]
    matched = best[best >= 0]
    assert len(matched) > 50 and all(keys[b].startswith('zz-') for b in matched)
    assert all(keys[i].startswith('zz-') for i in tki[:, 0] if i >= 0)


def _check_vs_oracle(corpus, fb, got, k):
    from oracle.native import OracleScorer
    best, ov, score, mov, msc, tki, tks = got
    orc = OracleScorer(*corpus.arrays() if hasattr(corpus, 'arrays') else
                       (corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack,
                        corpus.length, corpus.is_cc), n_vocab=corpus.n_vocab)
    # hash mode: the Set#& restatement, independent of the kernels' AND+popcount formulation
    eb, eo, es = orc.match(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, 98.0, mode=0)
    assert np.array_equal(best, eb) and np.array_equal(ov, eo) and np.array_equal(score, es)
    emov, emsc = orc.matrix(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive)
    assert np.array_equal(mov, emov) and np.array_equal(msc, emsc)
    # top-k: the k best of the (CC-filtered) row in stable-ascending-then-reversed order
    T = mov.shape[1]
    for i in range(fb.n):
        cand = [t for t in range(T) if not (corpus.is_cc[t] and fb.cc_false_positive[i])]
        ranked = sorted(cand, key=lambda t: (emsc[i, t], t), reverse=True)[:k]
        assert tki[i].tolist() == ranked + [-1] * (k - len(ranked)), i
        assert tks[i, :len(ranked)].tolist() == [emsc[i, t] for t in ranked], i


@pytest.mark.skipif(shutil.which('g++') is None, reason='needs g++')
def test_mixed_fast_slow_waves(tmp_path, monkeypatch):
    """Waves that mix fast lanes with lanes outside the fast envelope (|W_F| >= 2^20 or
    len_F >= 2^21) run MATCH_BODY(false) / MATRIX_BODY(false) -- the IEEE-double compares --
    for all 64 lanes (the shim's __all is wave-wide); other waves keep the exact rational path.
    Both must equal the oracle's hash mode bit for bit (content_helper.rb:128-133)."""
    from licensee_amd._native import FileBatch
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.license import License
    from tests.helpers import widen_lanes
    templates = License.all(hidden=True, pseudo=False)
    corpus = TemplateCorpus(templates)
    fb0 = corpus.intern_files(make_files(templates, 1024, 8))
    fb, idx = widen_lanes(fb0, seed=3)
    # waves 8..15 stay entirely fast: the same run covers both vote outcomes
    wf, ln = fb.wordset_size.copy(), fb.length.copy()
    wf[512:], ln[512:] = fb0.wordset_size[512:], fb0.length[512:]
    fb = FileBatch(fb.bits, wf, ln, fb.cc_false_positive)
    got = run_host(corpus, fb, 5, tmp_path, with_votes=True)
    assert got[-1] == 8, got[-1]
    _check_vs_oracle(corpus, fb, got[:-1], 5)


@pytest.mark.skipif(shutil.which('g++') is None, reason='needs g++')
def test_corpus_outside_fast_envelope(tmp_path, monkeypatch):
    """A corpus breaking 200*|Lf| < 1024*base (and one template length >= 2^20) compiles with
    CORPUS_FAST 0: every wave takes the IEEE-double path; scores above 100 occur."""
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.license import License
    from tests.helpers import outside_fast_envelope
    templates = License.all(hidden=True, pseudo=False)
    corpus = outside_fast_envelope(TemplateCorpus(templates))
    assert '#define CORPUS_FAST 0' in generated_source(corpus)
    fb = TemplateCorpus(templates).intern_files(make_files(templates, 300, 12) + [NormFile('')])
    got = run_host(corpus, fb, 4, tmp_path, with_votes=True)
    assert got[-1] == (fb.n + 63) // 64
    _check_vs_oracle(corpus, fb, got[:-1], 4)
    assert (got[2] > 100.0).any()
