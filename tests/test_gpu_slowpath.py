"""GPU parity of the kernels' IEEE-double slow paths, through the C-ABI.

The sparse program (dice_program.cpp) compares candidates by exact rational
cross-multiplication while every lane of a 64-file wave is inside the fast envelope
(|W_F| < 2^20, 0 <= len_F < 2^21) and the corpus is too (`corpus_in_fast_envelope`);
otherwise the whole wave runs MATCH_BODY(false) / MATRIX_BODY(false) on IEEE doubles. The
LDS and dense kernels decide per pair (dice_common.h `dice_ge`). Here:

  * waves mixing fast lanes with huge-|W_F| / huge-len_F lanes (set directly in the
    FileBatch, as a file with ~10^6 out-of-vocabulary words would have them) next to waves
    that stay fast;
  * a corpus outside the fast envelope (|Lf| - |Fld| = 1, a template length >= 2^20);

each checked bit-exact -- best, overlap, score, the full matrix and the top-k -- against the
C oracle's hash mode (the Set#& restatement of content_helper.rb:128-133).
"""
import numpy as np
import pytest

from licensee_amd.license import License
from tests.helpers import make_files, outside_fast_envelope, widen_lanes

pytestmark = pytest.mark.gpu


def _scorer(corpus):
    from licensee_amd._native import Scorer
    return Scorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack, corpus.length,
                  corpus.is_cc, corpus.n_vocab, device=0)


def _oracle(corpus):
    from oracle.native import OracleScorer
    return OracleScorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack,
                        corpus.length, corpus.is_cc, corpus.n_vocab)


def _check(sc, orc, fb, is_cc, k=5, thresholds=(98.0, 0.0)):
    for thr in thresholds:
        best, ov, score = sc.match(fb, thr)
        eb, eo, es = orc.match(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, thr, nthreads=16, mode=0)
        assert np.array_equal(ov, eo) and np.array_equal(score, es) and np.array_equal(best, eb), thr
    mov, msc, tki, tks = sc.matrix(fb, k)
    emov, emsc = orc.matrix(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, nthreads=16)
    assert np.array_equal(mov, emov) and np.array_equal(msc, emsc)
    # top-k = the stable-ascending-then-reversed ranking of the CC-filtered row (dice.rb:23-41)
    T = emsc.shape[1]
    tie_key = np.broadcast_to(np.arange(T), emsc.shape)
    order = np.lexsort((tie_key, emsc), axis=1)[:, ::-1]
    for i in range(fb.n):
        row = [t for t in order[i] if not (is_cc[t] and fb.cc_false_positive[i])][:k]
        assert tki[i].tolist() == row + [-1] * (k - len(row)), i
        assert tks[i, :len(row)].tolist() == emsc[i, row].tolist(), i
    return score


@pytest.fixture(scope='module')
def vendored():
    from licensee_amd.corpus import TemplateCorpus
    templates = License.all(hidden=True, pseudo=False)
    return templates, TemplateCorpus(templates)


def test_sparse_program_mixed_waves(vendored):
    from licensee_amd._native import FileBatch
    templates, corpus = vendored
    fb0 = corpus.intern_files(make_files(templates, 4096, 41))
    fb, idx = widen_lanes(fb0, seed=9)
    wf, ln = fb.wordset_size.copy(), fb.length.copy()
    wf[2048:], ln[2048:] = fb0.wordset_size[2048:], fb0.length[2048:]   # second half: all-fast waves
    fb = FileBatch(fb.bits, wf, ln, fb.cc_false_positive)
    assert (wf >= (1 << 20)).any() and (ln >= (1 << 21)).any()
    sc = _scorer(corpus)
    assert sc.info()[2] == 1
    _check(sc, _oracle(corpus), fb, corpus.is_cc, k=5)
    _check(sc, _oracle(corpus), fb, corpus.is_cc, k=16, thresholds=(50.0,))
    sc.close()


def test_sparse_program_corpus_outside_envelope(vendored):
    templates, corpus = vendored
    oc = outside_fast_envelope(corpus)
    fb = corpus.intern_files(make_files(templates, 2000, 43))
    fb, _ = widen_lanes(fb, seed=10, frac=0.05)
    sc = _scorer(oc)
    assert sc.info()[2] == 1
    score = _check(sc, _oracle(oc), fb, oc.is_cc, k=3)
    assert (score > 100.0).any()
    sc.close()


@pytest.mark.parametrize('kernel', ['post', 'lds', 'dense'])
def test_large_corpus_mixed_lanes(kernel, monkeypatch):
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.synth import SyntheticCorpus
    from licensee_amd.synth_templates import synthetic_templates
    monkeypatch.delenv('DICE_POST_DENSE', raising=False)
    monkeypatch.setenv('DICE_LARGE_KERNEL', 'lds' if kernel == 'lds' else 'post')
    if kernel == 'dense':
        monkeypatch.setenv('DICE_FORCE_DENSE', '1')
    else:
        monkeypatch.delenv('DICE_FORCE_DENSE', raising=False)
    corpus = TemplateCorpus(synthetic_templates(License.all(hidden=True, pseudo=False), 600, seed=5))
    fb = SyntheticCorpus(corpus).generate(0, 1500, seed=12, nthreads=8)
    fb, _ = widen_lanes(fb, seed=11)
    oc = outside_fast_envelope(corpus)
    for c in (corpus, oc):
        sc = _scorer(c)
        assert sc.info()[2] == {'dense': 0, 'lds': 2, 'post': 3}[kernel]
        _check(sc, _oracle(c), fb, c.is_cc, k=4)
        sc.close()
