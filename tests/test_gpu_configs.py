"""GPU parity at the BASELINE configs 3 and 4, through the C-ABI.

  * config 4 -- long/mixed COPYING files (SyntheticCorpus profile 1: 2-6 templates
    concatenated plus a 50-300-word notice; dice_matcher_spec.rb:43-54 stacks MIT+GPL) x the
    47 vendored templates: bit-exact vs the C oracle's hash mode (Set#& restatement) on 12k
    files (match, full matrix, top-k), then 1M files (the bench size) through size-independent
    properties: two launches bit-identical, match == thresholded top-1 of the matrix kernel,
    top-k sorted and consistent with the matrix rows, CC filter, and a 20k oracle sample.
  * config 3 -- one GPU's shard of the 10M x ~600-template run (1.25M files), postings kernel
    (default) and LDS record kernel: two launches bit-identical (for the LDS kernel also its
    asm-wait convention, dice_lds.hip:54-66), a 20k oracle sample in hash mode, and the
    match/matrix top-1 agreement on 50k files.
"""
import numpy as np
import pytest

from licensee_amd.license import License

pytestmark = pytest.mark.gpu


def _scorer(corpus):
    from licensee_amd._native import Scorer
    return Scorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack, corpus.length,
                  corpus.is_cc, corpus.n_vocab, device=0)


def _oracle(corpus):
    from oracle.native import OracleScorer
    return OracleScorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack,
                        corpus.length, corpus.is_cc, corpus.n_vocab)


def _sub(fb, idx):
    from licensee_amd._native import FileBatch
    return FileBatch(fb.bits[idx], fb.wordset_size[idx], fb.length[idx], fb.cc_false_positive[idx])


def _sample_vs_oracle(orc, fb, best, ov, score, n_sample, seed, thr=98.0):
    idx = np.sort(np.random.default_rng(seed).choice(fb.n, min(n_sample, fb.n), replace=False))
    s = _sub(fb, idx)
    eb, eo, es = orc.match(s.bits, s.wordset_size, s.length, s.cc_false_positive, thr, nthreads=16, mode=0)
    assert np.array_equal(best[idx], eb) and np.array_equal(ov[idx], eo) and np.array_equal(score[idx], es)


def _topk_properties(corpus, fb, best, ov, score, mov, msc, tki, tks, thr=98.0):
    rows = np.arange(fb.n)
    assert np.array_equal(tks[:, 0], score)
    assert np.array_equal(np.where(tks[:, 0] >= thr, tki[:, 0], -1), best)
    assert np.array_equal(mov[rows, tki[:, 0]], ov)
    for j in range(tki.shape[1] - 1):
        assert (tks[:, j] >= tks[:, j + 1]).all()
    for j in range(tki.shape[1]):
        assert np.array_equal(msc[rows, tki[:, j]], tks[:, j])
    cc_t = np.nonzero(corpus.is_cc)[0]
    assert not np.isin(tki[fb.cc_false_positive.astype(bool)], cc_t).any()


@pytest.fixture(scope='module')
def vendored():
    from licensee_amd.corpus import TemplateCorpus
    return TemplateCorpus(License.all(hidden=True, pseudo=False))


def test_config4_long_mixed_vs_oracle(vendored):
    from licensee_amd.synth import SyntheticCorpus
    corpus = vendored
    syn = SyntheticCorpus(corpus, profile=1)
    fb = syn.generate(0, 12_000, seed=20250202, nthreads=16)
    # long files: |W_F| well above any template's, many out-of-vocabulary words
    assert np.median(fb.length) > 10_000 and fb.wordset_size.max() > corpus.lf_size.max()
    sc, orc = _scorer(corpus), _oracle(corpus)
    best, ov, score = sc.match(fb, 98.0)
    eb, eo, es = orc.match(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, 98.0, nthreads=16, mode=0)
    assert np.array_equal(best, eb) and np.array_equal(ov, eo) and np.array_equal(score, es)
    mov, msc, tki, tks = sc.matrix(fb, 5)
    emov, emsc = orc.matrix(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, nthreads=16)
    assert np.array_equal(mov, emov) and np.array_equal(msc, emsc)
    _topk_properties(corpus, fb, best, ov, score, mov, msc, tki, tks)
    # stacked licenses do not match (dice_matcher_spec.rb:43-54): profile-1 files concatenating
    # >= 2 templates stay below the threshold
    assert (best >= 0).mean() < 0.05
    sc.close()


def test_config4_full_size_properties(vendored):
    from licensee_amd.synth import SyntheticCorpus
    corpus = vendored
    fb = SyntheticCorpus(corpus, profile=1).generate(0, 1_000_000, seed=20250202, nthreads=16)
    sc = _scorer(corpus)
    batch = sc.batch(fb.n)
    batch.upload(fb)
    batch.match(98.0)
    best, ov, score = batch.download_match()
    batch.match(98.0)
    b2, o2, s2 = batch.download_match()
    assert np.array_equal(best, b2) and np.array_equal(ov, o2) and np.array_equal(score, s2)
    batch.matrix(3)
    mov, msc, tki, tks = batch.download_matrix(3)
    _topk_properties(corpus, fb, best, ov, score, mov, msc, tki, tks)
    # every file against the independent hash-set Set#& restatement
    eb, eo, es = _oracle(corpus).match(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, 98.0,
                                       nthreads=16, mode=0)
    assert np.array_equal(best, eb) and np.array_equal(ov, eo) and np.array_equal(score, es)
    batch.close()
    sc.close()


@pytest.mark.parametrize('kernel', ['post', 'post-allpairs', 'lds'])
def test_config3_shard(kernel, monkeypatch):
    """The 1.25M-file config-3 shard on each large-corpus match path: 'post' runs the bound-pruned
    kernel (dice_prune.hip), checked on every file against the oracle's bitset mode (a full scan,
    independent of the pruning) plus a hash-mode sample; 'post-allpairs' the postings kernels."""
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.synth import SyntheticCorpus
    from licensee_amd.synth_templates import synthetic_templates
    for k in ('DICE_FORCE_DENSE', 'DICE_POST_DENSE'):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv('DICE_LARGE_KERNEL', 'lds' if kernel == 'lds' else 'post')
    monkeypatch.setenv('DICE_POST_PRUNE', '0' if kernel == 'post-allpairs' else '1')
    corpus = TemplateCorpus(synthetic_templates(License.all(hidden=True, pseudo=False), 600, seed=20250202))
    fb = SyntheticCorpus(corpus).generate(0, 1_250_000, seed=20250202, nthreads=16)
    sc = _scorer(corpus)
    assert sc.info()[2] == {'lds': 2, 'post': 3, 'post-allpairs': 3}[kernel]
    assert sc.match_kernel() == {'lds': 2, 'post': 4, 'post-allpairs': 3}[kernel]
    batch = sc.batch(fb.n)
    batch.upload(fb)
    batch.match(98.0)
    best, ov, score = batch.download_match()
    batch.match(98.0)
    b2, o2, s2 = batch.download_match()
    assert np.array_equal(best, b2) and np.array_equal(ov, o2) and np.array_equal(score, s2)
    assert ((best >= 0) == (score >= 98.0)).all() and best.max() < 600
    _sample_vs_oracle(_oracle(corpus), fb, best, ov, score, 20_000, seed=5)
    if kernel == 'post':
        eb, eo, es = _oracle(corpus).match(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, 98.0,
                                           nthreads=16, mode=1)
        assert np.array_equal(best, eb) and np.array_equal(ov, eo) and np.array_equal(score, es)
        # the bench's config-3 entry point (dice_batch_match_confidence: Dice#match + #confidence,
        # dice.rb:8-14,51-53) on every file of the shard: the oracle's match with the unmatched
        # files' overlap and score 0
        batch.match(98.0, confidence=True)
        cb, co, cs = batch.download_match()
        m = eb >= 0
        assert np.array_equal(cb, eb)
        assert np.array_equal(co, np.where(m, eo, 0)) and np.array_equal(cs, np.where(m, es, 0.0))
    batch.close()
    # matrix/top-k on a 50k slice agrees with the match kernel's argmax
    s = _sub(fb, np.arange(50_000))
    mov, msc, tki, tks = sc.matrix(s, 4)
    _topk_properties(corpus, s, best[:50_000], ov[:50_000], score[:50_000], mov, msc, tki, tks)
    sc.close()
