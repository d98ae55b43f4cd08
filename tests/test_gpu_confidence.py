"""GPU parity of the confidence entry points (dice_match_confidence, dice_batch_match_confidence).

A caller of the matcher reads Dice#match and Dice#confidence (dice.rb:8-14, 51-53): the matched
template and its similarity, or nil and 0 when no template reaches the threshold
(dice.rb:44-48). The confidence calls return exactly that -- best as dice_match, overlap/score of
the matched template, 0/0.0 for a file without a match -- and the bound-pruned kernel (T > 64)
uses it to drop every template whose bound is below the threshold from the start.

Expected values: the C oracle's Dice#match (hash mode, the Set#& restatement of
content_helper.rb:128-133) with the unmatched files' overlap and score set to 0. Checked on every
kernel (sparse program T <= 64, postings / pruned / LDS records T > 64, dense), for the small
host-buffer call, the batch call, deferral knobs and thresholds 98 (Licensee's default), 0, 50
and 100.5 (nothing matches).
"""
import numpy as np
import pytest

from tests.test_gpu_corpus_sizes import KIND, corpus_of, select_kernel
from tests.test_gpu_prune import _random_files

pytestmark = pytest.mark.gpu

THRESHOLDS = (98.0, 0.0, 50.0, 100.5)


def _expected(orc, fb, thr):
    best, ov, score = orc.match(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, thr, nthreads=16,
                                mode=0)
    ov = np.where(best >= 0, ov, 0).astype(np.uint32)
    score = np.where(best >= 0, score, 0.0)
    return best, ov, score


def _same(got, exp, where):
    for name, g, e in zip(('best', 'overlap', 'score'), got, exp):
        assert np.array_equal(g, e), (where, name, np.nonzero(g != e)[0][:10])


def _scorer(c):
    from licensee_amd._native import Scorer
    return Scorer(c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc, c.n_vocab, device=0)


def _oracle(c):
    from oracle.native import OracleScorer
    return OracleScorer(c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc, c.n_vocab)


def _check(sc, orc, fb, thresholds=THRESHOLDS):
    """Host call, batch call, and agreement with dice_match on the matched files."""
    for thr in thresholds:
        exp = _expected(orc, fb, thr)
        got = sc.match(fb, thr, confidence=True)
        _same(got, exp, ('dice_match_confidence', thr))
        full = sc.match(fb, thr)
        m = full[0] >= 0
        assert np.array_equal(full[0], got[0])
        assert np.array_equal(full[1][m], got[1][m]) and np.array_equal(full[2][m], got[2][m])
        b = sc.batch(max(fb.n, 1))
        try:
            b.upload(fb)
            b.match(thr, confidence=True)
            _same(b.download_match(), exp, ('dice_batch_match_confidence', thr))
        finally:
            b.close()


@pytest.fixture(scope='module')
def config3():
    import bench
    from licensee_amd.synth import SyntheticCorpus
    c = bench.build_workload(3)
    fb = SyntheticCorpus(c).generate(0, 20000, seed=20251017, nthreads=16)
    return c, fb


@pytest.mark.parametrize('prune', ['1', '0'])
def test_config3(config3, prune, monkeypatch):
    monkeypatch.setenv('DICE_POST_PRUNE', prune)
    c, fb = config3
    sc = _scorer(c)
    try:
        assert sc.match_kernel() == (4 if prune == '1' else 3)
        _check(sc, _oracle(c), fb)
    finally:
        sc.close()


@pytest.mark.parametrize('env', [{'DICE_PRUNE_MAX_EVALS': '1'}, {'DICE_PRUNE_MAX_EVALS': '0'},
                                 {'DICE_PRUNE_ROUTE': '0'}])
def test_config3_deferral_knobs(config3, env, monkeypatch):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    c, fb = config3
    from licensee_amd._native import FileBatch
    part = FileBatch(fb.bits[:3000], fb.wordset_size[:3000], fb.length[:3000], fb.cc_false_positive[:3000])
    sc = _scorer(c)
    try:
        _check(sc, _oracle(c), part, thresholds=(98.0, 50.0))
    finally:
        sc.close()


def test_config3_files_resembling_nothing(config3):
    """Random bitsets (loose bounds, empty and CC-flagged files): almost nothing reaches 98."""
    c, _ = config3
    sc = _scorer(c)
    try:
        _check(sc, _oracle(c), _random_files(c, 1500, seed=31, density=0.05))
    finally:
        sc.close()


@pytest.mark.parametrize('n_templates,kernel', [(47, 'program'), (47, 'dense'), (200, 'lds'), (200, 'post')])
def test_every_kernel(n_templates, kernel, monkeypatch):
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.synth import SyntheticCorpus
    select_kernel(monkeypatch, kernel)
    c = TemplateCorpus(corpus_of(n_templates))
    fb = SyntheticCorpus(c).generate(0, 3000, seed=n_templates + 17, nthreads=8)
    sc = _scorer(c)
    try:
        assert sc.info()[2] == KIND[kernel]
        _check(sc, _oracle(c), fb)
    finally:
        sc.close()


@pytest.mark.parametrize('n', [1, 5, 64, 65])
def test_small_calls(config3, n):
    """The small host-buffer path (one H2D, one D2H) with confidence outputs."""
    from licensee_amd._native import FileBatch
    c, fb = config3
    lo = 1234
    part = FileBatch(fb.bits[lo:lo + n], fb.wordset_size[lo:lo + n], fb.length[lo:lo + n],
                     fb.cc_false_positive[lo:lo + n])
    sc = _scorer(c)
    try:
        _check(sc, _oracle(c), part)
    finally:
        sc.close()


def _equality_thresholds(orc, fb, count=20):
    """`count` distinct exact top scores that occur in fb (the oracle's dice_match scores at
    threshold 0), spread over their range and including the largest below 100 and one >= 98."""
    _, _, top = orc.match(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, 0.0, nthreads=16, mode=1)
    u = np.unique(top[top > 0])
    pick = set(u[np.linspace(0, u.size - 1, count - 2).round().astype(int)].tolist())
    hi = u[(u >= 98.0) & (u < 100.0)]
    assert hi.size, 'no file scores in [98, 100)'
    pick.add(float(hi[hi.size // 2]))
    pick.add(float(u[u < 100.0].max()))
    return top, sorted(pick)[-count:]


def _check_equality(sc, orc, fb, top, thresholds, where):
    """Dice#matches keeps similarity >= minimum_confidence (dice.rb:44-48): a file whose top score
    EQUALS the threshold matches. The pruned kernels start their drop level at an f32 floor of the
    threshold; every such file must still match, identical to the oracle."""
    for thr in thresholds:
        exp = _expected_bitset(orc, fb, thr)
        eq = top == thr
        assert eq.any() and (exp[0][eq] >= 0).all(), (where, thr)
        got = sc.match(fb, thr, confidence=True)
        _same(got, exp, (where, 'dice_match_confidence', thr))
        full = sc.match(fb, thr)
        m = exp[0] >= 0
        assert np.array_equal(full[0], exp[0]), (where, 'dice_match', thr)
        assert np.array_equal(full[1][m], exp[1][m]) and np.array_equal(full[2][m], exp[2][m]), (where, thr)
        assert np.array_equal(full[2], top), (where, 'dice_match top score', thr)


def _expected_bitset(orc, fb, thr):
    best, ov, score = orc.match(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, thr, nthreads=16,
                                mode=1)
    return best, np.where(best >= 0, ov, 0).astype(np.uint32), np.where(best >= 0, score, 0.0)


@pytest.mark.parametrize('prune', ['1', '0'])
def test_threshold_equal_to_achieved_score_T600(config3, prune, monkeypatch):
    """20 exact scores achieved in a 20k-file config-3 sample as thresholds, on
    the bound-pruned kernel (and the postings kernels as a control)."""
    monkeypatch.setenv('DICE_POST_PRUNE', prune)
    c, fb = config3
    orc = _oracle(c)
    top, thresholds = _equality_thresholds(orc, fb)
    assert len(thresholds) == 20
    sc = _scorer(c)
    try:
        assert sc.match_kernel() == (4 if prune == '1' else 3)
        _check_equality(sc, orc, fb, top, thresholds, ('T600', prune))
        b = sc.batch(fb.n)
        try:
            b.upload(fb)
            for thr in thresholds[::4] + thresholds[-2:]:
                b.match(thr, confidence=True)
                _same(b.download_match(), _expected_bitset(orc, fb, thr), ('batch confidence', thr))
        finally:
            b.close()
    finally:
        sc.close()


def test_threshold_equal_to_achieved_score_T47():
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.license import License
    from licensee_amd.synth import SyntheticCorpus
    c = TemplateCorpus(License.all(hidden=True, pseudo=False))
    fb = SyntheticCorpus(c).generate(0, 20000, seed=4747, nthreads=16)
    orc = _oracle(c)
    top, thresholds = _equality_thresholds(orc, fb)
    sc = _scorer(c)
    try:
        assert sc.match_kernel() == 1
        _check_equality(sc, orc, fb, top, thresholds, 'T47')
    finally:
        sc.close()


def test_threshold_equality_sharded_confidence_three_contexts(config3):
    """dice_match_sharded_confidence over 3 contexts (all on device 0 here), both gathers, at
    thresholds equal to achieved scores."""
    from licensee_amd._native import DICE_GATHER_DEVICE, DICE_GATHER_HOST, match_sharded
    c, fb = config3
    orc = _oracle(c)
    top, thresholds = _equality_thresholds(orc, fb)
    scs = [_scorer(c) for _ in range(3)]
    try:
        for i, thr in enumerate(thresholds[::3] + thresholds[-1:]):
            gather = DICE_GATHER_DEVICE if i % 2 else DICE_GATHER_HOST
            got = match_sharded(scs, fb, thr, gather=gather, confidence=True)
            exp = _expected_bitset(orc, fb, thr)
            assert (exp[0][top == thr] >= 0).all()
            _same(got, exp, ('sharded confidence', gather, thr))
    finally:
        for s in scs:
            s.close()


def test_scored_pairs_counted_on_device(config3, monkeypatch):
    """dice_batch_scored_pairs: the postings kernels score every pair (n * T);
    the bound-pruned kernel scores between its deferred files' pairs and n * T, fewer through the
    confidence entry point (its drop level starts at the threshold), and the count is the same for
    two launches of the same batch."""
    c, fb = config3
    n, T = fb.n, len(c.templates)
    for prune in ('0', '1'):
        monkeypatch.setenv('DICE_POST_PRUNE', prune)
        sc = _scorer(c)
        b = sc.batch(n)
        try:
            b.upload(fb)
            b.match(98.0)
            top1 = b.scored_pairs()
            b.match(98.0)
            assert b.scored_pairs() == top1
            if prune == '0':
                assert top1 == n * T
                continue
            d = b.deferred()
            assert d * T <= top1 < n * T // 10, (top1, d)
            b.match(98.0, confidence=True)
            conf = b.scored_pairs()
            assert b.deferred() * T <= conf <= top1, (conf, top1)
        finally:
            b.close()
            sc.close()
