"""GPU parity: the HIP path (through the C-ABI) against the oracle, bit-exact.

Keys (argmax index) and overlap counts must be identical; scores are compared as IEEE
doubles with ==, i.e. bit-exact (tolerance 0; the north star allows 1e-9).
"""
import numpy as np
import pytest

from oracle import dice_oracle as O
from tests.helpers import NormFile, make_files, oracle_templates

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def templates():
    from licensee_amd.license import License
    return License.all(hidden=True, pseudo=False)


@pytest.fixture(scope='module', params=['program', 'dense'])
def engine(request, templates, monkeypatch_module):
    from licensee_amd.dice import DiceEngine
    if request.param == 'dense':
        monkeypatch_module.setenv('DICE_FORCE_DENSE', '1')
    else:
        monkeypatch_module.delenv('DICE_FORCE_DENSE', raising=False)
    eng = DiceEngine(templates, device=0)
    assert eng.scorer.info()[2] == (1 if request.param == 'program' else 0)
    yield eng
    eng.scorer.close()


@pytest.fixture(scope='module')
def monkeypatch_module():
    mp = pytest.MonkeyPatch()
    yield mp
    mp.undo()


@pytest.fixture(scope='module')
def otpl(templates):
    return oracle_templates(templates)


def _check_match(engine, otpl, files, thr):
    best, ov, score = engine.scorer.match(engine.intern(files), thr)
    for i, f in enumerate(files):
        ranked = O.matches_by_similarity(otpl, f.oracle, cc_fp=f.cc)
        if ranked:
            ti, ts = ranked[0]
            exp_best = ti if ts >= thr else -1
            exp_ov = O.overlap(otpl[ti], f.oracle.wordset)
        else:
            exp_best, ts, exp_ov = -1, 0.0, 0
        assert best[i] == exp_best, (i, best[i], exp_best)
        assert ov[i] == exp_ov, (i, ov[i], exp_ov)
        assert score[i] == ts, (i, score[i], ts)


@pytest.mark.parametrize('n,seed', [(1, 1), (63, 2), (64, 3), (65, 4), (700, 5)])
def test_match_synthetic(engine, templates, otpl, n, seed):
    _check_match(engine, otpl, make_files(templates, n, seed), 98.0)


@pytest.mark.parametrize('thr', [0.0, 50.0, 98.0, 100.0, 100.5])
def test_match_thresholds(engine, templates, otpl, thr):
    _check_match(engine, otpl, make_files(templates, 200, 11), thr)


def test_templates_match_themselves(engine, templates, otpl):
    files = [NormFile(l.content_normalized()) for l in templates]
    best, ov, score = engine.scorer.match(engine.intern(files), 98.0)
    assert best.tolist() == list(range(len(templates)))
    assert np.all(score == 100.0)


def test_cc_filter_and_edges(engine, templates, otpl):
    cc_by = [l for l in templates if l.key == 'cc-by-4.0'][0].content_normalized()
    files = [NormFile(cc_by, cc=True), NormFile(cc_by, cc=False), NormFile(''), NormFile('not really a license')]
    _check_match(engine, otpl, files, 98.0)
    best, _, _ = engine.scorer.match(engine.intern(files), 98.0)
    assert best[0] == -1 and templates[best[1]].key == 'cc-by-4.0'


def test_matrix_and_topk(engine, templates, otpl):
    files = make_files(templates, 130, 21)
    ov, score, tki, tks = engine.scorer.matrix(engine.intern(files), 5)
    for i, f in enumerate(files):
        for t, ot in enumerate(otpl):
            o, d, s = O.similarity_parts(ot, f.oracle)
            assert ov[i, t] == o and score[i, t] == s, (i, t)
        ranked = O.matches_by_similarity(otpl, f.oracle, cc_fp=f.cc)[:5]
        assert tki[i].tolist() == [r[0] for r in ranked] + [-1] * (5 - len(ranked))
        assert tks[i, :len(ranked)].tolist() == [r[1] for r in ranked]
