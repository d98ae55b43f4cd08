"""GPU tests of the product path against the reference's goldens and at full BASELINE size.

  * Dice matcher API (matchers.Dice over the HIP matrix kernel) on the
    dice_matcher_spec.rb goldens: exact floats 100.0 / 94.56967213114754 / 26.821370750134918.
  * LicenseFile#license chain (Copyright -> Exact -> Dice on GPU) on the fixtures.yml cases
    and on every vendored_license_spec.rb property case.
  * 1,000,000 synthetic files (BASELINE config 2 size): bit-exact vs the C oracle on a
    sample, plus size-independent properties over all files (idempotence, match/top-k
    consistency, top-k sortedness, CC filter).
  * LDS-tiled and dense kernels at T = 600 synthetic templates (config 3 regime) vs the C oracle.
"""
import json
import os

import numpy as np
import pytest

from licensee_amd.license import License
from licensee_amd.project_files import LicenseFile

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')


def golden(name):
    with open(os.path.join(GOLDEN, name), encoding='utf-8') as fh:
        return json.load(fh)


class GoldenLicenseFile(LicenseFile):
    """A LicenseFile whose normalized content comes from a golden vector (the raw text never
    leaves the build container); Copyright sees no raw content."""

    def __init__(self, rec):
        super().__init__('', 'LICENSE')
        self._content_normalized = rec['normalized']
        self._fp = rec['cc_false_positive']

    def potential_false_positive(self):
        return self._fp


def test_dice_matcher_spec():
    from licensee_amd.matchers import Dice
    cases = golden('dice_spec.json')['cases']
    d = Dice(GoldenLicenseFile(cases['gpl']['file']))
    assert [[l.key, s] for l, s in d.matches_by_similarity()[:3]] == cases['gpl']['by_similarity']
    assert d.match().key == 'gpl-3.0' and d.confidence() == 100.0
    for name in ('not_a_license', 'stacked', 'cc_nd'):
        d = Dice(GoldenLicenseFile(cases[name]['file']))
        assert d.match() is None and d.matches() == [] and d.confidence() == 0 and type(d.confidence()) is int
    lf = GoldenLicenseFile(cases['cc_by']['file'])
    assert lf.license().key == 'cc-by-4.0'
    # LicenseFile#license / #confidence (license_file.rb:92-98, project_file.rb:74-76)
    # the rendered GPL's wordset equals the template's, so the chain stops at Exact (exact.rb:6-12)
    lf = GoldenLicenseFile(cases['gpl']['file'])
    assert lf.license().key == 'gpl-3.0' and lf.confidence() == 100 and lf.matcher().name == 'exact'
    lf = GoldenLicenseFile(cases['stacked']['file'])
    assert lf.license().key == 'other' and lf.matcher() is None
    lf = GoldenLicenseFile(cases['not_a_license']['file'])
    assert lf.license().key == 'other' and lf.confidence() is None
    # License#similarity routed through the GPU (content_helper.rb:128-133)
    agpl = License.find('agpl-3.0')
    assert agpl.similarity(GoldenLicenseFile(cases['gpl']['file'])) == 94.56967213114754
    mit = License.find('mit')
    assert mit.similarity(mit) == 100.0


def test_content_helper_spec_similarity():
    """content_helper_spec.rb:68-75 with the spec's test helper (not a License: simple length
    delta, :343): mit.similarity(h) ~ 4, h.similarity(mit) ~ 3, mit.similarity(mit) == 100.0 --
    and both equal to the formula evaluated on the host sets (content_helper.rb:128-133)."""
    from tests.test_normalize import SPEC_CONTENT, Helper
    h = Helper(SPEC_CONTENT, 'license.md')
    mit = License.find('mit')

    def formula(a, b, simple):
        ov = len(a.wordset_fieldless() & b.wordset())
        total = len(a.wordset_fieldless()) + len(b.wordset()) - len(a.fields_normalized_set())
        delta = abs(a.length() - b.length())
        if not simple:
            delta = max(delta - 5 * max(len(a.fields_normalized()), a.spdx_alt_segments()), 0)
        return (ov * 200.0) / (total + delta // 4)
    s1, s2 = mit.similarity(h), h.similarity(mit)
    assert abs(s1 - 4) <= 1 and abs(s2 - 3) <= 1
    assert s1 == formula(mit, h, False) and s2 == formula(h, mit, True)
    assert mit.similarity(mit) == 100.0


def test_fixture_expectations_on_gpu():
    recs = golden('fixture_files.json')
    singles = [r for r in recs if sum(x['fixture'] == r['fixture'] for x in recs) == 1
               and 'unsupported' not in r and not r['copyright']]
    for r in singles:
        exp = r['expected']
        lf = GoldenLicenseFile(r)
        key = lf.license().key
        m = lf.matcher()
        if exp.get('matcher') in ('dice', 'exact'):
            assert (key, m.name) == (exp['key'], exp['matcher']), r['fixture']
        elif exp.get('key') == 'other':
            assert key == 'other' and m is None, r['fixture']


def test_vendored_properties_batched_on_gpu():
    from licensee_amd.dice import default_engine
    eng = default_engine()
    files, expect, keys = [], [], []
    for t in golden('vendored.json')['templates']:
        for name, rec in t['cases'].items():
            files.append(GoldenLicenseFile(rec))
            expect.append(rec['detected'])
            keys.append(t['key'])
    exact = [next((l.key for l in License.all(hidden=True, pseudo=False) if l.wordset() == f.wordset()), None)
             for f in files]
    dice = eng.match_files(files, 98)
    for i in range(len(files)):
        got = exact[i] or (dice[i][0].key if dice[i][0] is not None else 'other')
        assert (got == keys[i]) == expect[i], (keys[i], i, got)


def test_vendored_confidence_equals_similarity():
    """vendored_license_spec.rb:27-29: for every vendored license rendered with copyright info,
    LicenseFile#confidence == License#similarity(license_file) -- the confidence from the
    matcher chain (Exact, else Dice's batched GPU match) and the similarity from the GPU pair
    path, both equal to the oracle's Set#& restatement (content_helper.rb:128-133)."""
    from oracle import dice_oracle as O
    from tests.helpers import oracle_templates
    licenses = License.all(hidden=True, pseudo=False)
    otpl = {t.key: t for t in oracle_templates(licenses)}
    n = 0
    for t in golden('vendored.json')['templates']:
        rec = t['cases']['rendered']
        f = GoldenLicenseFile(rec)
        lic = License.find(t['key'])
        conf, sim = f.confidence(), lic.similarity(f)
        assert conf == sim, (t['key'], conf, sim)
        assert sim == O.similarity(otpl[t['key']], O.OracleFile(rec['normalized'])), t['key']
        n += 1
    assert n == len(licenses)


@pytest.fixture(scope='module')
def big():
    from licensee_amd._native import Scorer
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.synth import SyntheticCorpus
    corpus = TemplateCorpus(License.all(hidden=True, pseudo=False))
    fb = SyntheticCorpus(corpus).generate(0, 1_000_000, seed=20250202, nthreads=16)
    sc = Scorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack, corpus.length,
                corpus.is_cc, corpus.n_vocab, device=0)
    batch = sc.batch(fb.n)
    batch.upload(fb)
    yield corpus, fb, sc, batch
    batch.close()
    sc.close()


def test_full_size_match_vs_oracle_sample(big):
    from oracle.native import OracleScorer
    corpus, fb, sc, batch = big
    batch.match(98.0)
    best, ov, score = batch.download_match()
    batch.match(98.0)
    best2, ov2, score2 = batch.download_match()
    assert np.array_equal(best, best2) and np.array_equal(ov, ov2) and np.array_equal(score, score2)
    orc = OracleScorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack,
                       corpus.length, corpus.is_cc, corpus.n_vocab)
    # every file, in the bitset mode and in the independent hash-set Set#& restatement (no
    # AND+popcount; content_helper.rb:128-133)
    for mode in (1, 0):
        eb, eo, es = orc.match(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, 98.0, nthreads=16, mode=mode)
        assert np.array_equal(best, eb) and np.array_equal(ov, eo) and np.array_equal(score, es), mode
    assert ((best >= 0) == (score >= 98.0)).all()
    assert best.min() >= -1 and best.max() < len(corpus.templates)


def test_full_size_matrix_consistency(big):
    corpus, fb, sc, batch = big
    k = 3
    batch.match(98.0)
    best, ov, score = batch.download_match()
    batch.matrix(k)
    mov, msc, tki, tks = batch.download_matrix(k)
    rows = np.arange(fb.n)
    # top-1 of the matrix kernel is the argmax of the match kernel
    assert np.array_equal(tks[:, 0], score)
    assert np.array_equal(np.where(tks[:, 0] >= 98.0, tki[:, 0], -1), best)
    assert np.array_equal(mov[rows, tki[:, 0]], ov)
    # sorted best-first and consistent with the full matrix
    assert (tks[:, 0] >= tks[:, 1]).all() and (tks[:, 1] >= tks[:, 2]).all()
    for j in range(k):
        assert np.array_equal(msc[rows, tki[:, j]], tks[:, j])
    # CC filter: flagged files never rank a cc-* template
    cc_t = np.nonzero(corpus.is_cc)[0]
    flagged = fb.cc_false_positive.astype(bool)
    assert not np.isin(tki[flagged], cc_t).any()


@pytest.mark.parametrize('kernel', ['post', 'post-d0', 'post-d4', 'post-d16', 'lds', 'dense'])
def test_large_corpus_600_templates(kernel, monkeypatch):
    from licensee_amd._native import Scorer
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.synth import SyntheticCorpus
    from licensee_amd.synth_templates import synthetic_templates
    from oracle.native import OracleScorer
    tpl = synthetic_templates(License.all(hidden=True, pseudo=False), 600, seed=5)
    corpus = TemplateCorpus(tpl)
    fb = SyntheticCorpus(corpus).generate(0, 3000, seed=11, nthreads=8)
    if kernel == 'dense':
        monkeypatch.setenv('DICE_FORCE_DENSE', '1')
    else:
        monkeypatch.delenv('DICE_FORCE_DENSE', raising=False)
    monkeypatch.delenv('DICE_POST_DENSE', raising=False)
    # postings kernel: cost-model dense prefix, or forced to 0 / 4 / 16 u64 words
    monkeypatch.setenv('DICE_LARGE_KERNEL', 'post' if kernel.startswith('post') else 'lds')
    if kernel.startswith('post-d'):
        monkeypatch.setenv('DICE_POST_DENSE', kernel[6:])
    sc = Scorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack, corpus.length,
                corpus.is_cc, corpus.n_vocab, device=0)
    assert sc.info()[2] == (0 if kernel == 'dense' else 3 if kernel.startswith('post') else 2)
    orc = OracleScorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack,
                       corpus.length, corpus.is_cc, corpus.n_vocab)
    best, ov, score = sc.match(fb, 98.0)
    eb, eo, es = orc.match(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, 98.0, nthreads=16)
    assert np.array_equal(best, eb) and np.array_equal(ov, eo) and np.array_equal(score, es)
    mov, msc, tki, tks = sc.matrix(fb, 5)
    emov, emsc = orc.matrix(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, nthreads=16)
    assert np.array_equal(mov, emov) and np.array_equal(msc, emsc)
    assert np.array_equal(tks[:, 0], score)
    assert np.array_equal(np.where(tks[:, 0] >= 98.0, tki[:, 0], -1), best)
    rows = np.arange(fb.n)
    for j in range(5):
        assert np.array_equal(msc[rows, tki[:, j]], tks[:, j])
    assert (tks[:, :-1] >= tks[:, 1:]).all()
    sc.close()


def test_batch_detector_equals_per_file_chain():
    """batch.BatchDetector (native host Copyright/Exact + GPU Dice) == LicenseFile#license,
    #matcher and #confidence per file (license_file.rb:92-98, project_file.rb:69-80)."""
    from licensee_amd.batch import BatchDetector
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.synth import SyntheticCorpus
    texts = [c['normalized'] for t in golden('vendored.json')['templates'] for c in t['cases'].values()]
    texts += [l.content_normalized() for l in License.all(hidden=True, pseudo=False)]
    texts += ['Copyright (c) 2020 Foo Bar', 'Attribution-NonCommercial 4.0\n' +
              License.find('cc-by-4.0').content_normalized(), 'café licence', '', 'not a license']
    sc = SyntheticCorpus(TemplateCorpus(License.all(hidden=True, pseudo=False)))
    texts += [sc.text(i, seed=7)[0] for i in range(200)]
    bd = BatchDetector(nthreads=4)
    det = bd.detect(texts, ['LICENSE'] * len(texts))
    # the two-stage pipeline (host prep of batch k + 1 beside batch k on the device): the same
    # Detections, batch by batch, including ragged and empty batches
    cuts = [0, 1, 64, 64, 130, len(texts)]
    parts = [(texts[a:b], ['LICENSE'] * (b - a)) for a, b in zip(cuts, cuts[1:])]
    streamed = [d for chunk in bd.detect_stream(parts) for d in chunk]
    assert len(streamed) == len(det)
    assert all((x.license.key, x.matcher, x.confidence) == (y.license.key, y.matcher, y.confidence)
               for x, y in zip(streamed, det))
    kinds = set()
    for i, t in enumerate(texts):
        lf = LicenseFile(t, 'LICENSE')
        m = lf.matcher()
        assert det[i].license.key == lf.license().key, i
        assert det[i].matcher == (m.name if m is not None else None), i
        assert det[i].confidence == lf.confidence() and type(det[i].confidence) is type(lf.confidence()), i
        kinds.add(det[i].matcher)
    assert kinds == {'copyright', 'exact', 'dice', None}


def test_closest_licenses_unfiltered_topk():
    """detect.rb:93-98 ranks every template with no CC filter; the batched top-3 equals the
    oracle's stable-sort-reverse ranking over all 47 templates (oracle/dice_oracle.py)."""
    from licensee_amd.dice import default_engine
    from oracle import dice_oracle as O
    from tests.helpers import make_files, oracle_templates
    eng = default_engine()
    templates = eng.templates
    otpl = oracle_templates(templates)
    files = make_files(templates, 150, 33, cc_rate=0.3)
    files += [GoldenLicenseFile(golden('dice_spec.json')['cases'][c]['file']) for c in ('cc_nd', 'gpl', 'cc_by')]
    got = eng.closest_files(files, 3)
    for i, f in enumerate(files):
        of = f.oracle if hasattr(f, 'oracle') else O.OracleFile(f.content_normalized())
        ranked = O.matches_by_similarity(otpl, of, cc_fp=False)[:3]
        assert [(l.key, s) for l, s in got[i]] == [(templates[t].key, s) for t, s in ranked], i
        row = eng.licenses_by_similarity(f)[:3]
        assert [(l.key, s) for l, s in row] == [(l.key, s) for l, s in got[i]], i
    # the cc_nd golden file is CC-flagged: Dice drops cc-* templates, the CLI ranking keeps them
    assert any(l.key.startswith('cc-') for l, _ in got[-3])
