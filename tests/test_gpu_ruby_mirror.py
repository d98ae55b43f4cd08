"""The Ruby FFI binding's logic (restated in tests/ruby_mirror.py) against the
product path on the GPU:

  * Corpus#matches_by_similarity(file, Dice#potential_matches) == the product Dice's
    matches_by_similarity (dice.rb:34-41) -- golden spec files, fixtures, synthetic files --
    and == the oracle's stable-ascending-then-reversed ranking;
  * the same with byte-identical templates under later keys (exact ties: the later key first);
  * Corpus#match == Dice#match / #confidence per file, with the CC filter (dice.rb:23-31);
  * Corpus#detect == LicenseFile#license / #confidence / matcher per file (license_file.rb:92-98);
  * GpuDice.corpus is one process-wide object (license.rb:21's @all memo) until reset.

The mirror numbers the vocabulary in first-seen order, the product in packed order: equal
results also show that scores do not depend on word ids.
"""
import json
import os

import pytest

from licensee_amd.license import License
from licensee_amd.project_files import LicenseFile
from tests import ruby_mirror as R

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')


def golden(name):
    with open(os.path.join(GOLDEN, name), encoding='utf-8') as fh:
        return json.load(fh)


class GoldenLicenseFile(LicenseFile):
    def __init__(self, rec):
        super().__init__('', 'LICENSE')
        self._content_normalized = rec['normalized']
        self._fp = rec['cc_false_positive']

    def potential_false_positive(self):
        return self._fp


def _files():
    from tests.helpers import make_files
    cases = golden('dice_spec.json')['cases']
    files = [GoldenLicenseFile(c['file']) for c in cases.values()]
    files += [GoldenLicenseFile(r) for r in golden('fixture_files.json') if 'unsupported' not in r][:40]
    files += make_files(License.all(hidden=True, pseudo=False), 200, 77, cc_rate=0.2)
    return files


@pytest.fixture(scope='module')
def corpus():
    R.GpuDice.reset()
    c = R.GpuDice.corpus()
    yield c
    R.GpuDice.reset()


def test_corpus_is_process_wide(corpus):
    assert R.GpuDice.corpus() is corpus
    assert [l.key for l in corpus.licenses] == [l.key for l in License.all(hidden=True, pseudo=False)]


def test_matches_by_similarity_equals_product_and_oracle(corpus):
    from licensee_amd.matchers import Dice
    from oracle import dice_oracle as O
    from tests.helpers import oracle_templates
    otpl = oracle_templates(corpus.licenses)
    for i, f in enumerate(_files()):
        d = Dice(f)
        got = corpus.matches_by_similarity(f, d.potential_matches())
        want = d.matches_by_similarity()
        assert [(l.key, s) for l, s in got] == [(l.key, s) for l, s in want], i
        of = f.oracle if hasattr(f, 'oracle') else O.OracleFile(f.content_normalized())
        ranked = O.matches_by_similarity(otpl, of, cc_fp=bool(f.potential_false_positive()))
        assert [(l.key, s) for l, s in got] == [(otpl[t].key, s) for t, s in ranked], i


def test_exact_ties_rank_the_later_key_first():
    from tests.helpers import NormFile
    base = [License.find(k) for k in ('apache-2.0', 'isc', 'mit')]
    clones = [License('zz-' + l.key, {'title': l.title}, content_normalized=l.content_normalized(),
                      alt_segments=l.spdx_alt_segments()) for l in base]
    templates = sorted(base + clones, key=lambda l: l.key)
    c = R.Corpus(templates)
    try:
        for l in base:
            f = NormFile(l.content_normalized())
            ranked = c.matches_by_similarity(f, templates)
            assert ranked[0][0].key == 'zz-' + l.key and ranked[1][0].key == l.key
            assert ranked[0][1] == ranked[1][1] == 100.0
    finally:
        c.close()


def test_batched_match_equals_dice_per_file(corpus):
    from licensee_amd.matchers import Dice
    files = _files()
    for thr in (98, 90):
        got = corpus.match(files, thr)
        from licensee_amd import config
        old = config.confidence_threshold()
        config.set_confidence_threshold(thr)
        try:
            for i, f in enumerate(files):
                d = Dice(f)
                m = d.match()
                assert (got[i][0].key if got[i][0] else None) == (m.key if m else None), (i, thr)
                assert got[i][1] == d.confidence(), (i, thr)
        finally:
            config.set_confidence_threshold(old)


def test_detect_equals_license_file_chain(corpus):
    texts = [c['normalized'] for t in golden('vendored.json')['templates'][:10] for c in t['cases'].values()]
    texts += ['Copyright (c) 2020 Foo Bar', 'not a license', '',
              'Attribution-NonCommercial 4.0\n' + License.find('cc-by-4.0').content_normalized()]
    # Exact on the device (Corpus#exact): templates whose wordsets hold field words outside the
    # vocabulary (ncsa, postgresql: 'fullname'), and the same texts with that word swapped out
    for k in ('ncsa', 'postgresql', 'bsd-4-clause', 'vim'):
        body = License.find(k).content_normalized()
        texts += [body, body.replace('[fullname]', 'zzqxv').replace('[project]', 'zzqxw')]
    files = [LicenseFile(t, 'LICENSE') for t in texts]
    got = corpus.detect(files)
    kinds = set()
    for i, t in enumerate(texts):
        lf = LicenseFile(t, 'LICENSE')
        m = lf.matcher()
        assert got[i][0].key == lf.license().key, i
        assert got[i][1] == lf.confidence(), i
        assert got[i][2] == (m.name if m is not None else None), i
        kinds.add(got[i][2])
    assert kinds == {'copyright', 'exact', 'dice', None}
