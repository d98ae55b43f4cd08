"""Synthetic corpus generator (bench input): every generated file equals the interned text
path of its replayed token sequence; shards are pure functions of the global index."""
import numpy as np
import pytest

from licensee_amd.corpus import TemplateCorpus
from licensee_amd.license import License
from licensee_amd.synth import SyntheticCorpus
from tests.helpers import NormFile


@pytest.fixture(scope='module')
def corpus():
    return TemplateCorpus(License.all(hidden=True, pseudo=False))


@pytest.mark.parametrize('profile', [0, 1])
def test_replay_matches_text_path(corpus, profile):
    s = SyntheticCorpus(corpus, profile=profile)
    fb, src = s.generate(0, 400, seed=5, nthreads=4, with_source=True)
    for i in range(0, 400, 3):
        text, cc, sr = s.text(i, seed=5)
        bits, wf = corpus.intern(NormFile(text).wordset())
        assert np.array_equal(bits, fb.bits[i]) and wf == fb.wordset_size[i]
        assert len(text) == fb.length[i] and cc == bool(fb.cc_false_positive[i]) and sr == src[i]


def test_shards_are_index_pure(corpus):
    s = SyntheticCorpus(corpus)
    whole = s.generate(0, 1000, seed=3, nthreads=3)
    a = s.generate(0, 400, seed=3, nthreads=2)
    b = s.generate(400, 600, seed=3, nthreads=5)
    assert np.array_equal(np.vstack([a.bits, b.bits]), whole.bits)
    assert np.array_equal(np.concatenate([a.length, b.length]), whole.length)


def test_mix_of_perturbations(corpus):
    s = SyntheticCorpus(corpus)
    fb, src = s.generate(0, 20000, seed=20250202, nthreads=4, with_source=True)
    assert set(np.unique(src)) == set(range(len(corpus.templates)))   # every template used
    assert 0.002 < fb.cc_false_positive.mean() < 0.03                 # ~1% CC flag
    assert (fb.wordset_size > 0).all()
