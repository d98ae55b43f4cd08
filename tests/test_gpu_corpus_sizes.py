"""GPU parity across corpus shapes: template counts either side of the sparse-program limit
(64), of the dense kernel's 48-template tile, of the LDS kernel's one-pass capacity (640) and of
the postings kernel's 64-template lane rounds (65, 97, 130, 700),
tiny vocabularies (one 128-bit quad), every kernel where it applies. Bit-exact against the C oracle (oracle/dice_ref.c) for
match (keys, overlaps, scores with ==) and the full similarity matrix + top-k.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SIZES = [1, 2, 5, 33, 47, 48, 49, 63, 64, 65, 96, 97, 130, 700]


def corpus_of(n):
    from licensee_amd.license import License
    from licensee_amd.synth_templates import synthetic_templates
    real = License.all(hidden=True, pseudo=False)
    if n == 1:
        return [License.find('mit')]
    if n == 2:
        return [License.find('cc-by-4.0'), License.find('cc-by-sa-4.0')]
    if n <= len(real):
        return real[::-1][:n] if n % 2 else real[:n]
    return synthetic_templates(real, n, seed=n)


KIND = {'dense': 0, 'program': 1, 'lds': 2, 'post': 3}


# every kernel where it applies: the sparse program serves T <= 64, the postings kernel
# (default) and the LDS record kernel T > 64, the dense kernel (DICE_FORCE_DENSE) any T
CASES = [(n, k) for n in SIZES for k in ('program', 'lds', 'post', 'dense')
         if not (k == 'program' and n > 64) and not (k in ('lds', 'post') and n <= 64)]


def select_kernel(monkeypatch, kernel):
    monkeypatch.delenv('DICE_POST_DENSE', raising=False)
    if kernel == 'dense':
        monkeypatch.setenv('DICE_FORCE_DENSE', '1')
    else:
        monkeypatch.delenv('DICE_FORCE_DENSE', raising=False)
    monkeypatch.setenv('DICE_LARGE_KERNEL', 'lds' if kernel == 'lds' else 'post')


@pytest.mark.parametrize('n_templates,kernel', CASES)
def test_corpus_size(n_templates, kernel, monkeypatch):
    _check_corpus(n_templates, kernel, monkeypatch)


# the postings kernels' dense prefix in both launch shapes of the matrix-core kernel: 12 waves x 3
# 32-file M-tiles up to 640 templates (130, 600) and 11 waves x 2 M-tiles above (672, 700), plus
# narrower prefixes (DICE_POST_DENSE: 4 and 12 words)
PREFIX_VARIANTS = {'d20': {}, 'd4': {'DICE_POST_DENSE': '4'}, 'd12': {'DICE_POST_DENSE': '12'}}


@pytest.mark.parametrize('variant', sorted(PREFIX_VARIANTS))
@pytest.mark.parametrize('n_templates', [130, 600, 672, 700])
def test_postings_dense_prefix_variants(n_templates, variant, monkeypatch):
    for k, v in PREFIX_VARIANTS[variant].items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv('DICE_POST_PRUNE', '0')
    _check_corpus(n_templates, 'post', monkeypatch)


def _check_corpus(n_templates, kernel, monkeypatch):
    from licensee_amd._native import Scorer
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.synth import SyntheticCorpus
    from oracle.native import OracleScorer
    select_kernel(monkeypatch, kernel)
    c = TemplateCorpus(corpus_of(n_templates))
    fb = SyntheticCorpus(c).generate(0, 2000, seed=n_templates, nthreads=8)
    sc = Scorer(c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc, c.n_vocab, device=0)
    try:
        assert sc.info()[2] == KIND[kernel]
        orc = OracleScorer(c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc, c.n_vocab)
        for thr in (0.0, 98.0):
            best, ov, score = sc.match(fb, thr)
            eb, eo, es = orc.match(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, thr, nthreads=8)
            assert np.array_equal(best, eb) and np.array_equal(ov, eo) and np.array_equal(score, es), thr
        k = min(5, n_templates)
        mov, msc, tki, tks = sc.matrix(fb, k)
        emov, emsc = orc.matrix(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, nthreads=8)
        assert np.array_equal(mov, emov) and np.array_equal(msc, emsc)
        # top-k: descending scores, the later template first among exact ties (dice.rb:39);
        # CC templates are not candidates for flagged files (dice.rb:17-25), padding is -1
        filt = fb.cc_false_positive.astype(bool)[:, None] & c.is_cc.astype(bool)[None, :]
        key = np.where(filt, -np.inf, emsc)
        order = np.lexsort((-np.arange(n_templates)[None, :].repeat(fb.n, 0), -key), axis=1)[:, :k]
        valid = np.take_along_axis(~filt, order, 1)
        assert np.array_equal(tki, np.where(valid, order, -1))
        assert np.array_equal(tks[valid], np.take_along_axis(emsc, order, 1)[valid])
    finally:
        sc.close()


@pytest.mark.parametrize('kernel', ['lds', 'post'])
@pytest.mark.parametrize('n_files', [0, 1, 63, 150, 1000])
def test_lds_ragged_batches(n_files, kernel, monkeypatch):
    """LDS kernel (T = 130) on batches that end mid-tile and mid-group: a workgroup holds 2 tiles
    of 64 files, so 150 files leave a partial group and a 22-file tail; 0 files launch nothing.
    The postings kernel ('post', one 64-file tile per workgroup) on the same batches."""
    monkeypatch.setenv('DICE_LARGE_KERNEL', kernel)
    from licensee_amd._native import FileBatch, Scorer
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.synth import SyntheticCorpus
    from oracle.native import OracleScorer
    monkeypatch.delenv('DICE_FORCE_DENSE', raising=False)
    c = TemplateCorpus(corpus_of(130))
    fb = SyntheticCorpus(c).generate(0, max(n_files, 1), seed=7, nthreads=8)
    fb = FileBatch(fb.bits[:n_files], fb.wordset_size[:n_files], fb.length[:n_files], fb.cc_false_positive[:n_files])
    sc = Scorer(c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc, c.n_vocab, device=0)
    try:
        assert sc.info()[2] == KIND[kernel]
        orc = OracleScorer(c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc, c.n_vocab)
        best, ov, score = sc.match(fb, 98.0)
        assert best.shape == ov.shape == score.shape == (n_files,)
        if n_files == 0:
            return
        eb, eo, es = orc.match(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, 98.0, nthreads=8)
        assert np.array_equal(best, eb) and np.array_equal(ov, eo) and np.array_equal(score, es)
        mov, msc, tki, tks = sc.matrix(fb, 3)
        emov, emsc = orc.matrix(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, nthreads=8)
        assert np.array_equal(mov, emov) and np.array_equal(msc, emsc)
        assert np.array_equal(tks[:, 0], score)
    finally:
        sc.close()
