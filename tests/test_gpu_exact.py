"""Matchers::Exact on the device (dice_exact_setup / dice_batch_exact).

Reference: lib/licensee/matchers/exact.rb:6-12 -- the first template of License.all (key
order, no CC filter) whose wordset equals the file's; a template's wordset is Lf plus its field
words (content_helper.rb:108-110,323-335). The device decides |W_F| == |W_t| and W_t ⊆ W_F from
the resident bitset row, |W_F| and the file's mask of non-vocabulary field words. Checked here:
  - the product BatchDetector with Exact on the device == the host-Exact split == the per-file
    Python chain (Exact#match over Python sets) on template renderings, near misses and
    synthetic files;
  - adversarial near misses: a field word replaced by a non-vocabulary word (same size, Lf still
    held: only the field mask rejects it), a vocabulary word replaced (same size, Lf not held),
    a word added or dropped, duplicated templates (the first in key order wins);
  - a T = 600 corpus (postings / pruned kernels' row-major batch) against a numpy restatement.
"""
import numpy as np
import pytest

from licensee_amd.license import License

pytestmark = pytest.mark.gpu


def _python_exact(texts):
    from licensee_amd.matchers import Exact
    from licensee_amd.project_files import LicenseFile
    keys = [l.key for l in License.all(hidden=True, pseudo=False)]
    out = []
    for t in texts:
        e = Exact(LicenseFile(t, 'LICENSE')).match()
        out.append(keys.index(e.key) if e is not None else -1)
    return np.array(out, np.int32)


def _near_misses():
    texts = []
    for l in License.all(hidden=True, pseudo=False):
        body = l.content_normalized()
        texts.append(body)
        if '[fullname]' in body:
            texts.append(body.replace('[fullname]', 'zzqxv'))       # same |W|, field word missing
            texts.append(body.replace('[fullname]', ''))            # one word fewer
        words = body.split(' ')
        texts.append(' '.join(words + ['zzqxv']))                   # one word more
        for i, w in enumerate(words):
            if w.isalpha() and words.count(w) == 1 and len(w) > 3:
                texts.append(' '.join(words[:i] + ['zzqxv'] + words[i + 1:]))   # same |W|, a word swapped
                break
    return texts


def test_device_exact_equals_python_chain():
    from licensee_amd.batch import BatchDetector
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.synth import SyntheticCorpus
    texts = _near_misses()
    sc = SyntheticCorpus(TemplateCorpus(License.all(hidden=True, pseudo=False)))
    texts += [sc.text(i, seed=11)[0] for i in range(300)]
    texts += ['', 'fullname', 'year project fullname', 'ΣΟΦΙΑ license']
    exp = _python_exact(texts)
    assert (exp >= 0).sum() >= 40
    dev = BatchDetector(nthreads=4, exact_on='device')
    host = BatchDetector(nthreads=4, exact_on='host')
    assert dev.exact_on == 'device'
    fb, _, fm, _ = dev.host.prep_files(texts, None, nthreads=4, field_masks=True)
    got = dev.engine.scorer.exact(fb, fm)
    assert np.array_equal(got, exp)
    d1 = dev.detect(texts)
    d2 = host.detect(texts)
    for i in range(len(texts)):
        assert (d1[i].license.key, d1[i].matcher, d1[i].confidence) == \
               (d2[i].license.key, d2[i].matcher, d2[i].confidence), i
    # without field masks a template with a non-vocabulary field word cannot match exactly
    got0 = dev.engine.scorer.exact(fb, None)
    need = dev.host.field_need
    for i in range(len(texts)):
        if exp[i] >= 0 and need[exp[i]] == 0:
            assert got0[i] == exp[i], i
        elif exp[i] >= 0:
            assert got0[i] != exp[i], i


def _numpy_exact(bits, wf, fm, lf_bits, ws, fbits, need):
    T = lf_bits.shape[0]
    R = lf_bits | fbits
    out = np.full(bits.shape[0], -1, np.int32)
    for i in range(bits.shape[0]):
        for t in range(T):
            if ws[t] == wf[i] and (int(need[t]) & ~int(fm[i])) == 0 and np.array_equal(bits[i] & R[t], R[t]):
                out[i] = t
                break
    return out


def test_device_exact_large_corpus_and_duplicates():
    """T = 600 synthetic corpus (row-major batches) plus duplicated templates: every file that
    is a template's own wordset must return the first template in key order with that wordset."""
    from licensee_amd._native import FileBatch, Scorer
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.synth import SyntheticCorpus
    from licensee_amd.synth_templates import synthetic_templates
    base = License.all(hidden=True, pseudo=False)
    temps = synthetic_templates(base, 600, seed=5)
    temps = temps[:590] + temps[100:110]          # 10 duplicates later in key order
    c = TemplateCorpus(temps)
    T = len(temps)
    rng = np.random.default_rng(3)
    ws = c.lf_size.astype(np.uint32) + rng.integers(0, 3, T).astype(np.uint32)
    need = rng.integers(0, 4, T).astype(np.uint64) * (ws > c.lf_size)
    ws[590:], need[590:] = ws[100:110], need[100:110]   # the duplicates' wordsets are equal too
    fbits = np.zeros_like(c.lf_bits)
    fb = SyntheticCorpus(c).generate(0, 3000, seed=9, nthreads=8)
    bits, wf = fb.bits.copy(), fb.wordset_size.copy()
    fm = rng.integers(0, 4, fb.n).astype(np.uint64)
    # plant exact candidates: template rows with the template's size (and near misses)
    for i in range(0, fb.n, 5):
        t = int(rng.integers(0, T))
        bits[i] = c.lf_bits[t]
        wf[i] = ws[t] + (1 if i % 15 == 0 else 0)
        if i % 25 == 0:
            w = np.flatnonzero(bits[i])[0]
            bits[i, w] &= bits[i, w] - np.uint64(1)          # drop one Lf word
    files = FileBatch(bits, wf, fb.length, fb.cc_false_positive)
    sc = Scorer(c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc, c.n_vocab, device=0)
    sc.exact_setup(ws, fbits, need)
    got = sc.exact(files, fm)
    exp = _numpy_exact(bits, wf, fm, c.lf_bits, ws, fbits, need)
    assert (exp >= 0).sum() > 100
    assert np.array_equal(got, exp)
    # duplicates: the earlier key wins
    for t in range(100, 110):
        assert not (got == 590 + t - 100).any()
    # batch API on a stream, then Dice on the same resident batch
    b = sc.batch(fb.n)
    b.upload(files)
    b.exact(fm)
    b.match(98.0)
    assert np.array_equal(b.download_exact(), exp)
    b.close()
    sc.close()
