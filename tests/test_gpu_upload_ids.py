"""dice_batch_upload_ids: files handed over as word-id lists (CSR) score exactly as the same
files handed over as bitsets (dice_batch_upload), on every kernel, with the edge cases of the
id form -- empty files, unsorted and duplicate ids, ids outside the vocabulary (ignored), uint16
and uint32 ids, a batch reused with a longer id list (staging regrown) -- and the argument
checks (offsets that do not start at 0 or decrease are DICE_E_ARG)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from tests.test_gpu_corpus_sizes import KIND, corpus_of, select_kernel  # noqa: E402


def to_ids(bits, n_vocab, rng, id_dtype, noise=True):
    """Bitset rows -> (offsets, ids): shuffled, with duplicates and out-of-vocabulary ids mixed in."""
    n = bits.shape[0]
    dense = np.unpackbits(bits.view(np.uint8).reshape(n, -1), axis=1, bitorder='little')[:, :n_vocab]
    lists = []
    hi = np.iinfo(id_dtype).max
    for i in range(n):
        ids = np.flatnonzero(dense[i]).astype(np.int64)
        if noise and ids.size:
            ids = np.concatenate([ids, rng.choice(ids, size=min(3, ids.size)),
                                  rng.integers(n_vocab, min(hi, n_vocab + 5000) + 1, size=int(rng.integers(0, 4))),
                                  np.array([hi], np.int64)])
            rng.shuffle(ids)
        lists.append(ids)
    offsets = np.zeros(n + 1, np.int64)
    offsets[1:] = np.cumsum([len(x) for x in lists])
    flat = np.concatenate(lists) if lists else np.zeros(0, np.int64)
    return offsets, flat.astype(id_dtype)


CASES = [(47, 'program'), (47, 'dense'), (130, 'post'), (130, 'lds'), (700, 'post')]


@pytest.mark.parametrize('id_dtype', [np.uint16, np.uint32])
@pytest.mark.parametrize('n_templates,kernel', CASES)
def test_upload_ids_equals_bitset_upload(n_templates, kernel, id_dtype, monkeypatch):
    from licensee_amd._native import FileBatch, Scorer
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.synth import SyntheticCorpus
    select_kernel(monkeypatch, kernel)
    c = TemplateCorpus(corpus_of(n_templates))
    if id_dtype == np.uint16:
        assert c.n_vocab < 65535
    fb = SyntheticCorpus(c).generate(0, 1500, seed=n_templates + 3, nthreads=8)
    bits = fb.bits.copy()
    bits[::97] = 0                                                # empty files (no vocabulary word)
    fb = FileBatch(bits, fb.wordset_size, fb.length, fb.cc_false_positive)
    rng = np.random.default_rng(11)
    offsets, ids = to_ids(fb.bits, c.n_vocab, rng, id_dtype)
    sc = Scorer(c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc, c.n_vocab, device=0)
    try:
        assert sc.info()[2] == KIND[kernel]
        a, b = sc.batch(fb.n), sc.batch(fb.n)
        a.upload(fb)
        # first a short prefix (small staging), then the whole list (staging regrown)
        b.upload_ids(offsets[:11], ids, fb.wordset_size[:10], fb.length[:10], fb.cc_false_positive[:10])
        b.match(98.0)
        best10 = b.download_match()[0]
        b.upload_ids(offsets, ids, fb.wordset_size, fb.length, fb.cc_false_positive)
        for thr in (0.0, 98.0):
            a.match(thr)
            b.match(thr)
            ra, rb = a.download_match(), b.download_match()
            for x, y in zip(ra, rb):
                assert np.array_equal(x, y), thr
        assert np.array_equal(best10, sc.match(FileBatch(fb.bits[:10], fb.wordset_size[:10], fb.length[:10],
                                                         fb.cc_false_positive[:10]), 98.0)[0])
        k = min(4, n_templates)
        a.matrix(k)
        b.matrix(k)
        for x, y in zip(a.download_matrix(), b.download_matrix()):
            assert np.array_equal(x, y)
        a.close()
        b.close()
    finally:
        sc.close()


def test_upload_ids_edges_and_argument_checks(monkeypatch):
    from licensee_amd._native import DiceError, Scorer
    from licensee_amd.corpus import TemplateCorpus
    from oracle.native import OracleScorer
    select_kernel(monkeypatch, 'program')
    c = TemplateCorpus(corpus_of(47))
    sc = Scorer(c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc, c.n_vocab, device=0)
    try:
        b = sc.batch(8)
        z = np.zeros(0, np.uint32)
        b.upload_ids(np.zeros(1, np.int64), z, z, z.astype(np.int32), z.astype(np.uint8))   # n = 0
        assert b.download_match()[0].shape == (0,)
        # all files empty (no ids at all): no template overlaps
        n = 5
        wf = np.full(n, 40, np.uint32)
        ln = np.full(n, 300, np.int32)
        cc = np.zeros(n, np.uint8)
        b.upload_ids(np.zeros(n + 1, np.int64), z, wf, ln, cc)
        b.match(0.0)
        best, ov, score = b.download_match()
        orc = OracleScorer(c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc, c.n_vocab)
        eb, eo, es = orc.match(np.zeros((n, c.lf_bits.shape[1]), np.uint64), wf, ln, cc, 0.0, nthreads=1)
        assert np.array_equal(best, eb) and np.array_equal(ov, eo) and np.array_equal(score, es)
        # a file that is exactly template 0's word set, its ids only
        mit = np.flatnonzero(np.unpackbits(c.lf_bits[:1].view(np.uint8), bitorder='little')[:c.n_vocab])
        b.upload_ids(np.array([0, mit.size], np.int64), mit.astype(np.uint32), c.lf_size[:1] + c.fields_set_size[:1],
                     c.length[:1], np.zeros(1, np.uint8))
        b.match(0.0)
        assert b.download_match()[1][0] == c.lf_size[0]
        with pytest.raises(DiceError, match='offsets'):
            b.upload_ids(np.array([1, 2], np.int64), np.zeros(2, np.uint32), wf[:1], ln[:1], cc[:1])
        with pytest.raises(DiceError, match='non-decreasing'):
            b.upload_ids(np.array([0, 2, 1], np.int64), np.zeros(2, np.uint32), wf[:2], ln[:2], cc[:2])
        with pytest.raises(DiceError, match='capacity'):
            b.upload_ids(np.zeros(10, np.int64), z, np.zeros(9, np.uint32), np.zeros(9, np.int32),
                         np.zeros(9, np.uint8))
        b.close()
    finally:
        sc.close()
