"""C-ABI contract on the GPU: one ctx per host thread (no internal locking, include/licensee_dice.h
conventions), device-resident batches reused across uploads, empty / capacity-edge batches,
argument errors as status codes, and the host-buffer calls equal to the batch calls."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def corpus():
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.license import License
    return TemplateCorpus(License.all(hidden=True, pseudo=False))


def _scorer(c):
    from licensee_amd._native import Scorer
    return Scorer(c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc, c.n_vocab, device=0)


def test_one_ctx_per_thread_concurrently(corpus):
    from licensee_amd.synth import SyntheticCorpus
    from oracle.native import OracleScorer
    synth = SyntheticCorpus(corpus)
    batches = [synth.generate(i * 20000, 20000, seed=31, nthreads=4) for i in range(4)]
    out = [None] * 4
    errors = []

    def work(i):
        try:
            sc = _scorer(corpus)
            res = []
            for _ in range(3):   # repeated calls on the same ctx
                res.append(sc.match(batches[i], 98.0))
            sc.close()
            out[i] = res
        except Exception as e:   # surfaced below
            errors.append(e)
    th = [threading.Thread(target=work, args=(i,)) for i in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    orc = OracleScorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack, corpus.length,
                       corpus.is_cc, corpus.n_vocab)
    for i, fb in enumerate(batches):
        eb, eo, es = orc.match(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, 98.0, nthreads=8)
        for best, ov, score in out[i]:
            assert np.array_equal(best, eb) and np.array_equal(ov, eo) and np.array_equal(score, es)


def test_device_batch_reuse_and_edges(corpus):
    from licensee_amd._native import DiceError, FileBatch
    from licensee_amd.synth import SyntheticCorpus
    sc = _scorer(corpus)
    synth = SyntheticCorpus(corpus)
    big = synth.generate(0, 5000, seed=9, nthreads=4)
    ref = sc.match(big, 98.0)
    b = sc.batch(5000)
    for n in (5000, 1, 63, 64, 65, 4999, 0, 5000):   # shrink/grow within capacity, ragged tiles, empty
        fb = FileBatch(big.bits[:n], big.wordset_size[:n], big.length[:n], big.cc_false_positive[:n])
        b.upload(fb)
        b.match(98.0)
        best, ov, score = b.download_match()
        assert np.array_equal(best, ref[0][:n]) and np.array_equal(ov, ref[1][:n]) and np.array_equal(score, ref[2][:n])
        b.matrix(3)
        mov, msc, tki, tks = b.download_matrix(3)
        hmov, hmsc, htki, htks = sc.matrix(fb, 3)
        assert np.array_equal(mov, hmov) and np.array_equal(msc, hmsc)
        assert np.array_equal(tki, htki) and np.array_equal(tks, htks)
    over = FileBatch(np.zeros((5001, corpus.w64), np.uint64), np.zeros(5001, np.uint32), np.zeros(5001, np.int32),
                     np.zeros(5001, np.uint8))
    with pytest.raises(DiceError, match='dice error -1'):
        b.upload(over)                                   # beyond capacity: DICE_E_ARG, batch unchanged
    with pytest.raises(DiceError, match='dice error -1'):
        b.matrix(17)                                     # k > DICE_TOPK_MAX
    b.close()
    sc.close()
