"""Multi-device Dice through the C-ABI (dice_match_sharded[_confidence] / dice_similarity_matrix_sharded)
and the one-process-per-GPU path under torch.distributed.run.

On the one-GPU box the shards' contexts share device 0 (each still has its own host thread,
stream and resident templates); results must be bit-identical to the single-context calls,
for both gathers (host slices; device buffer on ctxs[0]'s device + one D2H), for 1-3 shards,
and with more shards than files. The torchrun test runs the HIP scorer at world size 1 with
the RCCL all-gather of device-packed results and checks it against the C oracle.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from licensee_amd.license import License

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _scorers(corpus, n):
    from licensee_amd._native import Scorer
    return [Scorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack, corpus.length,
                   corpus.is_cc, corpus.n_vocab, device=0) for _ in range(n)]


def _sub(fb, n):
    from licensee_amd._native import FileBatch
    return FileBatch(fb.bits[:n], fb.wordset_size[:n], fb.length[:n], fb.cc_false_positive[:n])


@pytest.fixture(scope='module')
def vendored():
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.synth import SyntheticCorpus
    corpus = TemplateCorpus(License.all(hidden=True, pseudo=False))
    fb = SyntheticCorpus(corpus).generate(0, 100_003, seed=31, nthreads=16)
    scs = _scorers(corpus, 3)
    yield corpus, fb, scs
    for s in scs:
        s.close()


@pytest.mark.parametrize('gather', [0, 1])
def test_match_sharded_equals_single(vendored, gather):
    from licensee_amd._native import match_sharded
    corpus, fb, scs = vendored
    ref = scs[0].match(fb, 98.0)
    for n_ctx in (1, 2, 3):
        got = match_sharded(scs[:n_ctx], fb, 98.0, gather)
        for a, b in zip(got, ref):
            assert np.array_equal(a, b), (n_ctx, gather)
    tiny = _sub(fb, 2)                       # more shards than files: empty shards
    got = match_sharded(scs, tiny, 98.0, gather)
    for a, b in zip(got, scs[1].match(tiny, 98.0)):
        assert np.array_equal(a, b)


@pytest.mark.parametrize('gather', [0, 1])
def test_stale_hip_error_on_caller_thread_is_not_a_shard_failure(vendored, gather):
    """ADVICE r3 (dice_shard.cpp enable_peer): a non-success HIP return leaves the calling thread's
    last error set; shard 0 runs on that thread and its launch checks read hipGetLastError. A stale
    error (as hipDeviceEnablePeerAccess -> AlreadyEnabled leaves) must not fail the call."""
    import ctypes

    from licensee_amd._native import hip_runtime_path, match_sharded
    corpus, fb, scs = vendored
    hip = ctypes.CDLL(hip_runtime_path() or 'libamdhip64.so.7')
    part = _sub(fb, 4097)
    ref = scs[0].match(part, 98.0)
    assert hip.hipSetDevice(ctypes.c_int(1 << 20)) != 0      # invalid ordinal: sets the sticky error
    got = match_sharded(scs[:2], part, 98.0, gather)
    for a, b in zip(got, ref):
        assert np.array_equal(a, b)
    assert hip.hipGetLastError() == 0


@pytest.mark.parametrize('gather', [0, 1])
def test_matrix_sharded_equals_single(vendored, gather):
    from licensee_amd._native import matrix_sharded
    corpus, fb, scs = vendored
    part = _sub(fb, 20_011)
    for k in (0, 3, 16):
        ref = scs[0].matrix(part, k)
        got = matrix_sharded(scs, part, k, gather)
        for a, b in zip(got, ref):
            assert np.array_equal(a, b), (k, gather)


def test_sharded_large_corpus_lds():
    from licensee_amd._native import match_sharded, matrix_sharded
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.synth import SyntheticCorpus
    from licensee_amd.synth_templates import synthetic_templates
    corpus = TemplateCorpus(synthetic_templates(License.all(hidden=True, pseudo=False), 600, seed=5))
    fb = SyntheticCorpus(corpus).generate(0, 30_001, seed=13, nthreads=16)
    scs = _scorers(corpus, 2)
    assert scs[0].info()[2] in (2, 3)
    ref = scs[0].match(fb, 98.0)
    conf = scs[0].match(fb, 98.0, confidence=True)
    for gather in (0, 1):
        for a, b in zip(match_sharded(scs, fb, 98.0, gather), ref):
            assert np.array_equal(a, b)
        # dice_match_sharded_confidence: the pruned kernel's confidence outputs, sharded
        for a, b in zip(match_sharded(scs, fb, 98.0, gather, confidence=True), conf):
            assert np.array_equal(a, b)
    assert np.array_equal(conf[0], ref[0]) and np.all(conf[2][ref[0] < 0] == 0.0)
    part = _sub(fb, 3001)
    for a, b in zip(matrix_sharded(scs, part, 4, 1), scs[1].matrix(part, 4)):
        assert np.array_equal(a, b)
    for s in scs:
        s.close()


def test_sharded_rejects_mismatched_corpora(vendored):
    from licensee_amd._native import DiceError, match_sharded
    from licensee_amd.corpus import TemplateCorpus
    corpus, fb, scs = vendored
    small = TemplateCorpus(License.all(hidden=True, pseudo=False)[:5])
    other = _scorers(small, 1)[0]
    with pytest.raises(DiceError, match='different corpora'):
        match_sharded([scs[0], other], _sub(fb, 10), 98.0)
    other.close()


def test_sharded_rejects_duplicate_ctx(vendored):
    """One ctx twice would make two shard threads share its scratch batch and stream."""
    from licensee_amd._native import DiceError, match_sharded, matrix_sharded
    corpus, fb, scs = vendored
    with pytest.raises(DiceError, match='twice'):
        match_sharded([scs[0], scs[0]], _sub(fb, 100), 98.0)
    with pytest.raises(DiceError, match='twice'):
        matrix_sharded([scs[1], scs[2], scs[1]], _sub(fb, 100), 3)


def test_device_gather_reports_peer_path(vendored):
    """Every context on device 0 (the one-GPU box): a device gather exercises no peer path and
    reports -1, as a host gather does; the results are those of one dice_match either way."""
    from licensee_amd._native import last_gather_peer, match_sharded
    corpus, fb, scs = vendored
    assert {sc.device for sc in scs} == {0}
    dev = match_sharded(scs, _sub(fb, 1000), 98.0, 1)
    assert last_gather_peer() == -1
    host = match_sharded(scs, _sub(fb, 1000), 98.0, 0)
    assert last_gather_peer() == -1
    for a, b in zip(dev, host):
        assert np.array_equal(a, b)


def test_sharded_pinned_staging_large_pageable_input():
    """Shards of more than 64 MB of pageable rows go through the ctx's two pinned staging
    buffers in 32 MB chunks (several chunks per shard, odd remainder): results equal one
    dice_match call on the same files, and page-locked inputs take the direct path."""
    import torch
    from licensee_amd._native import FileBatch, match_sharded
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.synth import SyntheticCorpus
    corpus = TemplateCorpus(License.all(hidden=True, pseudo=False))
    n = 400_037                                 # 448 B per file: 2 shards of ~90 MB
    fb = SyntheticCorpus(corpus).generate(0, n, seed=17, nthreads=16)
    scs = _scorers(corpus, 2)
    ref = scs[0].match(fb, 98.0)
    for gather in (0, 1):
        for a, b in zip(match_sharded(scs, fb, 98.0, gather), ref):
            assert np.array_equal(a, b)
    pin = lambda a: torch.from_numpy(a).pin_memory().numpy()
    pfb = FileBatch(pin(fb.bits), fb.wordset_size, fb.length, fb.cc_false_positive)
    for a, b in zip(match_sharded(scs, pfb, 98.0, 0), ref):
        assert np.array_equal(a, b)
    for s in scs:
        s.close()


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_torchrun_world1_hip_scorer_rccl_gather(tmp_path):
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.shard import unpack_results
    from licensee_amd.synth import SyntheticCorpus
    from oracle.native import OracleScorer
    out = str(tmp_path / 'gathered.npy')
    n_per = 50_000
    env = dict(os.environ, MASTER_ADDR='127.0.0.1')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=1',
           '--master-addr=127.0.0.1', f'--master-port={_free_port()}',
           os.path.join(ROOT, 'tests', 'dist_gpu_worker.py'), out, str(n_per)]
    subprocess.run(cmd, check=True, env=env, timeout=240, cwd=ROOT)
    b, o, s = unpack_results(np.load(out))
    corpus = TemplateCorpus(License.all(hidden=True, pseudo=False))
    fb = SyntheticCorpus(corpus).generate(0, n_per, seed=7, nthreads=16)
    orc = OracleScorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack,
                       corpus.length, corpus.is_cc, corpus.n_vocab)
    eb, eo, es = orc.match(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, 98.0, nthreads=16, mode=0)
    assert np.array_equal(b, eb) and np.array_equal(o, eo) and np.array_equal(s, es)
