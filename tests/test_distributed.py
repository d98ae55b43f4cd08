"""World-size-2 gloo test of the sharded path (licensee_amd/shard.py): disjoint shards by
global file index, per-rank scoring, results packed bit-exactly and gathered in shard order --
all-gathered, gathered to rank 0, and written into rank 0's node-shared host buffer (the host
gather bench.py times against RCCL); every gathered result equals a single-process oracle run
over all files. Each rank scores
through the HIP scorer where a GPU exists (the -m gpu case: both ranks on device 0 of the test
box); the C oracle stands in for it only in the CPU case."""
import pytest
import os
import socket

import numpy as np
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n_per, out_path, use_gpu):
    import torch
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.license import License
    from licensee_amd.shard import (SharedResults, all_gather_packed, gather_packed_to0, pack_results, shard_range,
                                    shm_gather)
    from licensee_amd.synth import SyntheticCorpus
    from oracle.native import OracleScorer
    corpus = TemplateCorpus(License.all(hidden=True, pseudo=False))
    first, count = shard_range(rank, world, n_per)
    fb = SyntheticCorpus(corpus).generate(first, count, seed=7, nthreads=2)
    if use_gpu:
        from licensee_amd._native import Scorer
        sc = Scorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack, corpus.length,
                    corpus.is_cc, corpus.n_vocab, device=0)
        res = pack_results(*sc.match(fb, 98.0))
        sc.close()
    else:
        orc = OracleScorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack,
                           corpus.length, corpus.is_cc, corpus.n_vocab)
        res = pack_results(*orc.match(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, 98.0, nthreads=2))
    out = all_gather_packed(torch.from_numpy(res))
    to0 = gather_packed_to0(torch.from_numpy(res))
    assert (to0 is None) == (rank != 0)
    # bench.py's collective gather leg (the RCCL leg of gather_compare, here over gloo with host
    # tensors): its packing, shard order and timing reduction
    import bench
    group = bench.Group(rank, world, 'gloo')
    leg_dst = torch.empty((world * n_per, 4), dtype=torch.int32) if rank == 0 else None
    leg_s = bench.collective_gather_leg(torch.from_numpy(res), leg_dst, group, rank, 2, lambda: None)
    assert leg_s > 0
    assert bench.gather_winner(leg_s, leg_s) == 'host' and bench.gather_winner(2.0, 1.0) == 'rccl'
    shared = SharedResults(f'licensee_test_{port}', world, n_per, create=rank == 0) if rank == 0 else None
    dist.barrier()                       # the segment exists before the other ranks attach
    if shared is None:
        shared = SharedResults(f'licensee_test_{port}', world, n_per, create=False)

    def write_local(b, o, s):
        from licensee_amd.shard import unpack_results
        lb, lo, ls = unpack_results(res)
        b[:], o[:], s[:] = lb, lo, ls
    shm_gather(dist.barrier, shared, rank, write_local)
    if rank == 0:
        np.save(out_path, out.numpy())
        np.save(out_path + '.to0.npy', to0.numpy())
        np.save(out_path + '.leg.npy', leg_dst.numpy())
        np.save(out_path + '.shm.npy', pack_results(shared.best.copy(), shared.overlap.copy(), shared.score.copy()))
    dist.barrier()
    shared.close()
    dist.destroy_process_group()


@pytest.mark.parametrize('use_gpu', [False, pytest.param(True, marks=pytest.mark.gpu)])
def test_two_rank_shard_and_gather(tmp_path, use_gpu):
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.license import License
    from licensee_amd.shard import pack_results, unpack_results
    from licensee_amd.synth import SyntheticCorpus
    from oracle.native import OracleScorer
    n_per, world = 3000, 2
    out_path = str(tmp_path / 'gathered.npy')
    mp.start_processes(_worker, args=(world, _free_port(), n_per, out_path, use_gpu), nprocs=world, start_method='spawn')
    gathered = np.load(out_path)
    assert np.array_equal(np.load(out_path + '.to0.npy'), gathered)
    assert np.array_equal(np.load(out_path + '.leg.npy'), gathered)
    assert np.array_equal(np.load(out_path + '.shm.npy'), gathered)
    corpus = TemplateCorpus(License.all(hidden=True, pseudo=False))
    fb = SyntheticCorpus(corpus).generate(0, world * n_per, seed=7, nthreads=2)
    orc = OracleScorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack,
                       corpus.length, corpus.is_cc, corpus.n_vocab)
    single = orc.match(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, 98.0, nthreads=2)
    assert np.array_equal(gathered, pack_results(*single))
    b, o, s = unpack_results(gathered)
    assert np.array_equal(b, single[0]) and np.array_equal(o, single[1]) and np.array_equal(s, single[2])
