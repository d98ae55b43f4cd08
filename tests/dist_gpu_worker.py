"""torch.distributed.run worker for tests/test_gpu_sharded.py (not a test module): each rank
scores its shard with the HIP scorer (C-ABI batch on the rank's GPU), packs the resident
results on the device (licensee_amd/shard.py) and all-gathers them with RCCL; rank 0 saves
the gathered block.  argv: out_path files_per_rank"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    out_path, n_per = sys.argv[1], int(sys.argv[2])
    rank, world, local = int(os.environ['RANK']), int(os.environ['WORLD_SIZE']), int(os.environ['LOCAL_RANK'])
    torch.cuda.set_device(local)
    dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    from licensee_amd._native import Scorer
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.license import License
    from licensee_amd.shard import all_gather_packed, device_results_packed, shard_range
    from licensee_amd.synth import SyntheticCorpus
    corpus = TemplateCorpus(License.all(hidden=True, pseudo=False))
    first, count = shard_range(rank, world, n_per)
    fb = SyntheticCorpus(corpus).generate(first, count, seed=7, nthreads=8)
    sc = Scorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack, corpus.length,
                corpus.is_cc, corpus.n_vocab, device=local)
    batch = sc.batch(count)
    stream = torch.cuda.current_stream().cuda_stream
    batch.upload(fb, stream)
    batch.match(98.0, stream)
    out = all_gather_packed(device_results_packed(batch))
    torch.cuda.synchronize()
    if rank == 0:
        np.save(out_path, out.cpu().numpy())
    dist.barrier()
    batch.close()
    sc.close()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
