"""Pruned vs postings match kernel on config-3 templates with long/mixed files (SyntheticCorpus
profile 1: concatenations of 2-6 templates plus notices). Prints ms per launch for each kernel and
checks both give identical results. Run on the GPU box: python tools/exp/prune_long_files.py [n]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    import bench
    from licensee_amd._native import Scorer
    from licensee_amd.synth import SyntheticCorpus
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 250_000
    c = bench.build_workload(3)
    for profile in (0, 1):
        fb = SyntheticCorpus(c, profile=profile).generate(0, n, seed=20250202, nthreads=16)
        res = {}
        for prune in ('1', '0'):
            os.environ['DICE_POST_PRUNE'] = prune
            sc = Scorer(c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc,
                        n_vocab=c.n_vocab, device=0)
            b = sc.batch(n)
            b.upload(fb)
            b.match(98.0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                b.match(98.0)
            out = b.download_match()
            dt = (time.perf_counter() - t0) / 5 * 1e3
            res[prune] = out
            print(f'profile {profile} kernel {"pruned" if prune == "1" else "postings"}: {dt:.3f} ms / {n} files '
                  f'({n / dt * 1e3:.3e} files/s), matches {int((out[0] >= 0).sum())}', flush=True)
            b.close()
            sc.close()
        same = all(np.array_equal(x, y) for x, y in zip(res['1'], res['0']))
        print(f'profile {profile}: identical results {same}', flush=True)


if __name__ == '__main__':
    main()
