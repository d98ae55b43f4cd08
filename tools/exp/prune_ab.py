"""Interleaved A/B of T > 64 match-mode variants on the GPU box (HIP events on one stream).

    python tools/exp/prune_ab.py [--n N] [--reps R] [--profiles 0,1] VARIANT ...

VARIANT is name or name:ENV=VAL,ENV=VAL (environment read at dice_create), e.g.
    base  post:DICE_POST_PRUNE=0  route6:DICE_PRUNE_ROUTE=6
Workload: the bench's config-3 corpus (600 synthetic templates); profile 0 = config-3 files,
profile 1 = long/mixed files (concatenations of 2-6 templates plus notices). Every variant's
results are checked equal to the first variant's; prints ms per launch (median of the reps,
each rep 10 launches) and the files deferred to the postings kernels.
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def parse(v):
    name, _, envs = v.partition(':')
    env = dict(kv.split('=', 1) for kv in envs.split(',') if kv)
    return name, env


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=1_250_000)
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--launches', type=int, default=10)
    ap.add_argument('--profiles', default='0,1')
    ap.add_argument('--long-n', type=int, default=250_000)
    ap.add_argument('variants', nargs='+')
    a = ap.parse_args()
    import torch
    import bench
    from licensee_amd._native import Scorer
    from licensee_amd.synth import SyntheticCorpus
    c = bench.build_workload(3)
    variants = [parse(v) for v in a.variants]
    stream = torch.cuda.Stream()
    sp = stream.cuda_stream
    for profile in [int(p) for p in a.profiles.split(',')]:
        n = a.n if profile == 0 else a.long_n
        fb = SyntheticCorpus(c, profile=profile).generate(0, n, seed=20250202, nthreads=16)
        runs = []
        for name, env in variants:
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                sc = Scorer(c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc,
                            n_vocab=c.n_vocab, device=0)
            finally:
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
            b = sc.batch(n)
            b.upload(fb, sp)
            b.match(98.0, sp)
            torch.cuda.synchronize()
            runs.append((name, sc, b, []))
        ref = None
        for name, sc, b, _ in runs:
            out = b.download_match(sp)
            if ref is None:
                ref = out
            same = all(np.array_equal(x, y) for x, y in zip(out, ref))
            print(f'profile {profile} {name}: kernel {sc.match_kernel()} deferred {b.deferred(sp)} '
                  f'identical {same}', flush=True)
        for rep in range(a.reps):
            for name, sc, b, ts in runs:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(a.launches):
                    b.match(98.0, sp)
                e1.record(stream)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / a.launches)
        for name, sc, b, ts in runs:
            print(f'profile {profile} n {n} {name}: {np.median(ts):.4f} ms  reps {" ".join(f"{t:.4f}" for t in ts)}',
                  flush=True)
            b.close()
            sc.close()


if __name__ == '__main__':
    main()
