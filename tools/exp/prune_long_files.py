"""Pruned vs postings match kernel on config-3 templates with long/mixed files (SyntheticCorpus
profile 1: concatenations of 2-6 templates plus notices), and the pruned kernel in confidence mode
(dice_batch_match_confidence). Prints ms per launch for each and checks the results agree (the
confidence mode's with the unmatched files' overlap/score set to 0). Run on the GPU box: python tools/exp/prune_long_files.py [n]"""
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
        for prune in ('1', '0', 'conf'):
            conf = prune == 'conf'
            os.environ['DICE_POST_PRUNE'] = '1' if conf else prune
            sc = Scorer(c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc,
                        n_vocab=c.n_vocab, device=0)
            b = sc.batch(n)
            b.upload(fb)
            st = torch.cuda.Stream()   # the events must be on the launch stream
            sp = st.cuda_stream
            b.match(98.0, sp, confidence=conf)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(5):
                b.match(98.0, sp, confidence=conf)
            e1.record(st)
            torch.cuda.synchronize()
            out = b.download_match(sp)
            dt = e0.elapsed_time(e1) / 5
            res[prune] = out
            name = {'1': 'pruned', '0': 'postings', 'conf': 'pruned-confidence'}[prune]
            print(f'profile {profile} kernel {name}: {dt:.3f} ms / {n} files '
                  f'({n / dt * 1e3:.3e} files/s), matches {int((out[0] >= 0).sum())}', flush=True)
            b.close()
            sc.close()
        same = all(np.array_equal(x, y) for x, y in zip(res['1'], res['0']))
        best, ov, score = res['1']
        exp = (best, np.where(best >= 0, ov, 0), np.where(best >= 0, score, 0.0))
        same_conf = all(np.array_equal(x, y) for x, y in zip(res['conf'], exp))
        print(f'profile {profile}: identical results {same}, confidence mode {same_conf}', flush=True)
        if not (same and same_conf):
            sys.exit(1)


if __name__ == '__main__':
    main()
