"""Diagnostic: per-wave start/end clocks of the config-2 sparse program (DICE_PROG_DIAG=timing).

    DICE_PROG_DIAG=timing python tools/exp/wave_timing.py

Scores 1M synthetic files once (warm), then once more recording each wave's s_memtime at start
and end and its HW_ID / XCC_ID, and prints the launch span, the wave-duration distribution by
start time, per-CU busy fractions and the tail."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    assert os.environ.get('DICE_PROG_DIAG') == 'timing'
    from licensee_amd._native import Scorer
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.license import License
    from licensee_amd.synth import SyntheticCorpus
    corpus = TemplateCorpus(License.all(hidden=True, pseudo=False))
    fb = SyntheticCorpus(corpus).generate(0, 1_000_000, seed=20250202, nthreads=16)
    sc = Scorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack, corpus.length,
                corpus.is_cc, corpus.n_vocab, device=0)
    b = sc.batch(fb.n)
    b.upload(fb)
    for _ in range(3):
        b.match(98.0)
    b.match(98.0)
    best, ov, score = b.download_match()
    nt = (fb.n + 63) // 64
    t0 = score[0::64][:nt].astype(np.int64)
    t1 = score[1::64][:nt].astype(np.int64)
    hw = ov[0::64][:nt].astype(np.int64)
    xcc = ov[1::64][:nt].astype(np.int64) & 0xF
    # s_memtime counters are per XCD: normalize each XCD to its own first wave start
    for x in np.unique(xcc):
        m = xcc == x
        b0 = t0[m].min()
        t0[m] -= b0
        t1[m] -= b0
    dur = t1 - t0
    print(f'waves {nt}, wave duration ticks: mean {dur.mean():.0f} p10 {np.percentile(dur, 10):.0f} '
          f'p50 {np.median(dur):.0f} p90 {np.percentile(dur, 90):.0f} max {dur.max()}')
    for x in np.unique(xcc):
        m = xcc == x
        span = t1[m].max()
        cu = ((hw[m] >> 8) & 0xF) | (((hw[m] >> 13) & 0x7) << 4)
        simd = (hw[m] >> 4) & 3
        key = cu * 4 + simd
        busy = np.bincount(key, weights=(t1[m] - t0[m]).astype(np.float64))
        last = np.zeros(busy.shape)
        np.maximum.at(last, key, t1[m].astype(np.float64))
        used = busy > 0
        d = dur[m]
        print(f'XCD {x}: {m.sum()} waves, span {span} ticks, mean wave {d.mean():.0f}, SIMDs {used.sum()}, '
              f'slot fill {busy[used].mean() / span:.2f} of 4, last-wave end per SIMD p10/p50 '
              f'{np.percentile(last[used], 10):.0f}/{np.median(last[used]):.0f}, 99% done at '
              f'{np.sort(t1[m])[int(0.99 * m.sum())] / span:.2f} of span')
        if x == np.unique(xcc)[0]:
            for q in range(8):
                lo, hi = span * q / 8, span * (q + 1) / 8
                mm = (t0[m] >= lo) & (t0[m] < hi)
                if mm.any():
                    print(f'    started in [{lo:7.0f}, {hi:7.0f}): {mm.sum():5d} waves, mean duration {d[mm].mean():7.0f}')


if __name__ == '__main__':
    main()
