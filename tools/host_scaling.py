"""Thread scaling of the native host stage (lh_normalize_files) by batch size.

    python tools/host_scaling.py [max_threads]

Prints files/s for 1, 2, 4, ... max_threads threads on 16,000 synthetic config-2 texts (bytes) in
batches of 16,000 / 4,000 / 1,000 files. (Round 6 measured a persistent worker pool against
threads spawned per call with it: the pool was 5-12% slower at 4-16 threads on the GPU box,
profiles/raw/r6g_host_scaling_*.txt, and was removed.)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    top = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    from licensee_amd import native_host
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.license import License
    from licensee_amd.synth import SyntheticCorpus
    corpus = TemplateCorpus(License.all(hidden=True, pseudo=False))
    syn = SyntheticCorpus(corpus)
    big = [syn.text(i)[0].encode() for i in range(16000)]
    hp = native_host.HostPrep(corpus)
    th = 1
    while th <= top:
        hp.normalize_files(big[:512], None, nthreads=th)
        row = []
        for bs in (16000, 4000, 1000):
            best = 1e9
            for _ in range(3):
                t0 = time.perf_counter()
                for i in range(0, len(big), bs):
                    hp.normalize_files(big[i:i + bs], None, nthreads=th)
                best = min(best, time.perf_counter() - t0)
            row.append(f'batch {bs}: {len(big) / best:9.3g}')
        print(f'threads {th:2d}: ' + '  '.join(row), flush=True)
        th *= 2


if __name__ == '__main__':
    main()
