"""The device wordset scan alone (dice_batch_upload_text, csrc/dice_words.hip), for rocprofv3.

    python tools/words_bench.py [n_texts] [reps]

Prepares n synthetic config-2 texts on the host (lh_normalize_files, 16 threads), uploads them
`reps` times and prints one JSON line: host normalization rate, the upload's wall time (H2D of
the texts + the scan kernel + status read-back), the kernel's HIP-event time on its stream, and
the algorithmic bytes per file (text bytes + offsets/lengths in, row + |W_F| + mask + status out).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    import numpy as np
    import torch
    from licensee_amd._native import Scorer
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.license import License
    from licensee_amd.native_host import HostPrep
    from licensee_amd.synth import SyntheticCorpus
    corpus = TemplateCorpus(License.all(hidden=True, pseudo=False))
    hp = HostPrep(corpus)
    syn = SyntheticCorpus(corpus)
    base = [syn.text(i)[0].encode('utf-8') for i in range(4000)]
    texts = [base[i % len(base)] for i in range(n)]
    hp.normalize_files(texts[:256], None, nthreads=16)
    t0 = time.perf_counter()
    text, off, tl, ln, cc, _, _ = hp.normalize_files(texts, None, nthreads=16)
    host_s = time.perf_counter() - t0
    sc = Scorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack, corpus.length,
                corpus.is_cc, corpus.n_vocab, device=0)
    sc.vocab_setup(corpus.vocab, hp.nv_fields)
    b = sc.batch(n)
    pin = torch.from_numpy(text).pin_memory().numpy()
    stream = torch.cuda.Stream()
    st = b.upload_text(pin, off, tl, ln, cc, stream.cuda_stream)
    assert not st.any()
    walls = []
    for _ in range(reps):
        t0 = time.perf_counter()
        b.upload_text(pin, off, tl, ln, cc, stream.cuda_stream)
        walls.append(time.perf_counter() - t0)
    w64 = (corpus.n_vocab + 63) // 64
    per_file = len(text) / n + 8 + 4 + 4 + 1 + 8 * w64 + 4 + 8 + 1
    out = {'n_texts': n, 'text_bytes_per_file': round(len(text) / n, 1), 'host_normalize_files_per_s': n / host_s,
           'upload_text_ms_median': sorted(walls)[len(walls) // 2] * 1e3,
           'upload_text_files_per_s': n / sorted(walls)[len(walls) // 2],
           'algorithmic_bytes_per_file': round(per_file, 1)}
    print(json.dumps(out))
    b.close()
    sc.close()


if __name__ == '__main__':
    main()
