"""Where the batched LicenseFile#license pipeline (batch.BatchDetector.detect_stream) spends its time.

    python tools/e2e_profile.py [batches] [batch_size] [threads] [torch] [heap] [objs] [prep] [oracle]

Times, on synthetic config-2 texts as bytes: the whole two-stage stream; the host stage alone
(BatchDetector._prep: lh_normalize_files, or lh_prep_files with wordset_on=host); the device
stage alone (_score: upload + wordset scan + Exact + Dice#match/#confidence + downloads +
Detection objects) and, inside it, the Detection objects. One JSON line per wordset mode.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    bs = int(sys.argv[2]) if len(sys.argv) > 2 else 4000
    threads = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    # (diagnostics: the conditions of bench.py's process) torch initialised with CPU tensor work
    # done, a large resident heap, bench.py's host-preparation phases, ~15 s of CPU load first
    keep = []
    if 'torch' in sys.argv[4:]:
        import torch
        torch.cuda.init()
        x = torch.randn(4096, 4096)
        keep.append((x @ x).sum().item())
        keep.append(torch.empty(1 << 24, dtype=torch.uint8).pin_memory())
    if 'objs' in sys.argv[4:]:   # a large heap of collector-tracked objects
        keep.append([[i] for i in range(3_000_000)])
    if 'heap' in sys.argv[4:]:
        import numpy as np
        keep.append(np.ones(1 << 31, np.uint8))
        keep.append([str(i) for i in range(5_000_000)])
    if 'prep' in sys.argv[4:] or 'oracle' in sys.argv[4:]:
        # bench.py's phases before its end-to-end leg: the batched host preparation and
        # normalization of 16,000 texts (results kept), and/or a CPU load like its baseline leg's
        from licensee_amd.corpus import TemplateCorpus as _TC
        from licensee_amd.license import License as _L
        from licensee_amd.native_host import HostPrep
        from licensee_amd.synth import SyntheticCorpus as _SC
        _c = _TC(_L.all(hidden=True, pseudo=False))
        _s = _SC(_c)
        big = [_s.text(i)[0].encode('utf-8') for i in range(16000)]
        if 'prep' in sys.argv[4:]:
            hp = HostPrep(_c)
            hp.prep_files(big, None, nthreads=threads)
            keep.append(hp.normalize_files(big, None, nthreads=threads))
        if 'oracle' in sys.argv[4:]:   # (the CPU-baseline leg's load: ~15 s on every granted core)
            hp2 = HostPrep(_c)
            t_end = time.perf_counter() + 15
            while time.perf_counter() < t_end:
                hp2.prep_files(big[:4000], None, nthreads=threads)
        keep.append(big)
    from licensee_amd.batch import BatchDetector
    from licensee_amd.dice import DiceEngine
    from licensee_amd.synth import SyntheticCorpus
    eng = DiceEngine(device=0)
    syn = SyntheticCorpus(eng.corpus)
    # bench.py's texts: 4 distinct batches (texts 0 .. 4 * batch_size - 1), cycled
    texts = [syn.text(i)[0].encode('utf-8') for i in range(bs * 4)]
    chunks = [(texts[(k % 4) * bs:(k % 4 + 1) * bs], None) for k in range(nb)]
    for mode in ('device', 'host'):
        det = BatchDetector(eng, nthreads=threads, wordset_on=mode)
        for _ in det.detect_stream(chunks[:2]):
            pass
        runs = []
        for _ in range(3):   # (the median of 3 streams)
            t0 = time.perf_counter()
            n = sum(len(d) for d in det.detect_stream(chunks))
            runs.append(time.perf_counter() - t0)
        stream_s = sorted(runs)[1]
        t0 = time.perf_counter()
        prepped = [det._prep(*c) for c in chunks[:2]]
        host_s = (time.perf_counter() - t0) / 2
        t0 = time.perf_counter()
        for p in prepped:
            det._score(p, 98.0)
        dev_s = (time.perf_counter() - t0) / 2
        if mode == 'device':
            t0 = time.perf_counter()
            r = det._score_text(prepped[0], 98.0)
            raw_s = time.perf_counter() - t0
            t0 = time.perf_counter()
            det._detections(*r)
            obj_s = time.perf_counter() - t0
        else:
            raw_s = obj_s = None
        print(json.dumps({'wordset_on': mode, 'batch': bs, 'threads': threads,
                          'stream_files_per_s': n / stream_s, 'stream_runs_files_per_s': [round(n / r) for r in runs], 'host_stage_ms': host_s * 1e3,
                          'device_stage_ms': dev_s * 1e3,
                          'device_stage_without_objects_ms': raw_s * 1e3 if raw_s else None,
                          'detection_objects_ms': obj_s * 1e3 if obj_s else None}), flush=True)
        det.close()


if __name__ == '__main__':
    main()
