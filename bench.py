"""Benchmark: license files scored/sec vs all templates (Dice), % of HBM roofline.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5] [--files-per-gpu F]

Default workload (BASELINE.json configs[1], "config2"): 1,000,000 synthetic perturbed
LICENSE files per GPU scored against the 47 vendored choosealicense.com templates
(Dice#match with the default threshold 98). Files are generated in normalized space
(licensee_amd/csrc/synth.cpp), interned to bitsets, uploaded once and stay resident in HBM;
a step is one dice_batch_match launch over the whole batch (inputs and results in HBM).
For N > 1 (torch.distributed.run, one rank per GPU) each rank scores its own disjoint
1M-file shard -- no data-path collective, "scaling": "weak"; results are gathered once
after the timed region (host D2H and RCCL all_gather both timed, reported as extras).

The JSON line also carries:
  roofline     -- algorithmic bytes per launch (tile bitset + |W_F| + len + cc + 16 B of
                  results per file) / average launch duration from HIP events on the launch
                  stream; peak 8000 GB/s (MI355X HBM3E). traffic = per-launch HBM bytes from
                  the committed rocprofv3 PMC pass (profiles/pmc_<config>.json) when present.
  cpu_baseline -- oracle/dice_ref.c (C port of the reference Set#& algorithm), rank 0 at N=1,
                  on a bounded sample of the same files, threads stated.
  parity       -- GPU results of the timed run vs the C oracle on that sample (bit-exact).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = 'license files scored/sec (whole node) vs all templates; % HBM roofline'
HBM_PEAK_GBS = 8000.0


def log(*a):
    print('[bench]', *a, file=sys.stderr, flush=True)


def build_workload(config: int):
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.license import License
    templates = License.all(hidden=True, pseudo=False)
    if config == 3:
        from licensee_amd.synth_templates import synthetic_templates
        templates = synthetic_templates(templates, 600, seed=20250202)
    corpus = TemplateCorpus(templates)
    return templates, corpus


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=100)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--config', type=int, default=2, choices=[2, 3, 4, 5])
    ap.add_argument('--files-per-gpu', type=int, default=None)
    ap.add_argument('--threshold', type=float, default=98.0)
    ap.add_argument('--topk', type=int, default=3)
    ap.add_argument('--cpu-seconds', type=float, default=15.0, help='CPU-work budget of the baseline sample')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--probe', action='store_true', help='diagnostic: stream-read the tiles only (read ceiling)')
    args = ap.parse_args()

    # stdout carries exactly one JSON line: anything native libraries print there (RCCL's
    # version banner at communicator init, for one) is sent to stderr instead.
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    distributed = 'RANK' in os.environ and 'MASTER_PORT' in os.environ   # launched by torch.distributed.run
    if distributed:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        torch.cuda.set_device(local_rank)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local_rank))
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()

    from licensee_amd.synth import SyntheticCorpus
    from licensee_amd._native import Scorer

    cfg = args.config
    default_files = {2: 1_000_000, 3: 1_250_000, 4: 1_000_000, 5: 1_000_000}[cfg]
    n_per = args.files_per_gpu or default_files
    templates, corpus = build_workload(cfg)
    synth = SyntheticCorpus(corpus, profile=1 if cfg == 4 else 0)
    nthreads = min(16, os.cpu_count() or 1)
    t0 = time.time()
    from licensee_amd.shard import shard_range
    first, count = shard_range(rank, world, n_per)
    files = synth.generate(first, count, seed=20250202, nthreads=nthreads)
    log(f'rank {rank}: generated {n_per} files in {time.time() - t0:.1f}s (V={corpus.n_vocab}, T={len(templates)})')

    scorer = Scorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack, corpus.length,
                    corpus.is_cc, n_vocab=corpus.n_vocab, device=dev)
    T, V, kind, entries = scorer.info()
    batch = scorer.batch(n_per)
    stream = torch.cuda.Stream()          # a real (non-null) stream: kernels and HIP events share it
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream
    batch.upload(files, sptr)
    torch.cuda.synchronize()

    def step():
        if args.probe:
            batch.stream_probe(sptr)
        elif cfg == 5:
            batch.matrix(args.topk, sptr)
        else:
            batch.match(args.threshold, sptr)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t_start = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t_start
    ev_ms = ev0.elapsed_time(ev1)
    if distributed:
        t = torch.tensor([wall, ev_ms], dtype=torch.float64, device='cuda')
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall, ev_ms = float(t[0]), float(t[1])

    total_files = n_per * world
    value = total_files * args.steps / wall
    launch_ms = ev_ms / args.steps
    tile_bytes = batch.bytes_per_file()
    if cfg == 5:
        out_bytes = T * 12 + args.topk * 12
    else:
        out_bytes = 16
    algo_bytes_per_file = tile_bytes + 4 + 4 + 1 + out_bytes
    achieved = algo_bytes_per_file * n_per / (launch_ms * 1e-3) / 1e9
    traffic = None
    traffic_src = None
    pmc_path = os.path.join(ROOT, 'profiles', f'pmc_config{cfg}.json')
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as fh:
                pmc = json.load(fh)
            if pmc.get('files_per_launch') == n_per and pmc.get('templates') == T:
                traffic = pmc.get('hbm_bytes_per_launch')
                traffic_src = f"profiles/pmc_config{cfg}.json ({pmc.get('tag')})"
        except Exception:
            traffic = None

    # ---- results: parity + gathers (outside the timed region) -------------------------
    extras = {}
    if cfg != 5:
        t_g = time.perf_counter()
        best, ov, score = batch.download_match(sptr)
        host_gather_s = time.perf_counter() - t_g
        extras['host_gather_ms'] = host_gather_s * 1e3
        extras['matches'] = int((best >= 0).sum())
        if distributed:
            # RCCL alternative: all_gather the 16-B/file results over xGMI
            res = torch.empty((n_per, 4), dtype=torch.int32, device='cuda')
            hip = ctypes.CDLL('libamdhip64.so.7')   # by soname: the runtime torch already loaded
            pb, po, ps = batch.result_ptrs()
            hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
            tmp_b = torch.empty(n_per, dtype=torch.int32, device='cuda')
            tmp_o = torch.empty(n_per, dtype=torch.int32, device='cuda')
            tmp_s = torch.empty(n_per, dtype=torch.float64, device='cuda')
            hip.hipMemcpy(tmp_b.data_ptr(), pb, n_per * 4, 3)
            hip.hipMemcpy(tmp_o.data_ptr(), po, n_per * 4, 3)
            hip.hipMemcpy(tmp_s.data_ptr(), ps, n_per * 8, 3)
            res[:, 0] = tmp_b
            res[:, 1] = tmp_o
            res[:, 2:4] = tmp_s.view(torch.int32).view(n_per, 2)
            out = torch.empty((world * n_per, 4), dtype=torch.int32, device='cuda')
            torch.cuda.synchronize()
            dist.barrier()
            t_g = time.perf_counter()
            dist.all_gather_into_tensor(out, res)
            torch.cuda.synchronize()
            rccl_s = time.perf_counter() - t_g
            t = torch.tensor([host_gather_s, rccl_s], dtype=torch.float64, device='cuda')
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            extras['host_gather_ms'] = float(t[0]) * 1e3
            extras['rccl_allgather_ms'] = float(t[1]) * 1e3
            extras['gather_winner'] = 'host' if t[0] <= t[1] else 'rccl'

    # ---- separately reported rates (never `value`): PCIe-inclusive end-to-end, host prep ----
    if rank == 0 and cfg != 5 and not args.probe:
        torch.cuda.synchronize()
        t_e = time.perf_counter()
        batch.upload(files, sptr)
        batch.match(args.threshold, sptr)
        batch.download_match(sptr)
        extras['e2e_pcie_files_per_s'] = n_per / (time.perf_counter() - t_e)
        from licensee_amd.project_files import LicenseFile
        sample = [synth.text(i)[0] for i in range(200)]
        t_h = time.perf_counter()
        prepped = [LicenseFile(txt, 'LICENSE') for txt in sample]
        for lf in prepped:
            lf.content_normalized()
        corpus.intern_files(prepped)
        extras['host_prep_python_files_per_s'] = len(sample) / (time.perf_counter() - t_h)
        from licensee_amd.native_host import HostPrep
        hp = HostPrep(corpus)
        big = [synth.text(i)[0] for i in range(2000)]
        t_h = time.perf_counter()
        hp.prep_files(big, None, nthreads=nthreads)
        extras['host_prep_native_files_per_s'] = len(big) / (time.perf_counter() - t_h)
        extras['host_prep_note'] = (f'normalize+intern+Copyright/Exact of synthetic texts: Python 1 thread; '
                                    f'native (csrc/normalize.cpp) {nthreads} threads')

    cpu_baseline = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle.native import OracleScorer, bits_to_csr
        orc = OracleScorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack,
                           corpus.length, corpus.is_cc, corpus.n_vocab)
        cpu_threads = nthreads
        # calibrate on a small slice, then size the sample to ~cpu_seconds of CPU work
        cal = min(n_per, 4000)
        csr = bits_to_csr(files.bits[:cal], corpus.n_vocab)
        tc = time.perf_counter()
        orc.match(files.bits[:cal], files.wordset_size[:cal], files.length[:cal], files.cc_false_positive[:cal],
                  args.threshold, nthreads=1, mode=0, csr=csr)
        per_file = (time.perf_counter() - tc) / cal
        sample = int(min(n_per, max(cal, args.cpu_seconds / max(per_file, 1e-9))))
        sl = slice(0, sample)
        csr = bits_to_csr(files.bits[sl], corpus.n_vocab)
        tc = time.perf_counter()
        cb, co, cs = orc.match(files.bits[sl], files.wordset_size[sl], files.length[sl],
                               files.cc_false_positive[sl], args.threshold, nthreads=cpu_threads, mode=0, csr=csr)
        cpu_s = time.perf_counter() - tc
        tc = time.perf_counter()
        orc.match(files.bits[sl], files.wordset_size[sl], files.length[sl], files.cc_false_positive[sl],
                  args.threshold, nthreads=cpu_threads, mode=1)
        cpu_bits_s = time.perf_counter() - tc
        cpu_baseline = {'value': sample / cpu_s, 'unit': 'files/s', 'cores': cpu_threads, 'kind': 'port',
                        'sample': f'first {sample} files of the same synthetic workload, hash-set Set#& '
                                  f'restatement (oracle/dice_ref.c), {cpu_threads} threads',
                        'bitset_variant_files_per_s': sample / cpu_bits_s}
        if cfg != 5:
            mism = int(np.sum(best[sl] != cb) + np.sum(ov[sl] != co) + np.sum(score[sl] != cs))
            parity = {'checked_files': sample, 'mismatches': mism, 'oracle': 'oracle/dice_ref.c'}
        else:
            ovm, scm, tki, tks = batch.download_matrix(args.topk, sptr)
            mov, msc = orc.matrix(files.bits[sl], files.wordset_size[sl], files.length[sl],
                                  files.cc_false_positive[sl], nthreads=cpu_threads)
            mism = int(np.sum(ovm[sl] != mov) + np.sum(scm[sl] != msc))
            parity = {'checked_files': sample, 'mismatches': mism, 'oracle': 'oracle/dice_ref.c (matrix)'}

    if rank == 0:
        workload = {2: 'config2: synthetic perturbed LICENSE files x 47 choosealicense.com templates, Dice#match thr 98',
                    3: 'config3: synthetic files x ~600 synthetic templates (LDS-tiled sparse kernel)',
                    4: 'config4: long/mixed COPYING files (2-6 templates + notices) x 47 templates',
                    5: f'config5: full N x T similarity matrix + top-{args.topk} x 47 templates'}[cfg]
        line = {
            'metric': METRIC, 'value': value, 'unit': 'files/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': wall / args.steps * 1e3, 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None, 'dtype': 'u32',
            'data': 'synthetic (normalized-space perturbations of the vendored templates, seed 20250202)',
            'config': {'workload': workload, 'files_per_gpu': n_per, 'global_files': total_files,
                       'templates': T, 'vocab': V, 'kernel': ['dense', 'sparse-program', 'lds-sparse'][kind],
                       'program_entries': entries, 'parallelism': f'shard{world}'},
            'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic,
                         'traffic_source': traffic_src,
                         'algorithmic_bytes_per_file': algo_bytes_per_file, 'launch_ms': launch_ms,
                         **({'note': 'config 3 is compute-bound (VALU/LDS issue of the LDS-tiled kernel); '
                                     'frac is its HBM share only (DESIGN.md 4b)'} if kind == 2 else {})},
            'cpu_baseline': cpu_baseline,
            'scores_per_s': value * T,
            'parity': parity,
            'extras': extras,
        }
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(line) + '\n').encode())
    if distributed:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
