"""Benchmark: license files scored/sec vs all templates (Dice), % of HBM roofline.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5] [--files-per-gpu F]

Default workload (BASELINE.json configs[1], "config2"): 1,000,000 synthetic perturbed
LICENSE files per GPU scored against the 47 vendored choosealicense.com templates
(Dice#match with the default threshold 98). Files are generated in normalized space
(licensee_amd/csrc/synth.cpp), interned to bitsets, uploaded once and stay resident in HBM;
a step is one dice_batch_match launch over the whole batch (inputs and results in HBM).
For N > 1 one process per GPU: `python bench.py --gpus N` starts the N ranks itself (a child
torch.distributed.run on 127.0.0.1, before any GPU call in this process) and relays rank 0's
line; under an external torch.distributed.run it runs as one of the ranks (WORLD_SIZE must equal
--gpus). Each rank scores its own disjoint 1M-file shard -- no data-path collective, "scaling":
"weak"; results are gathered once after the timed region (host D2H and RCCL all_gather both
timed, the faster reported as gather_winner). RCCL (backend nccl) when every rank has its own
device; gloo when ranks share one (the one-GPU box's rehearsal of the N > 1 path).

The JSON line also carries:
  roofline     -- algorithmic bytes per launch (tile bitset + |W_F| + len + cc + 16 B of
                  results per file) / average launch duration from HIP events on the launch
                  stream; peak 8000 GB/s (MI355X HBM3E). traffic = per-launch HBM bytes from
                  the committed rocprofv3 PMC pass (profiles/pmc_<config>.json) when present.
  cpu_baseline -- oracle/dice_ref.c (C port of the reference Set#& algorithm), rank 0, on a
                  bounded sample of its own shard, on every core the process may use (the other
                  ranks wait meanwhile).
  parity       -- GPU results of the timed run vs the C oracle's hash mode: every rank checks a
                  sample of its own shard; checked files and mismatches are summed over ranks.
  extras.configs -- the other BASELINE configs (3: ~600 templates, bound-pruned match
                  kernel through dice_batch_match_confidence: Dice#match + #confidence, 0 for a
                  file without a match; plus '3-top1': the same files through dice_batch_match,
                  which also ranks the unmatched files' templates, and '3-allpairs': the same files
                  on the postings kernel, which scores every pair; 4: long/mixed files; 5: full matrix + top-k) measured in the same
                  run (every rank, its own shard), each with its own HIP-event launch time, roofline
                  fraction, cpu_baseline and oracle parity sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = 'license files scored/sec (whole node) vs all templates; % HBM roofline'
HBM_PEAK_GBS = 8000.0
DEFAULT_FILES = {2: 1_000_000, 3: 1_250_000, 4: 1_000_000, 5: 1_000_000, '5-T600': 1_250_000}
KERNELS = ['dense', 'sparse-program', 'lds-records', 'postings', 'bound-pruned']
WORKLOADS = {2: 'config2: synthetic perturbed LICENSE files x 47 choosealicense.com templates, Dice#match thr 98',
             3: 'config3: synthetic files x ~600 synthetic templates, Dice#match thr 98, one GPU shard '
                'of the 10M-file node run',
             4: 'config4: long/mixed COPYING files (2-6 templates + notices) x 47 templates',
             5: 'config5: full N x T similarity matrix + top-k x 47 templates',
             '5-T600': 'config5 at T ~ 600: full N x T similarity matrix + top-k, config-3 files x 600 synthetic '
                       'templates (licensee detect closest licenses on a large corpus)'}


def log(*a):
    print('[bench]', *a, file=sys.stderr, flush=True)


def cpu_info():
    """Cores this process may run on: the affinity mask, capped by a cgroup CPU quota."""
    affinity = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open('/sys/fs/cgroup/cpu.max') as fh:
            q, p = fh.read().split()[:2]
            if q != 'max':
                quota = max(1, -(-int(q) // int(p)))
    except (OSError, ValueError):
        pass
    model = None
    try:
        with open('/proc/cpuinfo') as fh:
            for line in fh:
                if line.startswith('model name'):
                    model = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    usable = min(affinity, quota) if quota else affinity
    return {'threads': max(1, min(usable, 256)), 'affinity_cpus': affinity, 'cgroup_cpu_quota': quota,
            'nproc': os.cpu_count(), 'cpu_model': model}


def build_workload(config: int, corpus: str = 'synthetic'):
    """The template corpus of a config. Config 3's ~600 templates: 'synthetic' = the 47 vendored
    templates + synthetic ones; 'spdx' = 94 real texts (the 47 choosealicense.com templates and
    the 47 SPDX license-list-XML texts, licensee_amd/spdx.py) + synthetic ones."""
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.license import License
    templates = License.all(hidden=True, pseudo=False)
    if config == 3 and corpus == 'spdx':
        from licensee_amd.spdx import corpus_with_spdx
        templates = corpus_with_spdx(templates, total=600)
    elif config == 3:
        from licensee_amd.synth_templates import synthetic_templates
        templates = synthetic_templates(templates, 600, seed=20250202)
    return TemplateCorpus(templates)


def traffic_variant(cfg, run):
    """The committed PMC file of a run's mode: config 3 on the postings kernels '_post', on the pruned
    kernel through dice_batch_match '_top1'."""
    if cfg == 3 and run.match_kernel == 3:
        return '_post'
    if cfg == 3 and run.match_kernel == 4 and not run.confidence:
        return '_top1'
    return ''


def traffic_for(cfg, n_per, T, variant=''):
    """Per-launch HBM bytes from the committed PMC pass of this workload (variant '_post': config 3
    on the postings kernels), or None."""
    pmc_path = os.path.join(ROOT, 'profiles', f'pmc_config{cfg}{variant}.json')
    if not os.path.exists(pmc_path):
        return None, None
    try:
        with open(pmc_path) as fh:
            pmc = json.load(fh)
        if pmc.get('files_per_launch') == n_per and pmc.get('templates') == T:
            return pmc.get('hbm_bytes_per_launch'), f"profiles/pmc_config{cfg}{variant}.json ({pmc.get('tag')})"
    except Exception:
        pass
    return None, None


class Run:
    """One config's workload resident on the GPU: corpus, files, scorer, batch."""

    def __init__(self, cfg, n_per, rank, world, dev, nthreads, args):
        from licensee_amd._native import Scorer
        from licensee_amd.shard import shard_range
        from licensee_amd.synth import SyntheticCorpus
        self.tag = cfg
        if cfg == '5-T600':          # matrix mode over the config-3 corpus and files
            cfg, corpus_cfg = 5, 3
        else:
            corpus_cfg = cfg
        self.cfg, self.n_per, self.args = cfg, n_per, args
        t0 = time.time()
        self.corpus = build_workload(corpus_cfg, getattr(args, 'corpus', 'synthetic'))
        self.synth = SyntheticCorpus(self.corpus, profile=1 if cfg == 4 else 0)
        first, count = shard_range(rank, world, n_per)
        self.files = self.synth.generate(first, count, seed=20250202, nthreads=nthreads)
        log(f'config {cfg} rank {rank}: generated {n_per} files in {time.time() - t0:.1f}s '
            f'(V={self.corpus.n_vocab}, T={len(self.corpus.templates)})')
        c = self.corpus
        self.scorer = Scorer(c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc,
                             n_vocab=c.n_vocab, device=dev)
        self.T, self.V, self.kind, self.entries = self.scorer.info()
        self.match_kernel = self.scorer.match_kernel() if cfg != 5 else self.kind
        self.batch = self.scorer.batch(n_per)
        out_bytes = self.T * 12 + args.topk * 12 if cfg == 5 else 16
        # the file bitset as the kernels read it: tile layout (T <= 64) or row-major rows (T > 64)
        in_bytes = self.batch.bytes_per_file() if self.kind != 3 else 8 * ((self.V + 63) // 64)
        self.algo_bytes_per_file = in_bytes + 4 + 4 + 1 + out_bytes
        # dice_batch_match_confidence (Dice#match + #confidence) or dice_batch_match (also the top
        # template of an unmatched file); --match-mode auto: the former where it changes the work
        # (the bound-pruned kernel, config 3)
        mode = getattr(args, 'match_mode', 'auto')
        self.confidence = cfg != 5 and (mode == 'confidence' or (mode == 'auto' and self.match_kernel == 4))

    def step(self, sptr):
        if self.args.probe:
            self.batch.stream_probe(sptr)
        elif self.cfg == 5:
            self.batch.matrix(self.args.topk, sptr)
        else:
            self.batch.match(self.args.threshold, sptr, confidence=self.confidence)

    def close(self):
        self.batch.close()
        self.scorer.close()

    def rescore(self, env, dev):
        """Swap in a scorer built under extra environment switches (read at dice_create), same
        corpus and files; returns the old (scorer, batch) for restore()."""
        from licensee_amd._native import Scorer
        old_env = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            c = self.corpus
            sc = Scorer(c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc,
                        n_vocab=c.n_vocab, device=dev)
        finally:
            for k, v in old_env.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        saved = (self.scorer, self.batch, self.match_kernel)
        self.scorer, self.batch = sc, sc.batch(self.n_per)
        self.match_kernel = sc.match_kernel()
        return saved

    def restore(self, saved):
        self.close()
        self.scorer, self.batch, self.match_kernel = saved


class Group:
    """The ranks of this run (world 1: no-ops). Collectives go over the process group's backend:
    RCCL with device tensors, or gloo with host tensors when ranks share a device."""

    def __init__(self, rank=0, world=1, backend=None):
        self.rank, self.world, self.backend = rank, world, backend

    def _t(self, vals, dtype):
        import torch
        return torch.tensor(vals, dtype=dtype, device='cuda' if self.backend == 'nccl' else 'cpu')

    def barrier(self):
        if self.world > 1:
            import torch.distributed as dist
            dist.barrier()

    def reduce(self, vals, op='max'):
        """Element-wise max or sum of a list of floats over the ranks."""
        if self.world == 1:
            return list(vals)
        import torch
        import torch.distributed as dist
        t = self._t(vals, torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == 'max' else dist.ReduceOp.SUM)
        return [float(x) for x in t.cpu()]

    def bcast(self, val):
        """Rank 0's integer to every rank."""
        if self.world == 1:
            return val
        import torch
        import torch.distributed as dist
        t = self._t([int(val)], torch.int64)
        dist.broadcast(t, 0)
        return int(t.cpu()[0])


def timed(run, steps, warmup, stream, group):
    """W untimed steps, then K steps between barrier + synchronize; HIP events on the launch
    stream give the per-launch time; wall time and event time are max-reduced over ranks."""
    import torch
    sptr = stream.cuda_stream
    run.batch.upload(run.files, sptr)
    torch.cuda.synchronize()
    for _ in range(warmup):
        run.step(sptr)
    torch.cuda.synchronize()
    group.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t_start = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        run.step(sptr)
    ev1.record(stream)
    torch.cuda.synchronize()
    group.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t_start
    ev_ms = ev0.elapsed_time(ev1)
    wall, ev_ms = group.reduce([wall, ev_ms], 'max')
    launch_ms = ev_ms / steps
    achieved = run.algo_bytes_per_file * run.n_per / (launch_ms * 1e-3) / 1e9
    return wall, launch_ms, achieved


def staged_parity(group, check):
    """Every rank's oracle parity check of its own shard, rank 0 first while the others wait (so
    rank 0's oracle time -- the cpu_baseline -- runs on an otherwise idle host), then the rest
    together. check() -> dict with checked_files, mismatches, oracle[, oracle_files_per_s].
    Returns rank 0's dict with checked_files / mismatches summed over the ranks."""
    res = check() if group.rank == 0 else None
    group.barrier()
    if group.rank != 0:
        res = check()
    group.barrier()
    tot = group.reduce([res['checked_files'], res['mismatches']], 'sum')
    res['checked_files'], res['mismatches'] = int(tot[0]), int(tot[1])
    if group.world > 1:
        res['ranks_checked'] = group.world
    return res


def oracle_for(corpus):
    from oracle.native import OracleScorer
    return OracleScorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack,
                        corpus.length, corpus.is_cc, corpus.n_vocab)


def parity_sample(run, orc, sptr, threads, n_sample):
    """GPU results of the timed batch vs the C oracle's hash mode (Set#& restatement) on the
    first n_sample files: match results, or for config 5 the matrix and its top-1."""
    f = run.files
    sl = slice(0, min(n_sample, run.n_per))
    if run.cfg != 5:
        best, ov, score = run.batch.download_match(sptr)
        t0 = time.perf_counter()
        eb, eo, es = orc.match(f.bits[sl], f.wordset_size[sl], f.length[sl], f.cc_false_positive[sl],
                               run.args.threshold, nthreads=threads, mode=0)
        cpu_s = time.perf_counter() - t0
        if run.confidence:   # Dice#confidence: 0 for a file without a match (dice.rb:51-53)
            eo, es = np.where(eb >= 0, eo, 0), np.where(eb >= 0, es, 0.0)
        mism = int(np.sum(best[sl] != eb) + np.sum(ov[sl] != eo) + np.sum(score[sl] != es))
        return {'checked_files': sl.stop, 'mismatches': mism, 'oracle': 'oracle/dice_ref.c (hash Set#&)',
                'oracle_files_per_s': sl.stop / cpu_s}
    if run.n_per > n_sample:
        # the matrix of the sample only (a T ~ 600 matrix of the whole batch is ~9 GB): the same
        # files scored again in a batch of their own
        from licensee_amd._native import FileBatch
        sb = run.scorer.batch(sl.stop)
        sb.upload(FileBatch(f.bits[sl], f.wordset_size[sl], f.length[sl], f.cc_false_positive[sl]), sptr)
        sb.matrix(run.args.topk, sptr)
        ovm, scm, tki, tks = sb.download_matrix(run.args.topk, sptr)
        sb.close()
    else:
        ovm, scm, tki, tks = run.batch.download_matrix(run.args.topk, sptr)
    t0 = time.perf_counter()
    mov, msc = orc.matrix(f.bits[sl], f.wordset_size[sl], f.length[sl], f.cc_false_positive[sl], nthreads=threads)
    cpu_s = time.perf_counter() - t0
    mism = int(np.sum(ovm[sl] != mov) + np.sum(scm[sl] != msc))
    rows = np.arange(sl.stop)
    mism += int(np.sum(scm[rows, tki[sl, 0]] != tks[sl, 0]))
    return {'checked_files': sl.stop, 'mismatches': mism, 'oracle': 'oracle/dice_ref.c (matrix, hash Set#&)',
            'oracle_files_per_s': sl.stop / cpu_s}


def single_file_latency(run, n_calls=400):
    """The drop-in's per-call latency (license_file.rb:92-98 -> dice.rb:34-41 scores one file at a
    time; INTEGRATION.md's Ruby override calls dice_similarity_matrix with n = 1): p50/p99 wall
    time of dice_similarity_matrix and dice_match with n = 1 through ctypes (structs and outputs
    prepared beforehand, as an FFI binding would hold them), beside the C port's per-file time on
    one thread over the same files (oracle/dice_ref.c hash Set#&, no per-call overhead)."""
    import ctypes
    from licensee_amd._native import FileBatch, load_library
    from oracle.native import bits_to_csr
    lib = load_library()
    f, T = run.files, run.T
    n = min(n_calls, f.n)
    singles = [FileBatch(f.bits[i:i + 1], f.wordset_size[i:i + 1], f.length[i:i + 1], f.cc_false_positive[i:i + 1])
               for i in range(n)]
    structs = [fb._struct() for fb in singles]
    ov = np.empty(T, np.uint32)
    sc = np.empty(T, np.float64)
    tki = np.empty(3, np.int32)
    tks = np.empty(3, np.float64)
    b1 = np.empty(1, np.int32)
    o1 = np.empty(1, np.uint32)
    s1 = np.empty(1, np.float64)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    ctx = run.scorer._ctx
    out = {}
    for name, call in (('matrix_n1', lambda st: lib.dice_similarity_matrix(ctx, ctypes.byref(st), p(ov), p(sc), 3,
                                                                            p(tki), p(tks))),
                       ('match_n1', lambda st: lib.dice_match(ctx, ctypes.byref(st), 98.0, p(b1), p(o1), p(s1)))):
        for st in structs[:20]:
            call(st)                      # warm: scratch batch, code paths
        ts = []
        for st in structs:
            t0 = time.perf_counter()
            rc = call(st)
            ts.append(time.perf_counter() - t0)
            assert rc == 0
        ts = np.array(ts) * 1e6
        out[name] = {'p50_us': float(np.percentile(ts, 50)), 'p99_us': float(np.percentile(ts, 99)),
                     'mean_us': float(ts.mean())}
        # the same calls through the general path (scratch batch, pageable copies): the
        # small-call path's gain (DICE_NO_SMALL_CALL is read per call)
        os.environ['DICE_NO_SMALL_CALL'] = '1'
        try:
            for st in structs[:20]:
                call(st)
            tg = []
            for st in structs[:200]:
                t0 = time.perf_counter()
                call(st)
                tg.append(time.perf_counter() - t0)
        finally:
            os.environ.pop('DICE_NO_SMALL_CALL', None)
        out[name]['general_path_p50_us'] = float(np.percentile(np.array(tg) * 1e6, 50))
    orc = oracle_for(run.corpus)
    m = min(4000, f.n)
    csr = bits_to_csr(f.bits[:m], run.corpus.n_vocab)
    t0 = time.perf_counter()
    orc.match(f.bits[:m], f.wordset_size[:m], f.length[:m], f.cc_false_positive[:m], 98.0, nthreads=1, mode=0, csr=csr)
    out['port_1thread_us_per_file'] = (time.perf_counter() - t0) / m * 1e6
    out['note'] = ('wall time per call incl. ctypes; the GPU path is upload + kernel + download + sync of one file; '
                   'port = oracle/dice_ref.c, one thread, per file of a 4000-file run')
    return out


def measure_extra(r, c, args, stream, sptr, cpu, group):
    steps = min(args.steps, 20)
    w, lm, ach = timed(r, steps, 2, stream, group)
    tr, tr_src = traffic_for(c if c != '5-T600' else '5_T600', r.n_per, r.T, traffic_variant(c, r))
    files = r.n_per * group.world
    # exact-scored pairs per launch, counted on the device (dice_batch_scored_pairs: the pruned
    # kernel's exact scores + every pair of its deferred files; n * T for the other kernels)
    scored = r.n_per * r.T if r.cfg == 5 else r.batch.scored_pairs(sptr)
    scored = int(group.reduce([scored], 'sum')[0])
    workload = WORKLOADS[c]
    if r.cfg == 3 and r.match_kernel == 4:
        workload += (' -- entry point dice_batch_match_confidence (Dice#match + #confidence; rounds 1-3 measured '
                     'dice_batch_match: see 3-top1)' if r.confidence else ' -- entry point dice_batch_match (top '
                     'template of every file; the like-for-like figure of rounds 1-3)')
    rec = {'workload': workload, 'files_per_gpu': r.n_per, 'global_files': files, 'templates': r.T,
           'vocab': r.V, 'kernel': KERNELS[r.match_kernel], 'steps': steps, 'files_per_s': files * steps / w,
           'decided_pairs_per_s': files * steps / w * r.T, 'exact_scored_pairs_per_launch': scored,
           'exact_scored_pairs_per_s': scored * steps / w, 'launch_ms': lm,
           'algorithmic_bytes_per_file': r.algo_bytes_per_file, 'roofline_achieved_gbs': ach,
           'roofline_frac': ach / HBM_PEAK_GBS, 'traffic': tr, 'traffic_source': tr_src}
    if r.match_kernel == 4:
        rec['note'] = ('bound-pruned Dice#match: every (file, template) pair is decided, but only pairs whose '
                       'overlap bound can reach the threshold (dice_batch_match_confidence: Dice#match + '
                       '#confidence, dice.rb:8-14,51-53) or the top score (3-top1: dice_batch_match) are scored '
                       'exactly (DESIGN.md 4); decided_pairs_per_s counts every (file, template) pair decided, '
                       'exact_scored_pairs_per_s only those whose overlap was computed (device count). 3-allpairs '
                       'scores every pair')
        rec['entry_point'] = 'dice_batch_match_confidence' if r.confidence else 'dice_batch_match'
        rec['deferred_files'] = int(group.reduce([r.batch.deferred(sptr)], 'sum')[0])
    if not args.no_cpu_baseline:
        n_sample = {3: 20_000, 4: 30_000, 5: 50_000, '5-T600': 10_000}[c]
        threads = cpu['threads'] if group.rank == 0 else cpu['rank_threads']
        par = staged_parity(group, lambda: parity_sample(r, oracle_for(r.corpus), sptr, threads, n_sample))
        # rank 0's parity leg is the reference-equivalent CPU path on its own files: its rate
        rec['cpu_baseline'] = {'value': par.pop('oracle_files_per_s'), 'unit': 'files/s',
                               'cores': cpu['threads'], 'kind': 'port',
                               'sample': f"rank 0's parity sample: first {min(n_sample, r.n_per)} files of its "
                                         f"shard, hash-set Set#& restatement (oracle/dice_ref.c)"}
        rec['parity'] = par
    if group.rank == 0:
        log(f"config {c} ({rec['kernel']}): {rec['files_per_s']:.3e} files/s, launch {lm * 1e3:.1f} us, "
            f"frac {rec['roofline_frac']:.3f}, parity {rec.get('parity')}")
    return rec


def collective_gather_leg(res, host_dst, group, rank, reps, sync):
    """The collective form of the result gather: every rank's packed [n, 4] int32 results
    (licensee_amd.shard.pack_results layout) to rank 0 with dist.gather, then one copy into rank
    0's host buffer `host_dst` ([world * n, 4], shard order). Timed from a barrier, median of
    `reps`, max over ranks; returns seconds. `sync` drains the device (torch.cuda.synchronize with
    RCCL; a no-op for host tensors over gloo, which tests/test_distributed.py drives)."""
    from licensee_amd.shard import gather_packed_to0
    tr = []
    for _ in range(reps):
        sync()
        group.barrier()
        t0 = time.perf_counter()
        g = gather_packed_to0(res)
        if rank == 0:
            host_dst.copy_(g)
        sync()
        group.barrier()
        tr.append(time.perf_counter() - t0)
    return group.reduce([float(np.median(tr))], 'max')[0]


def gather_winner(host_s, rccl_s):
    """The faster result gather (north_star: RCCL solely for the gather, or the host gather if it
    proves faster); ties go to the host gather."""
    return 'host' if host_s <= rccl_s else 'rccl'


def gather_compare(batch, group, rank, world, n_per, best, ov, score, sptr, reps=3):
    """The one result move of a sharded run, two ways, both ending with every rank's 16-B/file
    results in rank 0's host memory (north_star: RCCL solely for the gather, or a host gather if
    faster), each timed end to end from a barrier (median of `reps`, max over ranks):
      host -- each rank's D2H lands straight in its slice of a node-shared, page-locked host buffer
              that rank 0 owns (licensee_amd.shard.SharedResults), then one barrier;
      rccl -- results packed on the device and gathered to rank 0 over xGMI (dist.gather), then
              one D2H into rank 0's page-locked buffer (nccl backend only: ranks on distinct
              devices).
    Rank 0 checks both gathers against each rank's own download."""
    import torch
    import torch.distributed as dist
    from licensee_amd._native import _check, _ptr, load_library
    from licensee_amd.shard import SharedResults, device_results_packed, pack_results
    lib = load_library()
    name = f"licensee_bench_{os.environ.get('MASTER_PORT', '0')}_{os.getppid()}"
    shared = SharedResults(name, world, n_per, create=True) if rank == 0 else None
    group.barrier()
    if shared is None:
        shared = SharedResults(name, world, n_per, create=False)
    out = {}
    pinned = False
    try:
        # page-lock this process's mapping of the segment (once, outside the timed region)
        try:
            rt = torch.cuda.cudart()
            pinned = int(rt.cudaHostRegister(shared.base_ptr, shared.nbytes, 0)) == 0
        except Exception:
            pinned = False
        mine = shared.slice(rank)

        def host_leg():
            _check(lib.dice_batch_download_match(batch._b, _ptr(mine[0]), _ptr(mine[1]), _ptr(mine[2]), sptr or None))
            group.barrier()

        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            group.barrier()
            t0 = time.perf_counter()
            host_leg()
            ts.append(time.perf_counter() - t0)
        host_s = group.reduce([float(np.median(ts))], 'max')[0]
        out['host_gather_ms'] = host_s * 1e3
        out['host_gather'] = {'kind': 'shared-memory host buffer owned by rank 0, each rank D2H into its slice',
                              'pinned': bool(pinned), 'bytes': 16 * n_per * world}
        ok_host = True
        if rank == 0:
            ok_host = bool(np.array_equal(shared.best[:n_per], best) and np.array_equal(shared.overlap[:n_per], ov)
                           and np.array_equal(shared.score[:n_per], score))
        if group.backend == 'nccl':
            res = device_results_packed(batch)
            host_dst = torch.empty((world * n_per, 4), dtype=torch.int32, pin_memory=True) if rank == 0 else None
            rccl_s = collective_gather_leg(res, host_dst, group, rank, reps, torch.cuda.synchronize)
            out['rccl_gather_ms'] = rccl_s * 1e3
            out['gather_winner'] = gather_winner(host_s, rccl_s)
            if rank == 0:
                ref = pack_results(shared.best, shared.overlap, shared.score)
                out['gather_agree'] = bool(np.array_equal(host_dst.numpy(), ref))
        else:
            out['gather_winner'] = 'host'
            out['gather_note'] = 'ranks share a device: no RCCL communicator, host gather only'
        oks = group.reduce([1.0 if ok_host else 0.0], 'sum')[0]
        if rank == 0:
            out['host_gather_checked'] = bool(ok_host) and oks == world
        # every rank checks its own slice of the shared buffer too
        mism = int(np.sum(mine[0] != best) + np.sum(mine[1] != ov) + np.sum(mine[2] != score))
        out['host_gather_mismatches'] = int(group.reduce([mism], 'sum')[0])
        group.barrier()
    finally:
        if pinned:
            try:
                torch.cuda.cudart().cudaHostUnregister(shared.base_ptr)
            except Exception:
                pass
        group.barrier()
        shared.close()
    return out


def abi_sharded_leg(run, args, n_dev, reps=3):
    """The drop-in's own multi-device path in ONE process (what a Ruby/FFI caller would use,
    INTEGRATION.md 3): dice_match_sharded_confidence over `contexts` scorers -- one per visible
    device, or several on one device when there are fewer -- with the results gathered into the
    caller's host buffers directly (DICE_GATHER_HOST) or through the first device (DICE_GATHER_DEVICE),
    timed end to end: H2D of the page-locked inputs, the kernels, the gather (PCIe-inclusive; never
    `value`). Checked against the timed batch's results (Dice#match + #confidence)."""
    import torch
    from licensee_amd._native import (DICE_GATHER_DEVICE, DICE_GATHER_HOST, FileBatch, Scorer, last_gather_peer,
                                      match_sharded)
    n_ctx = max(1, args.abi_contexts or n_dev)
    devices = [i % max(n_dev, 1) for i in range(n_ctx)]
    c, f = run.corpus, run.files
    scorers = [Scorer(c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc, n_vocab=c.n_vocab,
                      device=d) for d in devices]
    pin = lambda a: torch.from_numpy(np.ascontiguousarray(a)).pin_memory().numpy()
    files = FileBatch(pin(f.bits), pin(f.wordset_size), pin(f.length), pin(f.cc_false_positive))
    n = files.n
    outs = (pin(np.empty(n, np.int32)), pin(np.empty(n, np.uint32)), pin(np.empty(n, np.float64)))
    # expected: the resident batch through dice_batch_match_confidence
    run.batch.match(args.threshold, confidence=True)
    torch.cuda.synchronize()
    eb, eo, es = run.batch.download_match()
    rec = {'entry_point': 'dice_match_sharded_confidence', 'contexts': n_ctx, 'devices': devices, 'files': n,
           'input': 'page-locked host arrays (dice_files), results into page-locked host arrays'}
    try:
        for name, mode in (('host', DICE_GATHER_HOST), ('device', DICE_GATHER_DEVICE)):
            match_sharded(scorers, files, args.threshold, gather=mode, confidence=True, out=outs)   # warm
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                match_sharded(scorers, files, args.threshold, gather=mode, confidence=True, out=outs)
                ts.append(time.perf_counter() - t0)
            ms = float(np.median(ts)) * 1e3
            mism = int(np.sum(outs[0] != eb) + np.sum(outs[1] != eo) + np.sum(outs[2] != es))
            rec[name] = {'ms_per_call': ms, 'files_per_s': n / (ms * 1e-3), 'mismatches': mism,
                         'dice_last_gather_peer': last_gather_peer()}
        distinct = len(set(devices))
        if distinct >= 2:
            rec['winner'] = 'host' if rec['host']['ms_per_call'] <= rec['device']['ms_per_call'] else 'device'
        else:
            # every context on one device: the device gather moves nothing between devices, so the
            # two timings are no evidence about xGMI
            rec['winner'] = None
            rec['winner_reason'] = f'{distinct} distinct device(s): no cross-device gather to compare'
        rec['note'] = ('PCIe-inclusive (inputs start in host memory, as the FFI hands them over); the kernel-only rate '
                       'is `value`. dice_last_gather_peer: 1 = every remote shard written over xGMI peer access, '
                       '0 = some staged, -1 = no peer path exercised (host gather, or every context on one device)')
    finally:
        for sc in scorers:
            sc.close()
    return rec


def free_port():
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(n, argv, script=None):
    """`bench.py --gpus N` with no RANK in the environment: start the N ranks as a child
    torch.distributed.run (this process makes no GPU call, so nothing is initialized before the
    children exist) and relay rank 0's JSON line. Returns the children's exit code."""
    import subprocess
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
           '--master-addr=127.0.0.1', f'--master-port={free_port()}', script or os.path.abspath(__file__)] + argv
    log('self-launch:', ' '.join(cmd))
    p = subprocess.run(cmd, stdout=subprocess.PIPE, text=True)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
    if lines:
        sys.stdout.write(lines[-1] + '\n')
        sys.stdout.flush()
    return p.returncode if lines or p.returncode else 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=100)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--config', type=lambda x: int(x) if x.isdigit() else x, default=2,
                    choices=[2, 3, 4, 5, '5-T600'])
    ap.add_argument('--files-per-gpu', type=int, default=None)
    ap.add_argument('--threshold', type=float, default=98.0)
    ap.add_argument('--match-mode', choices=('auto', 'confidence', 'top1'), default='auto',
                    help='match configs: dice_batch_match_confidence (Dice#match + #confidence, 0 without a '
                         'match) or dice_batch_match (top1: also the top template of an unmatched file); auto: '
                         'confidence on the bound-pruned kernel (config 3), top1 elsewhere')
    ap.add_argument('--topk', type=int, default=3)
    ap.add_argument('--cpu-seconds', type=float, default=15.0, help='CPU-work budget of the baseline sample')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--extra-configs', default='3,4,5,5-T600',
                    help="configs also measured at N=1 (reported under extras.configs); '' for none")
    ap.add_argument('--extra-files-per-gpu', type=int, default=None,
                    help='files per GPU of the extra configs (default: each config\'s BASELINE size)')
    ap.add_argument('--probe', action='store_true', help='diagnostic: stream-read the tiles only (read ceiling)')
    ap.add_argument('--corpus', default='synthetic', choices=['synthetic', 'spdx'],
                    help="config 3's templates: synthetic, or the 94 real texts (47 choosealicense.com + 47 SPDX "
                         "license-list-XML) + synthetic ones")
    ap.add_argument('--shard-mode', choices=('auto', 'ranks', 'abi'), default='auto',
                    help="abi: also time the one-process multi-device entry point (dice_match_sharded_confidence, "
                         "host vs device gather, extras.abi_sharded) at world size 1; auto: that leg with the "
                         "extras at world size 1; ranks: never")
    ap.add_argument('--abi-contexts', type=int, default=0,
                    help='contexts of the abi leg (default: one per visible device)')
    ap.add_argument('--no-extras', action='store_true',
                    help='skip the separately reported host-side rates (PCIe end-to-end, host prep, single-file '
                         'calls): profiling runs then trace only the timed workload')
    args = ap.parse_args()

    if args.gpus > 1 and 'RANK' not in os.environ:
        sys.exit(self_launch(args.gpus, sys.argv[1:]))

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
    if distributed and world != args.gpus:
        raise SystemExit(f'bench.py: WORLD_SIZE={world} but --gpus {args.gpus}')
    group = Group()
    n_dev = torch.cuda.device_count()            # counts devices without initializing HIP
    if distributed:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        local_world = int(os.environ.get('LOCAL_WORLD_SIZE', str(world)))
        dev_index = local_rank % max(n_dev, 1)
        torch.cuda.set_device(dev_index)
        # RCCL needs one device per rank; ranks sharing a device (the one-GPU box rehearsing N > 1)
        # coordinate over gloo instead. Neither carries data-path traffic.
        backend = 'nccl' if n_dev >= local_world else 'gloo'
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', dev_index))
        else:
            dist.init_process_group('gloo')
        group = Group(rank, world, backend)
    else:
        local_world = 1
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()
    cpu = cpu_info()
    # host threads of one rank: every core for rank 0's timed CPU baseline; a 1/local_world share
    # for the other ranks' parity checks, which run together
    cpu['rank_threads'] = max(1, cpu['threads'] // local_world)
    nthreads = min(16, cpu['rank_threads'])      # generator / host-prep threads (box CPU share)

    cfg = args.config
    n_per = args.files_per_gpu or DEFAULT_FILES[cfg]
    run = Run(cfg, n_per, rank, world, dev, nthreads, args)
    matrix_mode = run.cfg == 5            # configs 5 and 5-T600: full matrix + top-k
    run_T_cfg3 = cfg in (3, '5-T600')     # config 3's template corpus
    stream = torch.cuda.Stream()          # a real (non-null) stream: kernels and HIP events share it
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream
    wall, launch_ms, achieved = timed(run, args.steps, args.warmup, stream, group)
    total_files = n_per * world
    exact_pairs = None
    if not args.probe:
        exact_pairs = n_per * run.T if matrix_mode else run.batch.scored_pairs(sptr)
        exact_pairs = int(group.reduce([exact_pairs], 'sum')[0])
    value = total_files * args.steps / wall
    traffic, traffic_src = traffic_for(cfg if cfg != '5-T600' else '5_T600', n_per, run.T, traffic_variant(cfg, run))
    batch, files, corpus, synth = run.batch, run.files, run.corpus, run.synth

    # ---- results: gathers (outside the timed region) -------------------------
    extras = {}
    if distributed:
        extras['process_group'] = {'backend': group.backend, 'world_size': dist.get_world_size(),
                                   'devices_visible': n_dev, 'ranks_per_device': -(-local_world // max(n_dev, 1))}
    best = ov = score = None
    if not matrix_mode:
        t_g = time.perf_counter()
        best, ov, score = batch.download_match(sptr)
        extras['host_gather_ms'] = (time.perf_counter() - t_g) * 1e3
        extras['matches'] = int(group.reduce([int((best >= 0).sum())], 'sum')[0])
        if distributed and world > 1:
            extras.update(gather_compare(batch, group, rank, world, n_per, best, ov, score, sptr))
    # ---- separately reported rates (never `value`): PCIe-inclusive end-to-end, host prep ----
    if rank == 0 and not matrix_mode and not args.probe and not args.no_extras:
        torch.cuda.synchronize()
        t_e = time.perf_counter()
        batch.upload(files, sptr)
        batch.match(args.threshold, sptr)
        batch.download_match(sptr)
        extras['e2e_pcie_files_per_s'] = n_per / (time.perf_counter() - t_e)
        # the same with the inputs in page-locked host memory (what a production caller stages
        # into): the H2D runs at the DMA rate instead of through the driver's bounce buffers
        from licensee_amd._native import FileBatch
        pin = lambda a: torch.from_numpy(a).pin_memory().numpy()
        pfw, pln, pcc = pin(files.wordset_size), pin(files.length), pin(files.cc_false_positive)
        pfiles = FileBatch(pin(files.bits), pfw, pln, pcc)
        torch.cuda.synchronize()
        t_e = time.perf_counter()
        batch.upload(pfiles, sptr)
        batch.match(args.threshold, sptr)
        batch.download_match(sptr)
        extras['e2e_pcie_pinned_files_per_s'] = n_per / (time.perf_counter() - t_e)
        del pfiles
        # the same files as pinned word-id lists (dice_batch_upload_ids: bitsets built on the
        # device), fewer bytes over the host link when the vocabulary is large
        from licensee_amd._native import bits_to_ids
        offs, ids = bits_to_ids(files.bits, corpus.n_vocab)
        offs, ids = pin(offs), pin(ids)
        extras['ids_bytes_per_file'] = round((ids.nbytes + offs.nbytes) / n_per, 1)
        extras['bitset_bytes_per_file'] = files.bits.shape[1] * 8
        torch.cuda.synchronize()
        t_e = time.perf_counter()
        batch.upload_ids(offs, ids, pfw, pln, pcc, sptr)
        batch.match(args.threshold, sptr)
        batch.download_match(sptr)
        extras['e2e_pcie_ids_pinned_files_per_s'] = n_per / (time.perf_counter() - t_e)
        del offs, ids
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
        # file contents as read from disk (bytes: project_file.rb:37-45 decodes them natively)
        big = [synth.text(i)[0].encode('utf-8') for i in range(16000)]
        hp.prep_files(big[:256], None, nthreads=nthreads)   # thread-local tables warm
        t_h = time.perf_counter()
        hp.prep_files(big, None, nthreads=nthreads)
        extras['host_prep_native_files_per_s'] = len(big) / (time.perf_counter() - t_h)
        # the host stage when the device scans the wordsets (lh_normalize_files: decode,
        # content_normalized, CC flag, Copyright), and the device scan itself (dice_batch_upload_text:
        # H2D of the texts + dice_words_kernel + status read-back + repack, wall time)
        hp.normalize_files(big[:256], None, nthreads=nthreads)
        t_h = time.perf_counter()
        norm = hp.normalize_files(big, None, nthreads=nthreads)
        extras['host_normalize_files_per_s'] = len(big) / (time.perf_counter() - t_h)
        if run.cfg == 2:
            run.scorer.vocab_setup(corpus.vocab, hp.nv_fields)
            wb = run.scorer.batch(len(big))
            text, off, tl, ln, ccf, _, _ = norm
            wb.upload_text(text, off, tl, ln, ccf)
            reps = []
            for _ in range(3):
                t_h = time.perf_counter()
                wb.upload_text(text, off, tl, ln, ccf)
                reps.append(time.perf_counter() - t_h)
            extras['device_wordset_files_per_s'] = len(big) / sorted(reps)[1]
            extras['device_wordset_note'] = (f'dice_batch_upload_text over the {len(big)} normalized texts '
                                             f'({len(text) / len(big) / 1024:.1f} KiB each): H2D from pageable '
                                             f'memory + the scan kernel + status read-back, median of 3 wall times')
            wb.close()
        # end to end on text: LicenseFile#license over byte strings through batch.BatchDetector's
        # two-stage pipeline (host threads prepare batch k + 1 while batch k is on the device:
        # upload, Exact, Dice#match + #confidence, download, Detection objects)
        if run.cfg == 2:   # (the vendored corpus: the texts above are config-2 files)
            from licensee_amd.batch import BatchDetector
            from licensee_amd.dice import DiceEngine
            chunks = [(big[i:i + 4000], None) for i in range(0, len(big), 4000)] * 2
            eng = DiceEngine(device=dev)
            for mode, key in (('device', 'end_to_end_text_files_per_s'),
                              ('host', 'end_to_end_text_host_wordset_files_per_s')):
                det = BatchDetector(eng, nthreads=nthreads, wordset_on=mode)
                for _ in det.detect_stream(chunks[:2]):   # both page-locked text buffers allocated
                    pass
                rates = []
                for _ in range(3):   # (one stream is ~60 ms: the median of 3)
                    t_h = time.perf_counter()
                    n_det = sum(len(d) for d in det.detect_stream(chunks))
                    rates.append(n_det / (time.perf_counter() - t_h))
                extras[key] = sorted(rates)[1]
                extras[key.replace('_files_per_s', '_runs')] = [round(r) for r in rates]
                # the two stages alone, per 4000-file batch (the stream's bound is the slower one)
                t_h = time.perf_counter()
                prepped = [det._prep(*c) for c in chunks[:2]]
                t_m = time.perf_counter()
                for p in prepped:
                    det._score(p, args.threshold)
                extras[key.replace('_files_per_s', '_stage_ms')] = {
                    'host': (t_m - t_h) / 2 * 1e3, 'device': (time.perf_counter() - t_m) / 2 * 1e3}
                det.close()
            extras['end_to_end_text_note'] = (f'batch.BatchDetector.detect_stream: {len(chunks)} batches of 4000 of '
                                              f'the texts above (median of 3 streams), the host stage ({nthreads} threads) of batch k + 1 '
                                              f'overlapping batch k on the GPU; wordset_on=device: host '
                                              f'content_normalized, the GPU scans the wordsets '
                                              f'(dice_batch_upload_text) and runs Exact and Dice#match + '
                                              f'#confidence; host_wordset: the host scans and interns too')
            eng.scorer.close()
        extras['host_prep_note'] = (f'normalize+intern+Copyright/Exact of synthetic texts: Python 1 thread; '
                                    f'native (csrc/normalize.cpp) {nthreads} threads on 16000 byte strings '
                                    f'(avg {sum(map(len, big)) / len(big) / 1024:.1f} KiB)')

    if rank == 0 and not matrix_mode and not args.probe and not args.no_extras:
        torch.cuda.synchronize()
        extras['single_file_us'] = single_file_latency(run)
        # Exact#match on the device over the resident batch (dice_batch_exact; the synthetic files
        # hold no template field words: all-zero field masks)
        from licensee_amd.batch import exact_tables
        from licensee_amd.native_host import HostPrep
        run.scorer.exact_setup(*exact_tables(corpus, HostPrep(corpus)))
        batch.upload(files, sptr)
        fm = np.zeros(n_per, np.uint64)
        batch.exact(fm, sptr)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(20):
            batch.exact(None, sptr)
        e1.record(stream)
        torch.cuda.synchronize()
        ex = batch.download_exact(sptr)
        extras['exact_kernel'] = {'launch_us': e0.elapsed_time(e1) / 20 * 1e3, 'files': n_per,
                                  'exact_matches': int((ex >= 0).sum()),
                                  'note': 'dice_batch_exact over the resident batch (kernel only, no field-mask '
                                          'upload): Exact#match for every file beside the Dice pass'}

    if world == 1 and not matrix_mode and not args.probe and (
            args.shard_mode == 'abi' or (args.shard_mode == 'auto' and not args.no_extras)):
        torch.cuda.synchronize()
        extras['abi_sharded'] = abi_sharded_leg(run, args, n_dev)
        log(f"abi sharded: {extras['abi_sharded']}")

    cpu_baseline = None
    parity = None
    if not args.no_cpu_baseline:
        from oracle.native import bits_to_csr
        orc = oracle_for(corpus)
        # rank 0 calibrates on a small slice and sizes the sample to ~cpu_seconds of CPU work;
        # every rank then checks that many files of its own shard
        sample = 0
        if rank == 0:
            cal = min(n_per, 4000)
            csr = bits_to_csr(files.bits[:cal], corpus.n_vocab)
            tc = time.perf_counter()
            orc.match(files.bits[:cal], files.wordset_size[:cal], files.length[:cal], files.cc_false_positive[:cal],
                      args.threshold, nthreads=1, mode=0, csr=csr)
            per_file = (time.perf_counter() - tc) / cal
            sample = int(min(n_per, max(cal, args.cpu_seconds / max(per_file, 1e-9))))
        sample = group.bcast(sample)
        sl = slice(0, sample)
        baseline = {}

        def check():
            threads = cpu['threads'] if rank == 0 else cpu['rank_threads']
            csr = bits_to_csr(files.bits[sl], corpus.n_vocab)
            tc = time.perf_counter()
            cb, co, cs = orc.match(files.bits[sl], files.wordset_size[sl], files.length[sl],
                                   files.cc_false_positive[sl], args.threshold, nthreads=threads, mode=0, csr=csr)
            baseline['hash_s'] = time.perf_counter() - tc
            if rank == 0:
                tc = time.perf_counter()
                orc.match(files.bits[sl], files.wordset_size[sl], files.length[sl], files.cc_false_positive[sl],
                          args.threshold, nthreads=threads, mode=1)
                baseline['bits_s'] = time.perf_counter() - tc
            if not matrix_mode:
                mism = int(np.sum(best[sl] != cb) + np.sum(ov[sl] != co) + np.sum(score[sl] != cs))
                return {'checked_files': sample, 'mismatches': mism, 'oracle': 'oracle/dice_ref.c (hash Set#&)'}
            res = parity_sample(run, orc, sptr, threads, sample)
            res.pop('oracle_files_per_s', None)
            return res

        parity = staged_parity(group, check)
        if rank == 0:
            cpu_baseline = {'value': sample / baseline['hash_s'], 'unit': 'files/s', 'cores': cpu['threads'],
                            'kind': 'port',
                            'sample': f"first {sample} files of rank 0's shard of the same synthetic workload, "
                                      f"hash-set Set#& restatement (oracle/dice_ref.c), {cpu['threads']} threads",
                            'bitset_variant_files_per_s': sample / baseline['bits_s'],
                            'nproc': cpu['nproc'], 'affinity_cpus': cpu['affinity_cpus'],
                            'cgroup_cpu_quota': cpu['cgroup_cpu_quota'], 'cpu_model': cpu['cpu_model']}

    head = {'templates': run.T, 'vocab': run.V, 'kernel': KERNELS[run.match_kernel], 'program_entries': run.entries,
            'algorithmic_bytes_per_file': run.algo_bytes_per_file}
    # ---- the other BASELINE configs, same run (every rank, its own shard) ------------------
    if not args.probe and args.extra_configs:
        run.close()
        run = None
        extras['configs'] = {}
        for c in [int(x) if x.strip().isdigit() else x.strip() for x in args.extra_configs.split(',') if x.strip()]:
            if c == cfg:
                continue
            r = Run(c, args.extra_files_per_gpu or DEFAULT_FILES[c], rank, world, dev, nthreads, args)
            variants = [(str(c), None)]
            if c == 3 and r.match_kernel == 4:
                variants += [('3-top1', 'top1'), ('3-allpairs', {'DICE_POST_PRUNE': '0'})]
            conf = r.confidence
            for tag, env in variants:
                r.confidence = conf and env is None
                saved = r.rescore(env, dev) if isinstance(env, dict) else None
                extras['configs'][tag] = measure_extra(r, c, args, stream, sptr, cpu, group)
                if saved:
                    r.restore(saved)
            r.close()

    if rank == 0:
        line = {
            'metric': METRIC, 'value': value, 'unit': 'files/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': wall / args.steps * 1e3, 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None, 'dtype': 'u32',
            'data': 'synthetic (normalized-space perturbations of the vendored templates, filler words from '
                    'the reference spec/fixtures/ipsum.txt, seed 20250202)',
            'config': {'workload': WORKLOADS[cfg] + (' (templates: 94 real texts incl. SPDX + synthetic)'
                                                     if args.corpus == 'spdx' and run_T_cfg3 else ''),
                       'files_per_gpu': n_per, 'global_files': total_files,
                       'templates': head['templates'], 'vocab': head['vocab'], 'kernel': head['kernel'],
                       'program_entries': head['program_entries'], 'parallelism': f'shard{world}'},
            'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic,
                         'traffic_source': traffic_src,
                         'algorithmic_bytes_per_file': head['algorithmic_bytes_per_file'], 'launch_ms': launch_ms,
                         **({'note': 'config 3 is latency/issue-bound, not HBM-bound; frac is its HBM share '
                                     'only (DESIGN.md 4b)'} if cfg == 3 else {}),
                         **({'per_rank_note': 'achieved = one rank\'s bytes / the slowest rank\'s launch time '
                                              '(per-GPU roofline; every rank runs the same shard size)'}
                            if world > 1 else {})},
            'cpu_baseline': cpu_baseline,
            'decided_pairs_per_s': value * head['templates'],
            'exact_scored_pairs_per_s': exact_pairs * args.steps / wall if exact_pairs is not None else None,
            'parity': parity,
            'extras': extras,
        }
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(line) + '\n').encode())
    if run is not None:
        run.close()
    if distributed:
        group.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
