"""Summarize a tools/profile_round.sh output directory into profiles/<tag>.md + pmc json.

    python tools/summarize_profile.py gpurun_out/prof_<tag> <tag> <config> <files_per_launch> <templates>
"""
import collections
import csv
import json
import os
import sys


def load_counters(path, kernel):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if kernel in r['Kernel_Name']:
            d[r['Counter_Name']].append(float(r['Counter_Value']))
    return {k: sum(v) / len(v) for k, v in d.items()}


def main():
    src, tag, config, files, templates = sys.argv[1], sys.argv[2], sys.argv[3].replace('-', '_'), int(sys.argv[4]), int(sys.argv[5])
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    stats = list(csv.DictReader(open(os.path.join(src, 'trace', 'run_kernel_stats.csv'))))
    # the product kernels of the timed region (copies/packing outside it are listed, not chosen):
    # the sparse program / dense / LDS kernels run one launch per step, the postings path two
    # (dice_post_dense + dice_post_narrow_*): a step's time and traffic sum over them
    prefixes = ('dice_prog_', 'dice_dense_', 'dice_lds_', 'dice_post_', 'dice_prune', 'dice_defer_', 'dice_confidence')
    def base(r):
        return r['Name'].split('(')[0].replace('void ', '').replace('dice::', '')
    product = [r for r in stats if base(r).startswith(prefixes)]
    if not product:
        product = [max(stats, key=lambda r: float(r['TotalDurationNs']))]
    top_calls = max(int(r['Calls']) for r in product)
    product = [r for r in product if int(r['Calls']) == top_calls]
    kernels = [r['Name'].split('(')[0].replace('void ', '') for r in product]
    kernel = ' + '.join(kernels)
    avg_ns = sum(float(r['AverageNs']) for r in product)
    def summed(path):
        out = collections.Counter()
        for k in kernels:
            for name, v in load_counters(path, k).items():
                out[name] += v
        return dict(out)
    fetch = summed(os.path.join(src, 'fetch', 'run_counter_collection.csv'))
    write = summed(os.path.join(src, 'write', 'run_counter_collection.csv'))
    sq = summed(os.path.join(src, 'sq', 'run_counter_collection.csv'))
    clk = summed(os.path.join(src, 'clk', 'run_counter_collection.csv'))
    # gfx950: FETCH_SIZE (KB) counts half the bytes of wide coalesced streaming reads -> x2
    # (MI355X_MICROARCH.md §HBM); WRITE_SIZE (KB) is exact for streaming stores.
    read_b = fetch.get('FETCH_SIZE', 0) * 1024 * 2
    write_b = write.get('WRITE_SIZE', 0) * 1024
    hbm = read_b + write_b
    eff_clk = clk.get('GRBM_GUI_ACTIVE', 0) / 8 / (avg_ns * 1e-9) / 1e9 if avg_ns else 0
    pmc = {'tag': tag, 'config': config, 'kernel': kernel, 'files_per_launch': files, 'templates': templates,
           'avg_kernel_ns': avg_ns, 'per_kernel_avg_ns': {k: float(r['AverageNs']) for k, r in zip(kernels, product)},
           'hbm_bytes_per_launch': hbm, 'read_bytes': read_b, 'write_bytes': write_b,
           'hbm_gbs': hbm / (avg_ns * 1e-9) / 1e9, 'effective_clock_ghz': eff_clk, 'sq': sq,
           'valu_busy_frac': sq.get('SQ_INSTS_VALU', 0) * 2 / 1024 / (clk.get('GRBM_GUI_ACTIVE', 1) / 8)}
    os.makedirs(os.path.join(root, 'profiles'), exist_ok=True)
    with open(os.path.join(root, 'profiles', f'pmc_config{config}.json'), 'w') as fh:
        json.dump(pmc, fh, indent=1)
    with open(os.path.join(root, 'profiles', f'{tag}.md'), 'w') as fh:
        fh.write(f'# rocprofv3 summary: {tag}\n\nCommand: `tools/profile_round.sh {tag}` '
                 f'(bench.py --config {config}, {files} files x {templates} templates per launch)\n\n')
        fh.write('## Kernel trace stats (`rocprofv3 --kernel-trace --stats`)\n\n| kernel | calls | avg ns | min ns | max ns | % |\n|---|---|---|---|---|---|\n')
        for r in stats:
            fh.write(f"| {r['Name'][:60]} | {r['Calls']} | {float(r['AverageNs']):.0f} | {r['MinNs']} | {r['MaxNs']} | {float(r['Percentage']):.1f} |\n")
        fh.write(f'\n## PMC (separate passes) for `{kernel}`, per step (summed over these kernels)\n\n')
        fh.write(f'- FETCH_SIZE {fetch.get("FETCH_SIZE", 0):.0f} KB (x2 gfx950 correction) -> read {read_b / 1e6:.1f} MB\n')
        fh.write(f'- WRITE_SIZE {write.get("WRITE_SIZE", 0):.0f} KB -> write {write_b / 1e6:.1f} MB\n')
        fh.write(f'- HBM traffic {hbm / 1e6:.1f} MB per launch = {pmc["hbm_gbs"]:.0f} GB/s at the kernel average\n')
        fh.write(f'- effective clock {eff_clk:.2f} GHz (GRBM_GUI_ACTIVE / 8 / kernel time)\n')
        fh.write(f'- VALU busy ~{pmc["valu_busy_frac"] * 100:.0f}% (SQ_INSTS_VALU x 2 cycles / 1024 SIMDs / cycles)\n')
        for k, v in sorted(sq.items()):
            fh.write(f'- {k} {v:.0f}\n')
    print(json.dumps(pmc))


if __name__ == '__main__':
    main()
