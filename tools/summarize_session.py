"""Summarize one tools/gpu_measure.sh session into profiles/ (tracked):

    python tools/summarize_session.py <tag>

Reads gpurun_out/<tag>_bench.json (the default bench line) and gpurun_out/prof_<tag>_same/
(rocprofv3 --kernel-trace --stats of the same primary workload and step count, same lease) and
writes profiles/<tag>_bench.json plus profiles/<tag>_session.md: the trace's product-kernel
average beside the bench's launch_ms / ms_per_step, and roofline.frac recomputed from the
profile's average, so the bench line's numbers follow from profiles/.
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PREFIXES = ('dice_prog_', 'dice_dense_', 'dice_lds_', 'dice_post_', 'dice_prune', 'dice_defer_', 'dice_confidence')


def base(name):
    return name.split('(')[0].replace('void ', '').replace('dice::', '')


def main():
    tag = sys.argv[1]
    out = os.path.join(ROOT, 'gpurun_out')
    bench = json.loads(open(os.path.join(out, f'{tag}_bench.json')).read().strip().splitlines()[-1])
    same_dir = os.path.join(out, f'prof_{tag}_same')
    same = json.loads(open(os.path.join(same_dir, 'bench.json')).read().strip().splitlines()[-1])
    stats = list(csv.DictReader(open(os.path.join(same_dir, 'trace', 'run_kernel_stats.csv'))))
    product = [r for r in stats if base(r['Name']).startswith(PREFIXES)]
    calls = max(int(r['Calls']) for r in product)
    step = [r for r in product if int(r['Calls']) == calls]
    avg_ns = sum(float(r['AverageNs']) for r in step)
    files = bench['config']['files_per_gpu']
    alg = bench['roofline']['algorithmic_bytes_per_file']
    frac = alg * files / (avg_ns * 1e-9) / 1e9 / bench['roofline']['peak']
    os.makedirs(os.path.join(ROOT, 'profiles'), exist_ok=True)
    with open(os.path.join(ROOT, 'profiles', f'{tag}_bench.json'), 'w') as fh:
        fh.write(json.dumps(bench) + '\n')
    with open(os.path.join(ROOT, 'profiles', f'{tag}_session.md'), 'w') as fh:
        fh.write(f'# Session {tag}: bench line + same-lease rocprofv3 trace\n\n')
        fh.write('Commands (one gpurun call, `tools/gpu_measure.sh {0}`):\n\n'
                 '1. `python bench.py` -> `profiles/{0}_bench.json`\n'
                 '2. `rocprofv3 --kernel-trace --stats -- python bench.py --extra-configs= --no-cpu-baseline` '
                 '(same primary workload and step count)\n\n'.format(tag))
        fh.write('| | value |\n|---|---|\n')
        fh.write(f"| bench `value` | {bench['value']:.4g} {bench['unit']} |\n")
        fh.write(f"| bench `ms_per_step` | {bench['ms_per_step'] * 1e3:.2f} us |\n")
        fh.write(f"| bench `roofline.launch_ms` (HIP events, kernel stream) | {bench['roofline']['launch_ms'] * 1e3:.2f} us |\n")
        fh.write(f"| bench `roofline.frac` | {bench['roofline']['frac']:.3f} |\n")
        fh.write(f"| traced bench `ms_per_step` (under rocprofv3) | {same['ms_per_step'] * 1e3:.2f} us |\n")
        fh.write(f"| rocprofv3 average of the step's product kernel(s) `{' + '.join(base(r['Name']) for r in step)}` "
                 f"| {avg_ns / 1e3:.2f} us ({calls} calls) |\n")
        fh.write(f"| frac recomputed from the rocprof average ({alg} B/file x {files} files) | {frac:.3f} |\n")
        fh.write(f"| rocprof average <= traced ms_per_step | {avg_ns * 1e-6 <= same['ms_per_step']} |\n\n")
        fh.write('## Kernel trace stats\n\n| kernel | calls | avg ns | min ns | max ns | % |\n|---|---|---|---|---|---|\n')
        for r in stats:
            fh.write(f"| {r['Name'][:70]} | {r['Calls']} | {float(r['AverageNs']):.0f} | {r['MinNs']} | {r['MaxNs']} | "
                     f"{float(r['Percentage']):.1f} |\n")
        ex = bench.get('extras', {}).get('configs', {})
        if ex:
            fh.write('\n## Extra configs measured in the same bench run (`extras.configs`)\n\n'
                     '| config | kernel | launch | files/s | roofline frac | parity |\n|---|---|---|---|---|---|\n')
            for c, e in sorted(ex.items()):
                p = e.get('parity') or {}
                fh.write(f"| {c} | {e.get('kernel')} | {e['launch_ms'] * 1e3:.1f} us | {e['files_per_s']:.3g} | "
                         f"{e['roofline_frac']:.3f} | {p.get('mismatches')} mismatches / {p.get('checked_files')} |\n")
        hp = bench.get('extras', {})
        if 'host_prep_native_files_per_s' in hp:
            fh.write(f"\nHost prep (native, {hp.get('host_prep_note', '')}): "
                     f"{hp['host_prep_native_files_per_s']:.3g} files/s; Python: {hp['host_prep_python_files_per_s']:.3g} files/s\n")
        rates = [('host stage with the device wordset scan (lh_normalize_files)', 'host_normalize_files_per_s'),
                 ('device wordset scan (dice_batch_upload_text, H2D included)', 'device_wordset_files_per_s'),
                 ('end to end, BatchDetector.detect_stream, wordset on the device', 'end_to_end_text_files_per_s'),
                 ('end to end, wordset on the host', 'end_to_end_text_host_wordset_files_per_s')]
        if any(k in hp for _, k in rates):
            fh.write('\n| real-text rate (16 host threads) | files/s |\n|---|---|\n')
            for name, k in rates:
                if k in hp:
                    fh.write(f'| {name} | {hp[k]:.3g} |\n')
    print(f'{tag}: bench launch {bench["roofline"]["launch_ms"] * 1e3:.2f} us, rocprof {avg_ns / 1e3:.2f} us, '
          f'traced step {same["ms_per_step"] * 1e3:.2f} us, frac(rocprof) {frac:.3f}')


if __name__ == '__main__':
    main()
