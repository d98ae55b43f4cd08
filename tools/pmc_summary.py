"""Average PMC counters per kernel launch from tools/pmc_kernel.sh output.
    python tools/pmc_summary.py gpurun_out/pmc_<tag> <kernel-name-substring> [files_per_launch]"""
import collections
import csv
import glob
import sys

src, kname = sys.argv[1], sys.argv[2]
files = int(sys.argv[3]) if len(sys.argv) > 3 else 0
agg = collections.defaultdict(list)
for f in glob.glob(src + '/**/run_counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if kname in r['Kernel_Name']:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
for k in sorted(agg):
    v = sum(agg[k]) / len(agg[k])
    print(f'{k:28s} {v:16.4g}' + (f'   per file {v / files:10.1f}' if files else ''))
