"""Kernel statistics from a rocprofv3 SQLite output (ROCm 7's default rocpd format).

    python tools/rocpd_summary.py DB [--seq N] [--match SUBSTR] [--md]

Prints per kernel: dispatches, average / min / max / total duration (us), grid and VGPRs,
sorted by total time; --seq N also lists the last N dispatches in time order (to attribute a
launch sequence such as pruned kernel -> dense -> narrow); --md prints a markdown table.
"""
import argparse
import glob
import os
import re
import sqlite3


def short(name):
    name = re.sub(r'\(.*', '', name)
    return name if len(name) < 90 else name[:87] + '...'


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('db')
    ap.add_argument('--seq', type=int, default=0)
    ap.add_argument('--match', default='')
    ap.add_argument('--md', action='store_true')
    a = ap.parse_args()
    path = a.db
    if os.path.isdir(path):
        path = sorted(glob.glob(os.path.join(path, '**', '*.db'), recursive=True))[-1]
    cur = sqlite3.connect(path).cursor()
    rows = cur.execute('select name, duration, grid_x, workgroup_x, vgpr_count, sgpr_count, lds_size, start '
                       'from kernels order by start').fetchall()
    rows = [r for r in rows if a.match in r[0]]
    stats = {}
    for name, dur, gx, wx, vg, sg, lds, st in rows:
        s = stats.setdefault(short(name), {'n': 0, 'tot': 0, 'min': 1e30, 'max': 0, 'grid': gx // max(wx, 1),
                                           'wg': wx, 'vgpr': vg, 'lds': lds})
        s['n'] += 1
        s['tot'] += dur
        s['min'] = min(s['min'], dur)
        s['max'] = max(s['max'], dur)
    order = sorted(stats.items(), key=lambda kv: -kv[1]['tot'])
    if a.md:
        print('| kernel | calls | avg us | min us | max us | total us | workgroups x size | VGPRs | LDS B |')
        print('|---|---|---|---|---|---|---|---|---|')
    for k, s in order:
        avg = s['tot'] / s['n'] / 1e3
        if a.md:
            print(f"| `{k}` | {s['n']} | {avg:.2f} | {s['min'] / 1e3:.2f} | {s['max'] / 1e3:.2f} | {s['tot'] / 1e3:.1f} | "
                  f"{s['grid']} x {s['wg']} | {s['vgpr']} | {s['lds']} |")
        else:
            print(f"{s['n']:6d} avg {avg:10.2f} us  min {s['min'] / 1e3:10.2f}  max {s['max'] / 1e3:10.2f}  "
                  f"tot {s['tot'] / 1e3:12.1f}  grid {s['grid']}x{s['wg']} vgpr {s['vgpr']}  {k}")
    if a.seq:
        print('--- last dispatches ---')
        for name, dur, gx, wx, vg, sg, lds, st in rows[-a.seq:]:
            print(f'{dur / 1e3:10.2f} us  grid {gx // max(wx, 1)}x{wx}  {short(name)}')


if __name__ == '__main__':
    main()
