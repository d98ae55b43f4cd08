"""Summarise `hipcc -Rpass-analysis=kernel-resource-usage` for one HIP source: per kernel
(demangled, shortened) VGPRs, SGPRs, SGPR/VGPR spills, scratch and occupancy.

    python tools/kernel_resources.py licensee_amd/csrc/dice_prune.hip [name-filter]
"""
import os
import re
import subprocess
import sys
import tempfile


def kernel_resources(src, extra_flags=()):
    """[{name, VGPRs, TotalSGPRs, SGPRs Spill, VGPRs Spill, ScratchSize [bytes/lane], Occupancy ...}] per kernel."""
    with tempfile.TemporaryDirectory() as d:
        out = subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-c', '-o',
                              os.path.join(d, 'kr.o'), src, '-Rpass-analysis=kernel-resource-usage', *extra_flags],
                             capture_output=True, text=True).stderr
    cur = None
    rows = []
    for line in out.splitlines():
        m = re.search(r'remark:\s+(.*?)\s*\[-Rpass', line)
        if not m:
            continue
        txt = m.group(1)
        if txt.startswith('Function Name:'):
            name = txt.split(':', 1)[1].strip()
            try:
                name = subprocess.run(['c++filt', name], capture_output=True, text=True).stdout.strip()
            except OSError:
                pass
            cur = {'name': re.sub(r'\(.*', '', name)}
            rows.append(cur)
        elif cur is not None and ':' in txt:
            k, v = txt.split(':', 1)
            cur[k.strip()] = v.strip()
    return rows


def main():
    src = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ''
    for r in kernel_resources(src):
        if filt in r['name']:
            print(f"{r['name'][:70]:70s} V={r.get('VGPRs')} S={r.get('TotalSGPRs')} Sspill={r.get('SGPRs Spill')} "
                  f"Vspill={r.get('VGPRs Spill')} scratch={r.get('ScratchSize [bytes/lane]')} occ={r.get('Occupancy [waves/SIMD]')}")


if __name__ == '__main__':
    main()
