"""Where a kernel's scratch spills sit: per scratch_load/store, the loop depth of its basic block
(from the compiler's `; in Loop: ... Depth=N` block comments), for one kernel of a HIP source.

    python tools/isa_spills.py licensee_amd/csrc/dice_prune.hip <mangled-name-prefix>
"""
import os
import re
import subprocess
import sys
import tempfile


def main():
    src, prefix = sys.argv[1], sys.argv[2]
    d = tempfile.mkdtemp()
    subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-c', '-save-temps',
                    '-o', os.path.join(d, 'x.o'), os.path.abspath(src)], cwd=d, capture_output=True)
    asm = [f for f in os.listdir(d) if f.endswith('gfx950.s')][0]
    s = open(os.path.join(d, asm)).read()
    name = re.search(r'^(' + re.escape(prefix) + r'[^:\s]*):', s, re.M).group(1)
    i = s.index(name + ':')
    body = s[i:s.index('.Lfunc_end', i)].split('\n')
    depth = 0
    out = {}
    for line in body:
        m = re.search(r'Depth=(\d+)', line)
        if re.match(r'^(\.LBB|; %bb)', line):
            depth = int(m.group(1)) if m else 0
        elif m and line.strip().startswith(';'):
            depth = int(m.group(1))
        if 'scratch_' in line:
            kind = 'load' if 'load' in line else 'store'
            out.setdefault((depth, kind), 0)
            out[(depth, kind)] += 1
    print(name[:80], {f'depth{k[0]}_{k[1]}': v for k, v in sorted(out.items())})


if __name__ == '__main__':
    main()
