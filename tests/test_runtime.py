"""One HIP runtime per process: liblicensee_dice.so loaded before torch.

The library needs libamdhip64.so.7 by soname; torch ships its own copy of that runtime. The
loader (licensee_amd._native) maps torch's copy first, so the library and torch share one
runtime whatever the import order; a host that maps a second copy anyway gets a clear
dice_create error naming both files (licensee_amd/csrc/dice.hip check_hip_runtime) instead of
a torch that later finds no GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_worker(mode):
    env = dict(os.environ)
    env.pop('LICENSEE_DICE_HIP_RUNTIME', None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'tests', 'runtime_worker.py'), mode],
                       capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-4000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


def test_library_first_shares_torchs_runtime():
    out = run_worker('shared')
    assert len(out['runtimes']) == 1, out
    if not out['torch_gpu']:
        assert out['create'].startswith('dice error -2') and 'reports no device' in out['create']


def test_second_runtime_is_refused_loudly():
    out = run_worker('second')
    assert len(out['runtimes']) == 2, out
    assert 'two HIP runtimes are mapped' in out['create'], out
    named = out['create'].split('(', 1)[1].split(')', 1)[0].split(', ')
    assert sorted(os.path.realpath(p) for p in named) == sorted(os.path.realpath(p) for p in out['runtimes'])


@pytest.mark.gpu
def test_library_first_then_torch_streams_on_gpu():
    """The library loads first, then torch: torch still sees the GPU, the library scores on a
    torch stream, results equal the oracle's."""
    out = run_worker('shared')
    assert out['torch_gpu'] and out['create'] == 'ok', out
    assert out['mismatches'] == 0 and out['torch_sum'] == 45.0, out
