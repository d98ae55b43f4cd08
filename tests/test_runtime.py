"""One HIP runtime per process: liblicensee_dice.so loaded before torch.

The library needs libamdhip64.so.7 by soname; torch ships its own copy of that runtime. The
loader (licensee_amd._native) maps torch's copy first, so the library and torch share one
runtime whatever the import order; a host that maps a second copy anyway gets a clear
dice_create error naming both files (licensee_amd/csrc/dice.hip check_hip_runtime) instead of
a torch that later finds no GPU."""
import importlib.util
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
needs_torch = pytest.mark.skipif(importlib.util.find_spec('torch') is None, reason='the worker imports torch')


def run_worker(mode, runtime=None):
    env = dict(os.environ)
    env.pop('LICENSEE_DICE_HIP_RUNTIME', None)
    if runtime is not None:
        env['LICENSEE_DICE_HIP_RUNTIME'] = runtime
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'tests', 'runtime_worker.py'), mode],
                       capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-4000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


def stub_runtime(tmp_path, soname):
    """An empty shared object named libamdhip64.so with the given DT_SONAME."""
    src = tmp_path / 'stub.c'
    src.write_text('int licensee_stub_runtime(void) { return 0; }\n')
    out = tmp_path / soname / 'libamdhip64.so'
    out.parent.mkdir()
    subprocess.run(['gcc', '-shared', '-fPIC', f'-Wl,-soname,{soname}', '-o', str(out), str(src)], check=True)
    return str(out)


def test_elf_dynamic_reads_sonames():
    from licensee_amd import _native
    assert _native.needed_hip_soname(_native.LIB_PATH) == 'libamdhip64.so.7'
    soname, needed = _native.elf_dynamic(_native.LIB_PATH)
    assert 'libamdhip64.so.7' in needed and 'libc.so.6' in needed
    assert _native.elf_dynamic(__file__) == (None, ())


def test_preload_only_a_runtime_with_the_needed_soname(tmp_path, monkeypatch):
    """a torch built for another ROCm major ships libamdhip64.so with soname .so.6; the
    library would never bind to it, so the loader must not map it (dice_create would then see two
    runtimes and refuse a process that works without the preload)."""
    from licensee_amd import _native
    old, same = stub_runtime(tmp_path, 'libamdhip64.so.6'), stub_runtime(tmp_path, 'libamdhip64.so.7')
    monkeypatch.setenv('LICENSEE_DICE_HIP_RUNTIME', old)
    p, why = _native.preload_decision()
    assert p is None and 'not preloaded' in why and 'libamdhip64.so.6' in why
    monkeypatch.setenv('LICENSEE_DICE_HIP_RUNTIME', same)
    assert _native.preload_decision()[0] == same
    monkeypatch.setenv('LICENSEE_DICE_HIP_RUNTIME', '')
    assert _native.preload_decision()[0] is None


def test_mismatched_runtime_is_skipped_in_a_process(tmp_path):
    out = run_worker('stub', stub_runtime(tmp_path, 'libamdhip64.so.6'))
    assert 'not preloaded' in out['decision'], out
    assert len(out['runtimes']) == 1 and 'so.6' not in out['runtimes'][0], out
    assert 'two HIP runtimes' not in out['create'], out


@pytest.mark.gpu
def test_mismatched_runtime_skipped_create_works_on_gpu(tmp_path):
    out = run_worker('stub', stub_runtime(tmp_path, 'libamdhip64.so.6'))
    assert out['create'] == 'ok', out


@needs_torch
def test_library_first_shares_torchs_runtime():
    out = run_worker('shared')
    assert len(out['runtimes']) == 1, out
    if not out['torch_gpu']:
        assert out['create'].startswith('dice error -2') and 'reports no device' in out['create']


@needs_torch
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
