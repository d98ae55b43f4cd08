"""The C-ABI library (no GPU needed): it loads, exports every function include/*.h declares,
and its device-free entry points and argument checks behave."""
import ctypes
import os
import re

import numpy as np
import pytest

from licensee_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions(header, prefix):
    src = open(os.path.join(ROOT, 'include', header)).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return set(re.findall(r'\b(' + prefix + r'[a-z0-9_]+)\s*\(', src))


def test_library_exports_every_declared_symbol():
    lib = _native.load_library()
    declared = declared_functions('licensee_dice.h', 'dice_')
    assert len(declared) >= 18
    for name in sorted(declared):
        assert hasattr(lib, name), name
    assert set(_native.EXPORTED_SYMBOLS) == declared


def test_host_library_exports_every_declared_symbol():
    from licensee_amd import native_host
    lib = native_host._load()
    declared = declared_functions('licensee_host.h', 'lh_')
    assert declared == {'lh_create', 'lh_destroy', 'lh_set_templates', 'lh_normalize', 'lh_prep_files'}
    for name in sorted(declared):
        assert hasattr(lib, name), name
    assert set(os.listdir(os.path.join(ROOT, 'include'))) == {'licensee_dice.h', 'licensee_host.h'}


def test_words64():
    lib = _native.load_library()
    assert [lib.dice_words64(v) for v in (0, 1, 64, 65, 3551)] == [0, 1, 1, 2, 56]


def test_create_rejects_bad_arguments():
    lib = _native.load_library()
    ctx = ctypes.c_void_p()
    assert lib.dice_create(None, 0, ctypes.byref(ctx)) == -1
    assert b'invalid' in lib.dice_last_error()
    t = _native._Templates(0, 0, None, None, None, None, None, None)
    assert lib.dice_create(ctypes.byref(t), 0, ctypes.byref(ctx)) == -1


def test_no_cpu_fallback_without_gpu():
    """On a machine without a gfx950 device the product fails loudly (DICE_E_DEVICE)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.license import License
    c = TemplateCorpus(License.all(hidden=True, pseudo=False)[:3])
    with pytest.raises(_native.DiceError, match='dice error -2'):
        _native.Scorer(c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc, c.n_vocab)


def test_program_source_and_precompile_without_device():
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.license import License
    lib = _native.load_library()
    c = TemplateCorpus(License.all(hidden=True, pseudo=False))
    keep = [c.lf_bits, c.lf_size, c.fields_set_size, c.length_slack, c.length, c.is_cc]
    t = _native._Templates(len(c.lf_size), c.n_vocab, *[k.ctypes.data for k in keep])
    n = lib.dice_program_source(ctypes.byref(t), None, 0)
    buf = ctypes.create_string_buffer(n + 1)
    assert lib.dice_program_source(ctypes.byref(t), buf, n + 1) == n
    src = buf.value.decode()
    assert 'dice_prog_match' in src and 'dice_prog_matrix4' in src and 'dice_prog_matrix16' in src
    entries = int(np.count_nonzero(c.lf_bits.view(np.uint32)))
    assert f'entries={entries}' in src
    path = ctypes.create_string_buffer(1024)
    assert lib.dice_precompile(ctypes.byref(t), path, 1024) == 0
    assert os.path.exists(path.value.decode())
