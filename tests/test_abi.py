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
    assert declared == {'lh_create', 'lh_destroy', 'lh_set_templates', 'lh_set_unicode', 'lh_normalize', 'lh_prep_files',
                        'lh_vocab_pack', 'lh_template_field_masks', 'lh_normalize_files'}
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


def test_device_wordset_calls_reject_bad_arguments():
    lib = _native.load_library()
    assert lib.dice_vocab_setup(None, 0, None, 0, None) == -1
    assert lib.dice_batch_upload_text(None, 0, None, 0, None, None, None, None, None, None, None) == -1
    assert lib.dice_batch_set_rows(None, 0, None, None, None, None, None) == -1
    assert lib.dice_batch_download_rows(None, None, None, None, None) == -1
    assert b'NULL' in lib.dice_last_error()


def test_sharded_calls_reject_bad_arguments():
    lib = _native.load_library()
    f = _native._Files(0, None, None, None, None)
    assert lib.dice_match_sharded(None, 1, ctypes.byref(f), 98.0, 0, None, None, None) == -1
    ctxs = (ctypes.c_void_p * 1)(None)
    assert lib.dice_match_sharded(ctxs, 0, ctypes.byref(f), 98.0, 0, None, None, None) == -1
    assert lib.dice_match_sharded(ctxs, 1, ctypes.byref(f), 98.0, 0, None, None, None) == -1
    assert b'NULL ctx' in lib.dice_last_error()
    assert lib.dice_similarity_matrix_sharded(ctxs, 1, ctypes.byref(f), 7, None, None, 0, None, None) == -1
    assert b'gather_mode' in lib.dice_last_error()
    assert lib.dice_batch_upload_ids(None, 0, None, None, 2, None, None, None, None) == -1
    assert b'NULL batch' in lib.dice_last_error()


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


def test_vocab_pack_is_a_permutation_and_never_worse():
    """lh_vocab_pack (csrc/vocab_pack.cpp): the packed order is a permutation, its reported
    cost is the true (template, dword) cost and never above the starting order's."""
    import ctypes

    import numpy as np

    from licensee_amd import native_host
    lib = native_host._load()
    fn = lib.lh_vocab_pack
    fn.restype = ctypes.c_int64
    vp = ctypes.c_void_p
    fn.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp, ctypes.c_int32, ctypes.c_int64,
                   ctypes.c_uint64, vp]
    rng = np.random.default_rng(5)
    for T, V, bin_bits in ((20, 700, 32), (130, 900, 64)):
        W = (T + 63) // 64
        M = rng.random((V, T)) < rng.random(T) * 0.3
        M[np.arange(V), rng.integers(0, T, V)] = True       # every word in >= 1 template
        sig = np.zeros((V, W), np.uint64)
        for t in range(T):
            sig[:, t // 64] |= M[:, t].astype(np.uint64) << np.uint64(t % 64)

        def cost(order):
            c = 0
            for b in range(0, V, bin_bits):
                ws = order[b:b + bin_bits]
                anyt, allt = M[ws].any(0), M[ws].all(0) & (len(ws) == 32)
                c += int(anyt.sum()) * (2 if bin_bits == 32 else 1) - (int(allt.sum()) if bin_bits == 32 else 0)
            return c
        init = rng.permutation(V).astype(np.int32)
        out = np.empty(V, np.int32)
        got = fn(sig.ctypes.data, V, W, T, init.ctypes.data, bin_bits, 200000, 7, out.ctypes.data)
        assert sorted(out.tolist()) == list(range(V))
        assert got == cost(out) <= cost(init)
        bad = init.copy()
        bad[0] = bad[1]
        assert fn(sig.ctypes.data, V, W, T, bad.ctypes.data, bin_bits, 10, 7, out.ctypes.data) == -1


def test_bits_to_ids_round_trip():
    """_native.bits_to_ids (the id-list form of dice_batch_upload_ids) lists each row's set bits
    in ascending order, uint16 up to 65,536 words, across chunk boundaries and empty rows."""
    rng = np.random.default_rng(3)
    for V, n, chunk in ((1000, 300, 70), (70000, 40, 16)):
        dense = rng.random((n, V)) < 0.01
        dense[5] = False
        pad = np.pad(dense, ((0, 0), (0, (-V) % 64)))
        bits = np.packbits(pad, axis=1, bitorder='little').view(np.uint64)
        offs, ids = _native.bits_to_ids(bits, V, chunk=chunk)
        assert ids.dtype == (np.uint16 if V <= 65536 else np.uint32)
        assert offs[0] == 0 and offs[-1] == ids.size
        for r in range(n):
            assert np.array_equal(ids[offs[r]:offs[r + 1]], np.flatnonzero(dense[r]))
