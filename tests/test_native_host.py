"""Native host normalizer/interner (csrc/normalize.cpp + rx.cpp) == the Python restatement.

Both run the same compiled patterns (content_helper.py); this checks the C++ op sequence,
regex engine, decoding and interning against the Python path on the reference's fixtures,
every vendored-license property text, all 47 raw template bodies (reference present), and
seeded fuzz texts built from markup fragments the normalizer handles.
"""
import json
import os
import random

import numpy as np
import pytest

from licensee_amd.content_helper import ContentHelper
from licensee_amd.license import License
from licensee_amd.project_files import LicenseFile

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')


@pytest.fixture(scope='module')
def hp():
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.native_host import HostPrep
    return HostPrep(TemplateCorpus(License.all(hidden=True, pseudo=False)))


def golden(name):
    with open(os.path.join(GOLDEN, name), encoding='utf-8') as fh:
        return json.load(fh)


class _Body(ContentHelper):
    def __init__(self, content):
        self.content = content

    @staticmethod
    def title_regex_provider():
        return License.title_regex()


def test_fixture_files(hp, reference_root):
    n = 0
    for r in golden('fixture_files.json'):
        if 'unsupported' in r:
            continue
        with open(os.path.join(reference_root, 'spec', 'fixtures', r['fixture'], r['file']), 'rb') as fh:
            raw = fh.read()
        got = hp.normalize(raw, r['file'])
        if got is not None:
            assert got == r['normalized'], r['fixture']
            n += 1
    assert n >= 50


def test_template_bodies(hp, reference_root):
    from licensee_amd.license import load_raw_corpus
    raw = load_raw_corpus(reference_root)
    n = 0
    for lic in raw:
        if lic.pseudo_license():
            continue
        got = hp.normalize(lic.content, None, is_file=False)
        expect = License.find(lic.key).content_normalized()
        assert got == expect, lic.key                # all 47 native, incl. cecill-2.1 / mulanpsl-2.0
        n += 1
    assert n == 47


def test_python_only_characters_are_exhaustive():
    """The characters the native path hands back (normalize.cpp python_only) are exactly the
    BMP code points where a per-character table cannot reproduce Python: re.I equating them
    with an ASCII letter, a multi-character lower(), or the Final_Sigma rule."""
    import re
    import sys
    letters = re.compile('[a-z]', re.I)
    found = set()
    for cp in range(128, 0x10000):
        ch = chr(cp)
        if letters.fullmatch(ch) or len(ch.lower()) != 1 or ch.lower() != (ch + 'x').lower()[:-1] or \
                ch.lower() != ('x' + ch).lower()[1:]:
            found.add(ch)
    assert found == PYTHON_ONLY


FRAGMENTS = ['# Title', 'The MIT License', 'Copyright (c) 2019 Foo Bar', 'All rights reserved.', '* * *',
             '=====', '-----', '> quoted', '[link](http://example.com)', '_em_ *strong* ~x~', '1. item',
             ' * bullet', '(a) sub', 'http://x.org/y', 'Version 2.0', 'licence & programme', 'sub-\nlicense',
             "it's the users' 'code'", '“quoted” — dash – en', 'END OF TERMS AND CONDITIONS', 'GNU GPLv3',
             'Developed by: someone\n\n', '(including the next paragraph)', 'creative commons zero',
             '/* comment */', '// c++', 'Attribution-NonCommercial 4.0', '﻿BOM', 'tab\there',
             'CRLF\r\nline', 'x\ry', 'Apache License 2.0', 'the apache license', 'foo-bar', 'per cent',
             # non-ASCII: native with Python's lower()/isalnum() tables, except the contextual five
             'CAFÉ Licence', 'ÀÉÎÕÜ ß straße', '软件许可证 MIT', 'Ωmega Ǆ ǅemal', 'élicence licenceé', 'Ⅻ² ①']
CONTEXTUAL = ['ΑΣ ΣΟΦΙΑ', 'İstanbul', 'Kelvin \u212a', 'ſome', 'ı dotless']
PYTHON_ONLY = {'\u0130', '\u0131', '\u017f', '\u212a', '\u03a3'}


def test_fuzz_texts(hp):
    rng = random.Random(20250202)
    checked = fell = 0
    for i in range(400):
        parts = [rng.choice(FRAGMENTS) for _ in range(rng.randint(1, 12))]
        if rng.random() < 0.05:
            parts.append(rng.choice(CONTEXTUAL))
        text = rng.choice(['\n', '\n\n', ' ', '  ']).join(parts)
        if rng.random() < 0.3:
            body = License.all(hidden=True, pseudo=False)[rng.randrange(47)].content_normalized()
            text = text + '\n\n' + body[:rng.randint(0, 3000)]
        got = hp.normalize(text, 'LICENSE')
        if got is None:                               # contextual characters: Python path
            assert any(ch in PYTHON_ONLY for ch in text)
            fell += 1
            continue
        checked += 1
        assert got == LicenseFile(text, 'LICENSE').content_normalized(), (i, text[:200])
    assert checked > 350 and fell > 0


def test_spelling_and_link_markup_fuzz(hp):
    """normalize_spelling (content_helper.rb:314-316) and strip_link_markup (:289-291) on texts
    dense in varietal words: alone, recased, prefixed/suffixed, split, bracketed, inside link
    markup, beside punctuation/dashes/quotes/non-ASCII -- exercises the native two-character key
    index and the "](" gate of the link pass."""
    from licensee_amd.content_helper import VARIETAL_WORDS
    rng = random.Random(3)
    keys = list(VARIETAL_WORDS)
    checked = 0
    for i in range(300):
        words = []
        for _ in range(rng.randint(1, 60)):
            k = rng.choice(keys)
            words.append(rng.choice([k, k.upper(), k.capitalize(), k + 's', 'x' + k, k + '_', k + '-', '(' + k + ')',
                                     k[:2], k[:3] + ' ' + k[3:], '[' + k + '](http://a)', '[' + k + ']']))
            if rng.random() < 0.3:
                words.append(rng.choice(['&', '--', '\u2014', '"q"', '\n', '  ', '\u00e9', 'colour', 'licence', '](']))
        text = ' '.join(words)
        got = hp.normalize(text, 'LICENSE')
        if got is None:
            continue
        checked += 1
        assert got == LicenseFile(text, 'LICENSE').content_normalized(), (i, text[:200])
    assert checked > 250


def test_batch_prep_matches_python(hp):
    from licensee_amd.matchers import Copyright, Exact
    vend = golden('vendored.json')['templates']
    texts = [c['normalized'] for t in vend for c in t['cases'].values()]
    texts += ['Copyright 2020 Foo', 'Attribution-NoDerivatives 4.0', 'café license', '', 'ΣΟΦΙΑ license',
              'CAFÉ LICENCE 软件']
    texts += [License.find(k).content_normalized() for k in ('mit', 'gpl-3.0', 'vim', 'postgresql')]
    fb, cr, ex, fell = hp.prep_files(texts, ['LICENSE'] * len(texts), nthreads=4)
    assert fell.sum() == 1                       # only 'ΣΟΦΙΑ' (Final_Sigma) takes the Python path
    corpus = hp.corpus
    keys = [t.key for t in corpus.templates]
    for i, t in enumerate(texts):
        lf = LicenseFile(t, 'LICENSE')
        bits, wf = corpus.intern(lf.wordset())
        assert np.array_equal(fb.bits[i], bits) and fb.wordset_size[i] == wf and fb.length[i] == lf.length(), i
        assert bool(fb.cc_false_positive[i]) == bool(lf.potential_false_positive())
        assert cr[i] == (Copyright(lf).match() is not None), i
        e = Exact(lf).match()
        assert ex[i] == (keys.index(e.key) if e is not None else -1), i


def test_field_masks_match_python(hp):
    """lh_prep_files' per-file field masks (device Exact, dice_batch_exact): bit k = the file's
    wordset holds the k-th template field word outside the vocabulary; the template need masks
    (lh_template_field_masks) hold the same words of each template's fields_normalized."""
    corpus = hp.corpus
    assert hp.nv_fields, 'the vendored templates have field words outside the vocabulary (fullname)'
    for t, tpl in enumerate(corpus.templates):
        fs = set(tpl.fields_normalized())
        assert int(hp.field_need[t]) == sum(1 << k for k, w in enumerate(hp.nv_fields) if w in fs), tpl.key
    ncsa = License.find('ncsa').content_normalized()
    assert '[fullname]' in ncsa
    texts = [ncsa, ncsa.replace('[fullname]', 'zzzq'), ncsa.replace('[fullname]', 'fullname'), 'fullname only',
             'ΣΟΦΙΑ fullname', '', 'year project fullname']
    texts += [License.find(k).content_normalized() for k in ('bsd-3-clause', 'gpl-3.0', 'isc')]
    fb, cr, fm, fell = hp.prep_files(texts, ['LICENSE'] * len(texts), nthreads=3, field_masks=True)
    assert fell.sum() == 1
    fb2, cr2, _, _ = hp.prep_files(texts, ['LICENSE'] * len(texts), nthreads=3)
    assert np.array_equal(fb.bits, fb2.bits) and np.array_equal(fb.wordset_size, fb2.wordset_size)
    assert np.array_equal(cr, cr2)
    for i, t in enumerate(texts):
        ws = LicenseFile(t, 'LICENSE').wordset() or frozenset()
        assert int(fm[i]) == sum(1 << k for k, w in enumerate(hp.nv_fields) if w in ws), i


def test_wordset_token_fuzz(hp):
    """The wordset scan (content_helper.rb:109, (?:[\\w/-](?:'s|(?<=s)')?)+) on texts dense in its
    corner cases: apostrophes after 's' and before 's' (including "it's'" where the 's' taken by
    's gets no s' of its own), doubled quotes, '/' and '-' inside and around tokens, tokens and
    runs longer than the native scan's 64-character blocks, vocabulary and non-vocabulary words."""
    rng = random.Random(11)
    vocab = hp.corpus.vocab
    pieces = ["it's'", "users'", "s''s", "'s", "s'", "x's's", "don't", "a/b-c", "--", "//", "-x-", "s's'",
              "q'", "'", "''", "/'s", "-'", "_'s_"]
    texts = []
    for i in range(300):
        toks = []
        for _ in range(rng.randint(1, 80)):
            r = rng.random()
            if r < 0.4:
                toks.append(rng.choice(vocab))
            elif r < 0.7:
                toks.append(rng.choice(pieces))
            elif r < 0.8:
                toks.append(''.join(rng.choice('abs-/_\'') for _ in range(rng.randint(60, 140))))
            else:
                toks.append(rng.choice(vocab) + rng.choice(pieces) + rng.choice(vocab))
        texts.append(''.join(rng.choice([' ', '\n', ', ', '.']) + t for t in toks))
    fb, cr, ex, fell = hp.prep_files(texts, ['LICENSE'] * len(texts), nthreads=2)
    assert not fell.any()
    corpus = hp.corpus
    for i, t in enumerate(texts):
        lf = LicenseFile(t, 'LICENSE')
        bits, wf = corpus.intern(lf.wordset())
        assert fb.wordset_size[i] == wf and np.array_equal(fb.bits[i], bits), (i, t[:200])


def test_thousands_of_copyright_lines(hp):
    """A file opening with ~10k consecutive copyright lines (the copyright pattern's repeated
    group, content_helper.rb:255 + copyright.rb:8-11, nests the backtracking matcher once per
    line): batch workers (256 MiB stacks) finish it natively; on an ordinary 8 MiB thread the
    match aborts at the frame limit and the text goes to the Python path. No crash, and every
    result equals the Python LicenseFile path."""
    from licensee_amd.matchers import Copyright, Exact
    mit = License.find('mit').content_normalized()
    texts = [''.join(f'Copyright (c) {1990 + i % 30} Holder Number {i} <h{i}@example.com>\n' for i in range(n)) + mit
             for n in (50, 2_000, 10_000)]
    texts.append('\n'.join(f'Copyright {i} Foo' for i in range(12_000)))   # copyright-only file
    fb, cr, ex, fell = hp.prep_files(texts, ['LICENSE'] * len(texts), nthreads=4)
    assert not fell.any()
    corpus = hp.corpus
    keys = [t.key for t in corpus.templates]
    for i, t in enumerate(texts):
        lf = LicenseFile(t, 'LICENSE')
        bits, wf = corpus.intern(lf.wordset())
        assert np.array_equal(fb.bits[i], bits) and fb.wordset_size[i] == wf and fb.length[i] == lf.length(), i
        assert cr[i] == (Copyright(lf).match() is not None), i
        e = Exact(lf).match()
        assert ex[i] == (keys.index(e.key) if e is not None else -1), i
    assert cr[3] and not cr[0]
    # single-text entry point on this (8 MiB) thread: small texts native, the deep one falls back
    assert hp.normalize(texts[0]) == LicenseFile(texts[0], 'LICENSE').content_normalized()
    assert hp.normalize(texts[2]) is None


def test_byte_path_equals_utf32_path(hp, monkeypatch):
    """ASCII texts are normalized as bytes (normalize.cpp prep_ascii); LH_NO_BYTE_PATH=1 sends
    them through the UTF-32 passes instead. Both paths give identical batch outputs on ASCII
    fuzz texts, the template bodies and texts with CR / CRLF line ends."""
    from licensee_amd.native_host import HostPrep
    monkeypatch.setenv('LH_NO_BYTE_PATH', '1')
    wide = HostPrep(hp.corpus)
    monkeypatch.delenv('LH_NO_BYTE_PATH')
    rng = random.Random(11)
    ascii_frags = [f for f in FRAGMENTS if f.isascii()]
    bodies = [t.content_normalized() for t in License.all(hidden=True, pseudo=False)]
    texts = []
    for i in range(600):
        parts = [rng.choice(ascii_frags) for _ in range(rng.randint(1, 20))]
        text = rng.choice(['\n', '\r\n', '\r', ' ']).join(parts)
        if rng.random() < 0.5:
            b = rng.choice(bodies)
            text += '\n\n' + b[:rng.randint(0, len(b))]
        texts.append(text)
    texts += bodies + ['', ' ', '\r', 'a' * 40 + '-' + 'b' * 40]
    names = ['LICENSE'] * len(texts)
    a = hp.prep_files(texts, names, nthreads=4)
    b = wide.prep_files(texts, names, nthreads=4)
    assert not a[3].any() and not b[3].any()
    for field in ('bits', 'wordset_size', 'length', 'cc_false_positive'):
        assert np.array_equal(getattr(a[0], field), getattr(b[0], field)), field
    assert np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
    for t in texts[:200]:
        assert hp.normalize(t, 'LICENSE') == wide.normalize(t, 'LICENSE')


def test_spelling_keys_at_block_edges(hp):
    """The byte path's spelling prefilter (normalize.cpp spell_prefix_mask) reads 64-byte blocks
    and a zero-padded copy near the text's end: every key at every offset around the block and
    half-block edges and at the very end of the text is still replaced."""
    from licensee_amd.content_helper import VARIETAL_WORDS
    checked = 0
    for key in VARIETAL_WORDS:
        for off in (0, 1, 29, 30, 31, 32, 33, 61, 62, 63, 64, 65, 95, 96, 127, 128):
            filler = ('ab ' * 64)[:off]
            for tail in ('', ' end', ' ' + 'z' * 70):
                text = filler + key + tail
                got = hp.normalize(text, 'LICENSE')
                assert got == LicenseFile(text, 'LICENSE').content_normalized(), (key, off, tail)
                checked += 1
    assert checked == len(VARIETAL_WORDS) * 16 * 3


def test_border_lines_fuzz(hp):
    """The hand-written border_markup pass (normalize.cpp strip_borders: ^[*-](.*?)[*-]$ -> \\1)
    on texts dense in lines that start and/or end with '*' / '-', on both text paths."""
    rng = random.Random(7)
    pieces = ['*', '-', '--', '**', '*-', '-*', '* x *', '- item -', '-x', 'x-', '*x', 'x*', '---', '- a', 'b -',
              '* * *', ' * y *', '-- z --', 'plain line', '', 'licence - x', '*é*', '- café -']
    checked = 0
    for i in range(500):
        lines = [rng.choice(pieces) for _ in range(rng.randint(1, 25))]
        text = rng.choice(['\n', '\n\n']).join(lines)
        if rng.random() < 0.3:
            text = 'The MIT License\n\n' + text + '\n\nPermission is granted.'
        got = hp.normalize(text, 'LICENSE')
        if got is None:
            continue
        checked += 1
        assert got == LicenseFile(text, 'LICENSE').content_normalized(), (i, text[:300])
    assert checked > 450


def _as_scan_bytes(text):
    """content_normalized as the device wordset scan reads it: one byte per character,
    non-ASCII characters as 0x80 (lh_normalize_files)."""
    return bytes(ord(c) if ord(c) < 0x80 else 0x80 for c in text)


def test_normalize_files_matches_python(hp):
    """lh_normalize_files (the device-wordset host stage): per file the normalized text as scan
    bytes at a 16-byte aligned offset, its length in characters and the CC / Copyright flags --
    equal to the Python path and to lh_prep_files, the Python-path files (Final_Sigma) appended."""
    vend = golden('vendored.json')['templates']
    texts = [c['normalized'] for t in vend for c in t['cases'].values()][:120]
    texts += ['Copyright 2020 Foo', 'Attribution-NoDerivatives 4.0', 'café license', '', 'ΣΟΦΙΑ license',
              'CAFÉ LICENCE 软件', "it's the users' s''s a/b-c work's"]
    texts += [License.find(k).content_normalized() for k in ('mit', 'gpl-3.0', 'vim', 'postgresql')]
    data = [t.encode('utf-8') for t in texts]
    text, off, tl, ln, cc, cr, fell = hp.normalize_files(data, ['LICENSE'] * len(texts), nthreads=3)
    fb, cr2, _, fell2 = hp.prep_files(data, ['LICENSE'] * len(texts), nthreads=3)
    assert np.array_equal(fell, fell2) and fell.sum() == 1
    assert (off % 16 == 0).all() and (off >= 0).all() and (off + tl <= len(text)).all()
    assert np.array_equal(cr, cr2) and np.array_equal(cc, fb.cc_false_positive) and np.array_equal(ln, fb.length)
    for i, t in enumerate(texts):
        cn = LicenseFile(t, 'LICENSE').content_normalized()
        assert bytes(text[off[i]:off[i] + tl[i]]) == _as_scan_bytes(cn), i
        assert ln[i] == len(cn), i


def test_normalize_files_without_room_appends_the_rest(hp):
    """normalize_files with a buffer too small for every text: the files lh_normalize_files had no room
    for (status 3) are appended by the wrapper, at 16-byte aligned offsets, with the same bytes."""
    texts = [License.find(k).content_normalized().encode() for k in ('mit', 'gpl-3.0', 'apache-2.0', 'isc', 'bsd-2-clause')]
    full = hp.normalize_files(texts, None, nthreads=2)
    small = hp.normalize_files(texts, None, nthreads=2, out=lambda nbytes: np.empty(20000, np.uint8))
    for a, b in zip(full[3:6], small[3:6]):
        assert np.array_equal(a, b)
    text, off, tl = small[0], small[1], small[2]
    assert (off % 16 == 0).all() and (off + tl <= len(text)).all()
    for i in range(len(texts)):
        assert bytes(text[off[i]:off[i] + tl[i]]) == bytes(full[0][full[1][i]:full[1][i] + full[2][i]])
