"""The wordset scan on the device (dice_batch_upload_text, csrc/dice_words.hip) == the host scan.

ContentHelper#wordset (content_helper.rb:108-110, /(?:[\\w\\/-](?:'s|(?<=s)')?)+/ over
content_normalized) interned into the vocabulary bitset, |W_F| (every distinct word) and the
field-word masks of device Exact: the device builds them from the normalized texts of
lh_normalize_files; the host path (lh_prep_files, itself pinned to the Python restatement by
tests/test_native_host.py) is the checker. Bit-exact on every row, |W_F| and mask.
"""
import random

import numpy as np
import pytest

from licensee_amd.license import License

pytestmark = pytest.mark.gpu


def _scorer(corpus):
    from licensee_amd._native import Scorer
    return Scorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack, corpus.length,
                  corpus.is_cc, corpus.n_vocab, device=0)


@pytest.fixture(scope='module')
def vendored():
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.native_host import HostPrep
    corpus = TemplateCorpus(License.all(hidden=True, pseudo=False))
    hp = HostPrep(corpus)
    sc = _scorer(corpus)
    sc.vocab_setup(corpus.vocab, hp.nv_fields)
    yield corpus, hp, sc
    sc.close()


def _device_rows(sc, hp, texts, filenames=None):
    text, off, tl, ln, cc, cr, fell = hp.normalize_files(texts, filenames, nthreads=8)
    b = sc.batch(max(len(texts), 1))
    st = b.upload_text(text, off, tl, ln, cc)
    bits, wf, fm = b.download_rows()
    b.close()
    return bits, wf, fm, st, ln, cc, cr, fell


def _check_equal(sc, hp, texts, allow_overflow=False):
    data = [t if isinstance(t, bytes) else t.encode('utf-8') for t in texts]
    bits, wf, fm, st, ln, cc, cr, fell = _device_rows(sc, hp, data)
    fb, cr2, fm2, fell2 = hp.prep_files(data, None, nthreads=8, field_masks=True)
    if not allow_overflow:
        assert not st.any()
    ok = st == 0
    assert np.array_equal(fell, fell2)
    bad = np.nonzero(ok & ((bits != fb.bits).any(axis=1) | (wf != fb.wordset_size) | (fm != fm2)))[0]
    assert bad.size == 0, [(int(i), data[i][:120], int(wf[i]), int(fb.wordset_size[i])) for i in bad[:3]]
    assert np.array_equal(ln, fb.length) and np.array_equal(cc, fb.cc_false_positive) and np.array_equal(cr, cr2)
    return st


def test_synthetic_texts_and_fixtures(vendored):
    """3,000 synthetic config-2 texts (SyntheticCorpus.text), the vendored-property cases and
    every raw template body: device rows, |W_F| and field masks equal the host scan's."""
    import json
    import os
    corpus, hp, sc = vendored
    from licensee_amd.synth import SyntheticCorpus
    syn = SyntheticCorpus(corpus)
    texts = [syn.text(i)[0] for i in range(3000)]
    golden = os.path.join(os.path.dirname(__file__), 'golden', 'vendored.json')
    with open(golden, encoding='utf-8') as fh:
        vend = json.load(fh)['templates']
    texts += [c['normalized'] for t in vend for c in t['cases'].values()]
    texts += [t.content_normalized() for t in corpus.templates]
    texts += ['', 'Copyright 2020 Foo', 'café license', 'ΣΟΦΙΑ license', 'CAFÉ LICENCE 软件 ünïcödé-wörds']
    _check_equal(sc, hp, texts)


def test_token_corner_cases(vendored):
    """The scan's corner cases: apostrophes ('s, s', runs re-scanned across 64-byte blocks and
    1 KiB chunks), '/' and '-', tokens of 15-17, 63-65 and 1,023-1,025+ characters, texts ending
    exactly at block and chunk edges with a word character, vocabulary words with suffixes, long
    vocabulary words (URLs: the tail compare), non-ASCII separators."""
    corpus, hp, sc = vendored
    rng = random.Random(5)
    vocab = corpus.vocab
    longv = [w for w in vocab if len(w) > 16]
    assert longv, 'the vendored vocabulary holds words longer than 16 bytes (URLs)'
    pieces = ["it's'", "users'", "s''s", "'s", "s'", "x's's", "don't", "a/b-c", "--", "//", "-x-", "s's'",
              "q'", "'", "''", "/'s", "-'", "_'s_", 'é', '—', '软']
    texts = []
    for i in range(400):
        toks = []
        for _ in range(rng.randint(1, 120)):
            r = rng.random()
            if r < 0.35:
                toks.append(rng.choice(vocab))
            elif r < 0.45:
                toks.append(rng.choice(longv))
            elif r < 0.7:
                toks.append(rng.choice(pieces))
            elif r < 0.8:
                toks.append(''.join(rng.choice("abs-/_'") for _ in range(rng.randint(10, 200))))
            else:
                toks.append(rng.choice(vocab) + rng.choice(pieces) + rng.choice(vocab))
        texts.append(''.join(rng.choice([' ', '\n', ', ', '.', ' é ']) + t for t in toks))
    for n in (15, 16, 17, 63, 64, 65, 1023, 1024, 1025, 2047, 2048, 2049, 5000):
        texts.append('x' * n)
        texts.append('a ' + 'y' * n + ' b')
        texts.append('license ' + 's' * n + "'s tail")
    for n in (62, 63, 64, 65, 127, 128, 1022, 1023, 1024, 1025, 2046, 2047, 2048, 2049):
        base = ('permission ' * 300)[:n]
        texts.append(base)                   # ends with a word character at the edge (or near it)
        texts.append(base[:-2] + "s'")
        texts.append(base[:-3] + "x's")
        texts.append(base + "'s more")
    _check_equal(sc, hp, texts)


def test_apostrophes_across_chunk_edges(vendored):
    """The chunk-at-once scan joins runs over the apostrophes the regex consumes and hands chunks
    with "'s'" (or a joining apostrophe in their last two bytes) to the block loop: every such
    pattern placed across the 1 KiB chunk edges (and the 16-byte lane edges next to them), with
    the chunks around it taking either path."""
    corpus, hp, sc = vendored
    pats = ["users'", "x's", "s's'", "a's's", "it's'", "users''s", "s'x", "'s", "x'sx", "licensor's'", "s'''s",
            "don't", "its's's", "s's", "-'s", "/'s'"]
    filler = 'permission is hereby granted '
    texts = []
    for edge in (1024, 2048):
        for shift in range(-7, 7):
            for pat in pats:
                head = (filler * 100)[:edge + shift]
                tail = " licensor's grant users' rights " + filler * 3
                texts.append(head + pat + tail)
                texts.append(head + pat + "'s" + pat + tail)   # the block loop's chunk, then more
    texts += [("x's " * 300)[:k] + "s's' tail" for k in range(1010, 1030)]
    _check_equal(sc, hp, texts)


def test_overflowing_set_is_flagged_and_patched(vendored):
    """A file with more distinct non-vocabulary words than the device set holds is flagged
    (status 1, row left empty); dice_batch_set_rows then installs the host-prepared row."""
    corpus, hp, sc = vendored
    rng = random.Random(9)
    many = ' '.join('zq' + ''.join(rng.choice('abcdefghijklmnop') for _ in range(8)) for _ in range(1000))
    texts = ['permission is hereby granted ' + many, License.find('mit').content_normalized(), 'zq zq zq ' * 100]
    data = [t.encode() for t in texts]
    text, off, tl, ln, cc, cr, fell = hp.normalize_files(data, None)
    b = sc.batch(8)
    st = b.upload_text(text, off, tl, ln, cc)
    assert st.tolist() == [1, 0, 0]
    fb, _, fm, _ = hp.prep_files(data, None, field_masks=True)
    b.set_rows(np.array([0]), fb.bits[:1], fb.wordset_size[:1], fm[:1])
    bits, wf, fmd = b.download_rows()
    assert np.array_equal(bits, fb.bits) and np.array_equal(wf, fb.wordset_size) and np.array_equal(fmd, fm)
    assert wf[0] > 1000
    b.close()


def test_large_vocabulary_corpus():
    """The config-3 shape: 600 templates, V ~ 23.5k (368 words per row): 2,000 texts."""
    from licensee_amd.corpus import TemplateCorpus
    from licensee_amd.native_host import HostPrep
    from licensee_amd.synth import SyntheticCorpus
    from licensee_amd.synth_templates import synthetic_templates
    corpus = TemplateCorpus(synthetic_templates(License.all(hidden=True, pseudo=False), 600, seed=3))
    hp = HostPrep(corpus)
    sc = _scorer(corpus)
    sc.vocab_setup(corpus.vocab, hp.nv_fields)
    syn = SyntheticCorpus(corpus)
    texts = [syn.text(i)[0] for i in range(2000)]
    _check_equal(sc, hp, texts)
    sc.close()


def test_batch_detector_device_wordset_equals_host_wordset(vendored):
    """LicenseFile#license in bulk (batch.BatchDetector) with the wordset scanned on the device
    equals the host-scan chain, file by file, including a file that overflows the device set."""
    from licensee_amd.batch import BatchDetector
    from licensee_amd.dice import DiceEngine
    from licensee_amd.synth import SyntheticCorpus
    corpus, hp, _ = vendored
    syn = SyntheticCorpus(corpus)
    rng = random.Random(2)
    many = ' '.join('zq' + ''.join(rng.choice('abcdefgh') for _ in range(9)) for _ in range(900))
    texts = [syn.text(i)[0].encode() for i in range(1500)]
    texts += [License.find(k).content_normalized().encode() for k in ('mit', 'gpl-3.0', 'ncsa', 'bsd-3-clause', 'cc-by-4.0')]
    texts += [(License.find('mit').content_normalized() + ' ' + many).encode(), b'', 'ΣΟΦΙΑ license'.encode()]
    eng = DiceEngine(device=0)
    dev = BatchDetector(eng, nthreads=8, wordset_on='device')
    host = BatchDetector(eng, nthreads=8, wordset_on='host')
    assert dev.wordset_on == 'device'
    a, b = dev.detect(texts), host.detect(texts)
    assert [(d.license.key, d.matcher, d.confidence) for d in a] == [(d.license.key, d.matcher, d.confidence) for d in b]
    assert sum(d.matcher == 'dice' for d in a) > 500 and sum(d.matcher == 'exact' for d in a) >= 4
    stream = [list(x) for x in dev.detect_stream([(texts[:700], None), (texts[700:], None)])]
    assert [(d.license.key, d.confidence) for d in stream[0] + stream[1]] == [(d.license.key, d.confidence) for d in b]
    dev.close()
    host.close()
