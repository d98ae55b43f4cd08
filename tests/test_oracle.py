"""The oracle (test infrastructure) pinned against the reference's own goldens, and the
C restatement (oracle/dice_ref.c) against the Python one.

  dice_matcher_spec.rb:23-78      exact similarity floats, match / confidence, stacked, CC
  vendored_license_spec.rb:9-94   every template detected as itself (rendered, no title,
                                  double title, rewrapped) and NOT with 75 random words
  fixtures.yml                    19 `matcher: dice` fixtures -> key; `other` fixtures -> no match
"""
import json
import os

import numpy as np
import pytest

from licensee_amd.license import License
from oracle import dice_oracle as O
from tests.helpers import make_files, oracle_templates

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')


def golden(name):
    with open(os.path.join(GOLDEN, name), encoding='utf-8') as fh:
        return json.load(fh)


@pytest.fixture(scope='module')
def templates():
    return License.all(hidden=True, pseudo=False)


@pytest.fixture(scope='module')
def otpl(templates):
    return oracle_templates(templates)


def chain(templates, otpl, rec, thr=98):
    """LicenseFile#license over (Copyright, Exact, Dice) with the oracle as Dice. Copyright
    cannot fire on these normalized-space records' license texts (checked separately)."""
    f = O.OracleFile(rec['normalized'])
    for t, l in zip(otpl, templates):
        if l.wordset() == f.wordset:
            return l.key, 'exact', 100
    idx, conf = O.match(otpl, f, thr, cc_fp=rec['cc_false_positive'])
    if idx >= 0:
        return templates[idx].key, 'dice', conf
    return 'other', None, None


def test_dice_spec_goldens(templates, otpl):
    cases = golden('dice_spec.json')['cases']
    keys = [l.key for l in templates]
    gpl = cases['gpl']
    f = O.OracleFile(gpl['file']['normalized'])
    ranked = O.matches_by_similarity(otpl, f, cc_fp=gpl['file']['cc_false_positive'])
    assert [[keys[i], s] for i, s in ranked[:3]] == gpl['by_similarity']      # exact float equality
    assert O.match(otpl, f)[1] == 100.0
    for name in ('not_a_license', 'stacked', 'cc_nd'):
        c = cases[name]
        idx, conf = O.match(otpl, O.OracleFile(c['file']['normalized']), cc_fp=c['file']['cc_false_positive'])
        assert idx == -1 and conf == 0 and type(conf) is int, name
    c = cases['cc_by']
    idx, _ = O.match(otpl, O.OracleFile(c['file']['normalized']), cc_fp=c['file']['cc_false_positive'])
    assert keys[idx] == 'cc-by-4.0'
    assert cases['cc_nd']['file']['cc_false_positive'] is True


def test_vendored_license_properties(templates, otpl):
    for t in golden('vendored.json')['templates']:
        for name, rec in t['cases'].items():
            key, matcher, conf = chain(templates, otpl, rec)
            assert (key == t['key']) == rec['detected'], (t['key'], name, key)


def test_fixture_expectations(templates, otpl):
    recs = golden('fixture_files.json')
    singles = [r for r in recs if sum(x['fixture'] == r['fixture'] for x in recs) == 1 and 'unsupported' not in r]
    n_dice = 0
    for r in singles:
        exp = r['expected']
        if r['copyright']:
            assert exp.get('matcher') == 'copyright'
            continue
        key, matcher, _ = chain(templates, otpl, r)
        if exp.get('matcher') in ('dice', 'exact'):
            assert (key, matcher) == (exp['key'], exp['matcher']), r['fixture']
            n_dice += exp['matcher'] == 'dice'
        elif exp.get('key') == 'other':
            assert key == 'other', r['fixture']
    assert n_dice == 18   # 19 dice fixtures minus the HTML one (reverse_markdown, unpinned)


def test_c_oracle_equals_python_oracle(templates, otpl):
    from licensee_amd.corpus import TemplateCorpus
    from oracle.native import OracleScorer
    corpus = TemplateCorpus(templates)
    files = make_files(templates, 400, 99)
    fb = corpus.intern_files(files)
    orc = OracleScorer(corpus.lf_bits, corpus.lf_size, corpus.fields_set_size, corpus.length_slack,
                       corpus.length, corpus.is_cc, corpus.n_vocab)
    for mode in (0, 1):
        best, ov, score = orc.match(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, 98.0,
                                    nthreads=4, mode=mode)
        for i, f in enumerate(files):
            ti, ts = O.matches_by_similarity(otpl, f.oracle, cc_fp=f.cc)[0]
            assert best[i] == (ti if ts >= 98 else -1) and score[i] == ts
            assert ov[i] == O.overlap(otpl[ti], f.oracle.wordset)
    mov, msc = orc.matrix(fb.bits, fb.wordset_size, fb.length, fb.cc_false_positive, nthreads=4)
    for i in range(0, 400, 37):
        for t in range(len(otpl)):
            o, d, s = O.similarity_parts(otpl[t], files[i].oracle)
            assert mov[i, t] == o and msc[i, t] == s


def test_tie_rule_later_template_wins():
    # two identical templates: the later one in key order ranks first (documented rule)
    a = O.OracleTemplate('a-1', 'foo bar baz qux', 0)
    b = O.OracleTemplate('b-1', 'foo bar baz qux', 0)
    f = O.OracleFile('foo bar baz qux')
    assert O.matches_by_similarity([a, b], f)[0][0] == 1
    assert O.best_argmax([(4, 8), (4, 8)], [True, True]) == 1
