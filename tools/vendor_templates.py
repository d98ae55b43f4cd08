"""Regenerate licensee_amd/data/templates.json (and data/ipsum.json) from a reference checkout.

Reads the 47 vendored choosealicense.com templates + their SPDX XML (alt-segment counts),
normalizes each body with licensee_amd.content_helper (pinned by the reference's
spec/fixtures/license-hashes.json) and writes the derived table the product loads at run
time. Also copies the reference's filler word list spec/fixtures/ipsum.txt (a test data
fixture: the words add_random_words draws from, spec_helper.rb:82-91) as data/ipsum.json,
lowercased as the downcase step of content_normalized would leave it
(content_helper.rb:153-168; the list holds letters only). Run in the build container only:

    python tools/vendor_templates.py [/root/reference]
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from licensee_amd.license import DATA_PATH, License, load_raw_corpus  # noqa: E402


def build_table(reference_root: str) -> dict:
    corpus = load_raw_corpus(reference_root)
    License.set_corpus(corpus)
    with open(os.path.join(reference_root, 'spec', 'fixtures', 'license-hashes.json')) as fh:
        golden = json.load(fh)
    rows = []
    for lic in License.all(hidden=True, pseudo=False):
        digest = lic.content_hash()
        if golden.get(lic.key) != digest:
            raise SystemExit(f'{lic.key}: normalized SHA1 {digest} != reference {golden.get(lic.key)}')
        rows.append({'key': lic.key, 'meta': lic.meta_dict(), 'content_normalized': lic.content_normalized(),
                     'alt_segments': lic.spdx_alt_segments(), 'sha1': digest})
    return {'source': 'firoj0/licensee vendor/choosealicense.com + vendor/license-list-XML',
            'generator': 'tools/vendor_templates.py', 'licenses': rows}


def ipsum_table(reference_root: str) -> dict:
    with open(os.path.join(reference_root, 'spec', 'fixtures', 'ipsum.txt'), encoding='utf-8') as fh:
        raw = fh.read().split()   # ipsum.split, spec_helper.rb:85 (repeats kept: same draw weights)
    assert all(w.isalpha() for w in raw)
    return {'source': 'firoj0/licensee spec/fixtures/ipsum.txt', 'generator': 'tools/vendor_templates.py',
            'note': 'whitespace-split words, lowercased (normalized space)', 'words': [w.lower() for w in raw]}


def main(argv):
    root = argv[1] if len(argv) > 1 else '/root/reference'
    table = build_table(root)
    os.makedirs(os.path.dirname(DATA_PATH), exist_ok=True)
    with open(DATA_PATH, 'w', encoding='utf-8') as fh:
        json.dump(table, fh, ensure_ascii=False, indent=1, sort_keys=True)
        fh.write('\n')
    print(f'wrote {DATA_PATH}: {len(table["licenses"])} templates')
    ipsum = ipsum_table(root)
    path = os.path.join(os.path.dirname(DATA_PATH), 'ipsum.json')
    with open(path, 'w', encoding='utf-8') as fh:
        json.dump(ipsum, fh, indent=0)
        fh.write('\n')
    print(f'wrote {path}: {len(ipsum["words"])} words')


if __name__ == '__main__':
    main(sys.argv)
