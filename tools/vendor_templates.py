"""Regenerate licensee_amd/data/templates.json from a reference checkout.

Reads the 47 vendored choosealicense.com templates + their SPDX XML (alt-segment counts),
normalizes each body with licensee_amd.content_helper (pinned by the reference's
spec/fixtures/license-hashes.json) and writes the derived table the product loads at run
time. Run in the build container only:

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


def main(argv):
    root = argv[1] if len(argv) > 1 else '/root/reference'
    table = build_table(root)
    os.makedirs(os.path.dirname(DATA_PATH), exist_ok=True)
    with open(DATA_PATH, 'w', encoding='utf-8') as fh:
        json.dump(table, fh, ensure_ascii=False, indent=1, sort_keys=True)
        fh.write('\n')
    print(f'wrote {DATA_PATH}: {len(table["licenses"])} templates')


if __name__ == '__main__':
    main(sys.argv)
