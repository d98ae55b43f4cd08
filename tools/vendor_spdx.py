"""Write licensee_amd/data/spdx.json from a reference checkout's vendored SPDX license-list-XML
(vendor/license-list-XML/src/*.xml): per license its id, name, template text
(licensee_amd/spdx.py text_from_xml) and alt-segment count (license.rb:273-283).

    python tools/vendor_spdx.py [/root/reference]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else '/root/reference'
    from licensee_amd.spdx import DATA_PATH, ingest_dir
    recs = ingest_dir(os.path.join(ref, 'vendor', 'license-list-XML', 'src'))
    with open(DATA_PATH, 'w', encoding='utf-8') as fh:
        json.dump({'source': 'vendor/license-list-XML/src (reference checkout), licensee_amd/spdx.py',
                   'licenses': recs}, fh, indent=1, ensure_ascii=False)
        fh.write('\n')
    print(f'{len(recs)} SPDX templates -> {DATA_PATH}')


if __name__ == '__main__':
    main()
