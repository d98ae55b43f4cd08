"""SPDX license-list-XML template ingestion.

The reference reads the SPDX XML of a license only for ``spdx_alt_segments``
(lib/licensee/license.rb:273-283: <text> minus <copyrightText>, <titleText> and <optional>,
then the count of <alt ...> tags); its templates' text comes from choosealicense.com. Config 3
of BASELINE.json asks for the SPDX template set (~600) itself as the Dice corpus, so this module
turns a license-list-XML file into a template text:

  * the <text> element of the <license>;
  * <titleText> and <copyrightText> are dropped (licensee strips the title and copyright lines
    of a license file too: content_helper.rb strip_title / strip_copyright);
  * <optional> content is kept (SPDX matching guideline: optional text may be present);
  * each <alt> contributes its element text, the default wording that its `match` regex
    accepts;
  * <p> ends a paragraph (blank line), <br/> a line, <list>/<item> put each item on its own
    line after its <bullet>;
  * whitespace inside a paragraph is collapsed (the XML's indentation is not license text).

The result goes through the same ``content_normalized`` as every other text. Parsing uses the
standard library's ElementTree on the vendored files (no entity expansion beyond the five XML
built-ins). ``tools/vendor_spdx.py`` writes the 47 vendored XMLs' texts to
``licensee_amd/data/spdx.json`` (the GPU box has no reference tree); tests/test_spdx.py pins the
data file to the XMLs and the alt-segment counts to license.rb's regex restatement.

Parity of the text extraction itself is unpinned: the reference never builds these texts.
"""
from __future__ import annotations

import json
import os
import re
import xml.etree.ElementTree as ET
from typing import Dict, List, Optional

from .content_helper import ContentHelper, FIELD_REGEX, WORDSET_REGEX
from .license import spdx_alt_segments_from_xml

DATA_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'data', 'spdx.json')
_NS = '{http://www.spdx.org/license}'
_WS = re.compile(r'\s+')


def _local(tag: str) -> str:
    return tag[len(_NS):] if tag.startswith(_NS) else tag


_LINE, _PARA = '\x01', '\x02'   # explicit breaks; the XML's own line breaks are only wrapping


def _walk(el, out: List[str]):
    name = _local(el.tag)
    if name in ('titleText', 'copyrightText'):
        return
    if name == 'p':
        out.append(_PARA)
    elif name in ('list', 'item', 'br'):
        out.append(_LINE)
    if el.text:
        out.append(el.text)
    for ch in el:
        _walk(ch, out)
        if ch.tail:
            out.append(ch.tail)
    if name == 'p':
        out.append(_PARA)
    elif name == 'list':
        out.append(_LINE)


def _render(parts: List[str]) -> str:
    s = _WS.sub(' ', ''.join(parts))
    s = re.sub(r' *([\x01\x02]) *', r'\1', s)
    s = re.sub(r'[\x01\x02]*\x02[\x01\x02]*', '\n\n', s)
    s = s.replace(_LINE, '\n')
    return s.strip()


def text_from_xml(raw_xml: str) -> str:
    """The template text of one license-list-XML document (rules in the module docstring)."""
    root = ET.fromstring(raw_xml)
    lic = root.find(_NS + 'license')
    if lic is None:
        lic = root
    text = lic.find(_NS + 'text')
    if text is None:
        raise ValueError('no <text> element')
    out: List[str] = []
    _walk(text, out)
    return _render(out) + '\n'


def license_info_from_xml(raw_xml: str) -> Dict:
    root = ET.fromstring(raw_xml)
    lic = root.find(_NS + 'license')
    if lic is None:
        lic = root
    return {'id': lic.get('licenseId'), 'name': lic.get('name'), 'text': text_from_xml(raw_xml),
            'alt_segments': spdx_alt_segments_from_xml(raw_xml)}


def ingest_dir(spdx_dir: str) -> List[Dict]:
    """Every license-list-XML file of a directory, sorted by license id."""
    out = []
    for fn in sorted(os.listdir(spdx_dir)):
        if fn.endswith('.xml'):
            with open(os.path.join(spdx_dir, fn), 'r', encoding='utf-8', newline='') as fh:
                out.append(license_info_from_xml(fh.read()))
    out.sort(key=lambda r: r['id'].lower())
    return out


class SpdxTemplate(ContentHelper):
    """A Dice template built from an SPDX XML (key = lower-cased license id), with the
    reference's alt-segment rule for its length slack (content_helper.rb:337-347)."""

    def __init__(self, license_id: str, name: Optional[str], text: str, alt_segments: int, key_prefix: str = ''):
        self.key = key_prefix + license_id.lower()
        self.spdx_id = license_id
        self.title = name
        self.content = text
        self._alt_segments = alt_segments

    def __repr__(self):
        return f'#<SpdxTemplate {self.spdx_id}>'

    def spdx_alt_segments(self) -> int:
        return self._alt_segments

    def has_spdx_alt_segments(self) -> bool:
        return True

    def creative_commons(self) -> bool:
        return self.key.startswith('cc-')

    @staticmethod
    def title_regex_provider():
        from .license import License
        return License.title_regex()


def load(key_prefix: str = '') -> List[SpdxTemplate]:
    """The vendored SPDX templates (licensee_amd/data/spdx.json), sorted by license id."""
    with open(DATA_PATH, 'r', encoding='utf-8') as fh:
        recs = json.load(fh)['licenses']
    return [SpdxTemplate(r['id'], r['name'], r['text'], r['alt_segments'], key_prefix) for r in recs]


def corpus_with_spdx(real: List, total: int = 600, seed: int = 20250202) -> List:
    """Config 3 with real texts: the 47 choosealicense.com templates, the 47 SPDX templates
    (keys prefixed 'spdx:' so both sets coexist in key order) and synthetic ones up to `total`
    (licensee_amd/synth_templates.py), in key order."""
    from .synth_templates import synthetic_templates
    spdx = load('spdx:')
    return synthetic_templates(list(real) + spdx, total=total, seed=seed)


__all__ = ['text_from_xml', 'license_info_from_xml', 'ingest_dir', 'SpdxTemplate', 'load', 'corpus_with_spdx',
           'FIELD_REGEX', 'WORDSET_REGEX']
