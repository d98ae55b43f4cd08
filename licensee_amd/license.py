"""License template corpus: restates ``Licensee::License`` (lib/licensee/license.rb).

At run time the corpus comes from ``licensee_amd/data/templates.json``: per template the
metadata the path needs (key, title, spdx_id, nickname, hidden, featured), its
``content_normalized`` and its ``spdx_alt_segments`` count. That file is derived data,
produced in the build container from ``/root/reference/vendor`` by
``tools/vendor_templates.py`` with this package's own normalizer and pinned by the
reference's ``spec/fixtures/license-hashes.json`` (tests/test_normalize.py). Raw template
bodies never ship; ``License.from_raw`` rebuilds a template from its vendored file when the
reference tree is present (vendoring and CPU tests only).

Reference map:
    License.all / keys / find            license.rb:20-47 (sorted by key; hidden/pseudo filters)
    name / name_without_version          license.rb:134-142
    creative_commons?                    license.rb:209-212
    parts (front matter split)           license.rb:263-267
    spdx_alt_segments                    license.rb:273-283
    LicenseMeta defaults                 license_meta.rb:293-296 (hidden: true, featured: false)
"""
from __future__ import annotations

import json
import os
import re
from typing import Dict, List, Optional

from .content_helper import ContentHelper, build_title_regex, name_without_version

DATA_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'data', 'templates.json')
PSEUDO_LICENSES = ('other', 'no-license')                      # license.rb:92
_FRONT_MATTER = re.compile(r'\A(---\n.*\n---\n+)?(.*)', re.S)   # license.rb:266 (/m)


class InvalidLicense(ValueError):
    """license.rb:6"""


class License(ContentHelper):
    """One license template. ``similarity`` is routed through the HIP scorer
    (``licensee_amd.dice``); there is no CPU scoring path in the product."""

    _corpus: Optional[List['License']] = None
    _title_regex = None

    def __init__(self, key: str, meta: Optional[dict] = None, content: Optional[str] = None,
                 content_normalized: Optional[str] = None, alt_segments: Optional[int] = None):
        self.key = key.lower()
        meta = dict(meta or {})
        self.title = meta.get('title')
        self.spdx_id_meta = meta.get('spdx_id')
        self.nickname = meta.get('nickname')
        self.hidden = meta.get('hidden', True) if meta.get('hidden') is not None else True
        self.featured = meta.get('featured', False) if meta.get('featured') is not None else False
        self.content = content
        if content_normalized is not None:
            self._content_normalized = content_normalized
        self._alt_segments = alt_segments

    # -- identity / metadata ----------------------------------------------------------
    def __repr__(self):
        return f'#<Licensee::License key={self.key}>'

    def __eq__(self, other):
        return isinstance(other, License) and other.key == self.key

    def __hash__(self):
        return hash(self.key)

    @property
    def spdx_id(self):
        if self.spdx_id_meta:
            return self.spdx_id_meta
        if self.key == 'other':
            return 'NOASSERTION'
        if self.key == 'no-license':
            return 'NONE'
        return None

    def pseudo_license(self) -> bool:
        return self.key in PSEUDO_LICENSES

    @property
    def name(self) -> str:
        if self.pseudo_license():
            return self.key.replace('-', ' ').capitalize()
        return self.title or self.spdx_id

    def name_without_version(self) -> str:
        return name_without_version(self.name)

    def creative_commons(self) -> bool:
        return self.key.startswith('cc-')

    cc = creative_commons

    def other(self) -> bool:
        return self.key == 'other'

    def gpl(self) -> bool:
        return self.key in ('gpl-2.0', 'gpl-3.0')

    def lgpl(self) -> bool:
        return self.key in ('lgpl-2.1', 'lgpl-3.0')

    # -- ContentHelper hooks ----------------------------------------------------------
    def spdx_alt_segments(self) -> int:
        if self._alt_segments is None:
            raise InvalidLicense(f'no SPDX alt-segment count for {self.key}')
        return self._alt_segments

    def content_normalized(self, wrap=None):
        if self.pseudo_license():
            return None
        return super().content_normalized(wrap)

    @staticmethod
    def title_regex_provider():
        return License.title_regex()

    # -- similarity: GPU-routed (content_helper.rb:128-133) ---------------------------
    def similarity(self, other) -> float:
        from .dice import pair_similarity
        return pair_similarity(self, other)

    # -- corpus ---------------------------------------------------------------------
    @classmethod
    def _load(cls) -> List['License']:
        if cls._corpus is None:
            with open(DATA_PATH, 'r', encoding='utf-8') as fh:
                table = json.load(fh)
            cls._corpus = [cls(t['key'], t['meta'], content_normalized=t['content_normalized'],
                               alt_segments=t['alt_segments']) for t in table['licenses']]
            cls._corpus += [cls(k) for k in PSEUDO_LICENSES]
        return cls._corpus

    @classmethod
    def set_corpus(cls, licenses: List['License']):
        """Install an explicit corpus (vendoring tool / tests); resets the title regex and the
        process-wide Dice engine, whose resident templates belong to the previous corpus."""
        cls._corpus = list(licenses)
        cls._title_regex = None
        from . import dice
        dice.reset_default_engine()

    @classmethod
    def all(cls, hidden: bool = False, featured: Optional[bool] = None, pseudo: bool = True,
            psuedo: Optional[bool] = None) -> List['License']:
        """license.rb:20-36"""
        if psuedo is not None:
            pseudo = psuedo
        out = list(cls._load())
        if not hidden:
            out = [l for l in out if not l.hidden]
        if not pseudo:
            out = [l for l in out if not l.pseudo_license()]
        out.sort(key=lambda l: l.key)
        if featured is not None:
            out = [l for l in out if l.featured == featured]
        return out

    @classmethod
    def find(cls, key: str, hidden: bool = True) -> Optional['License']:
        for l in cls.all(hidden=hidden):
            if l.key == key.lower():
                return l
        return None

    @classmethod
    def title_regex(cls):
        if cls._title_regex is None:
            cls._title_regex = build_title_regex(cls.all(hidden=True, pseudo=False))
        return cls._title_regex

    # -- raw vendored files (build container only) --------------------------------------
    @classmethod
    def from_raw(cls, key: str, raw: str, alt_segments: Optional[int]) -> 'License':
        import yaml
        m = _FRONT_MATTER.match(raw)
        front, body = m.group(1), m.group(2)
        meta = {}
        if front:
            y = yaml.safe_load(front[3:].rstrip('\n').rstrip('-')) or {}
            meta = {'title': y.get('title'), 'spdx_id': y.get('spdx-id'),
                    'nickname': y.get('nickname'), 'hidden': y.get('hidden'),
                    'featured': y.get('featured')}
        return cls(key, meta, content=body, alt_segments=alt_segments)

    def meta_dict(self) -> Dict:
        return {'title': self.title, 'spdx_id': self.spdx_id_meta, 'nickname': self.nickname,
                'hidden': self.hidden, 'featured': self.featured}


def spdx_alt_segments_from_xml(raw_xml: str) -> int:
    """license.rb:273-283"""
    text = re.search(r'<text>(.*)</text>', raw_xml, re.S).group(1)
    text = re.sub(r'<copyrightText>.*?</copyrightText>', '', text, flags=re.S)
    text = re.sub(r'<titleText>.*?</titleText>', '', text, flags=re.S)
    text = re.sub(r'<optional.*?>.*?</optional>', '', text, flags=re.S)
    return len(re.findall(r'<alt .*?>', text, re.S))


def load_raw_corpus(reference_root: str) -> List[License]:
    """Build the 47 templates from a reference checkout (license.rb:20-36, 58-68)."""
    lic_dir = os.path.join(reference_root, 'vendor', 'choosealicense.com', '_licenses')
    spdx_dir = os.path.join(reference_root, 'vendor', 'license-list-XML', 'src')
    out = []
    for fn in sorted(os.listdir(lic_dir)):
        if not fn.endswith('.txt'):
            continue
        key = fn[:-4].lower()
        with open(os.path.join(lic_dir, fn), 'r', encoding='utf-8', newline='') as fh:
            raw = fh.read()
        lic = License.from_raw(key, raw, None)
        with open(os.path.join(spdx_dir, lic.spdx_id + '.xml'), 'r', encoding='utf-8', newline='') as fh:
            lic._alt_segments = spdx_alt_segments_from_xml(fh.read())
        out.append(lic)
    out += [License(k) for k in PSEUDO_LICENSES]
    return out
