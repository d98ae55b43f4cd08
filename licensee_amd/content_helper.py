"""Host-side text normalization: a Python restatement of ``Licensee::ContentHelper``.

The north star keeps ``content_normalized`` on the host ("Ruby stays the host
language"); Ruby is not in this image, so the host language here is Python and
this module restates the reference rules one for one:

    reference: lib/licensee/content_helper.rb:9-347   (regexes, order, strip/normalize ops)
               lib/licensee/license.rb:134-175          (name, name_without_version, title_regex)
               lib/licensee/matchers/copyright.rb:8-11  (Copyright::REGEX, reused by strip_copyright)
               lib/licensee/license_field.rb:50         (FIELD_REGEX)

Onigmo -> Python ``re`` translation rules used throughout (SURVEY.md §7 "hard part 1"):
  * Ruby ``\\s \\S \\d \\w`` are ASCII classes; Python's are Unicode, so they are spelled out
    explicitly (``_S``, ``_NS``, ``_D``, ``_W``).
  * Ruby ``^``/``$`` are always line anchors -> every pattern is compiled with ``re.M``;
    Ruby ``/m`` (dot matches newline) is Python ``re.S``.
  * Flags embedded by regexp interpolation / ``Regexp.union`` (``(?i-mx:...)``,
    ``(?-mix:...)``) become Python scoped flags ``(?i:...)`` / ``(?-i:...)`` so that e.g. a
    license nickname stays case-sensitive inside the case-insensitive title union.
  * ``String#strip`` strips ``\\0\\t\\n\\v\\f\\r`` and space only; ``squeeze(' ')`` collapses
    runs of spaces; ``length`` counts characters (Python ``len`` of ``str``).

Pinned by the reference's own goldens: ``spec/fixtures/license-hashes.json`` (47 template
SHA1s), ``spec/fixtures/fixtures.yml`` (fixture SHA1s), ``spec/fixtures/detect.json`` and
``spec/licensee/content_helper_spec.rb`` -- see tests/test_normalize.py.

HTML input (``strip_html``, content_helper.rb:293-299) needs the ``reverse_markdown`` gem,
which has no equivalent here: HTML files raise ``NotImplementedError`` (parity unpinned).
"""
from __future__ import annotations

import hashlib
import re
from typing import Dict, List, Optional

# --- Ruby character classes spelled out in ASCII --------------------------------------
_WS = ' \t\n\v\f\r'
_S = r'[ \t\n\v\f\r]'          # Ruby \s
_NS = r'[^ \t\n\v\f\r]'        # Ruby \S
_D = r'[0-9]'                  # Ruby \d
_W = r'[A-Za-z0-9_]'           # Ruby \w
_STRIP_CHARS = '\0' + _WS      # String#strip

START_REGEX_SRC = r'\A' + _S + '*'                                   # content_helper.rb:9
_M = re.M


def _c(src: str, flags: int = 0) -> 're.Pattern[str]':
    return re.compile(src, flags | _M)


# content_helper.rb:10
END_OF_TERMS_REGEX = _c(r'^[ \t\n\v\f\r#*_]*end of (the )?terms and conditions[ \t\n\v\f\r#*_]*$', re.I)

# content_helper.rb:11-33
REGEXES: Dict[str, 're.Pattern[str]'] = {
    'bom': _c(START_REGEX_SRC + '\ufeff'),
    'hrs': _c('^' + _S + r'*[=\-*]{3,}' + _S + '*$'),
    'all_rights_reserved': _c(START_REGEX_SRC + r'all rights reserved\.?$', re.I),
    'whitespace': _c(_S + '+'),
    'markdown_headings': _c('^' + _S + '*#+'),
    'version': _c(START_REGEX_SRC + 'version.*$', re.I),
    'span_markup': _c(r'[_*~]+(.*?)[_*~]+'),
    'link_markup': _c(r'\[(.+?)\]\(.+?\)'),
    'block_markup': _c('^' + _S + '*>'),
    'border_markup': _c(r'^[*-](.*?)[*-]$'),
    'comment_markup': _c('^' + _S + r'*?[/*]{1,2}'),
    'url': _c(START_REGEX_SRC + r'https?://[^ ]+\n'),
    'bullet': _c(r'\n\n' + _S + r'*(?:[*-]|\(?[0-9a-z]{1,2}[).])' + _S + '+', re.I),
    'developed_by': _c(START_REGEX_SRC + r'developed by:.*?\n\n', re.I | re.S),
    'cc_dedication': _c(r'The' + _S + r'+text' + _S + r'+of' + _S + r'+the' + _S + r'+Creative' + _S
                        + r'+Commons.*?Public' + _S + r'+Domain' + _S + r'+Dedication.', re.I | re.S),
    'cc_wiki': _c(r'wiki.creativecommons.org', re.I),
    'cc_legal_code': _c('^' + _S + '*Creative Commons Legal Code' + _S + '*$', re.I),
    'cc0_info': _c(r'For more information, please see' + _S + '*' + _NS + '+zero' + _NS + '+', re.I | re.S),
    'cc0_disclaimer': _c(r'CREATIVE COMMONS CORPORATION.*?\n\n', re.I | re.S),
    'unlicense_info': _c(r'For more information, please.*' + _NS + '+unlicense' + _NS + '+', re.I | re.S),
    'mit_optional': _c(r'\(including the next paragraph\)', re.I),
}

# content_helper.rb:34-41 (order matters: applied in insertion order)
NORMALIZATIONS = {
    'lists': (_c('^' + _S + r'*(?:' + _D + r'\.|[*-])(?: [*_]{0,2}\(?[0-9a-z]\)[*_]{0,2})?' + _S
                 + r'+([^\n])'), r'- \1'),
    'https': (_c(r'http:'), 'https:'),
    'ampersands': ('&', 'and'),
    'dashes': (_c(r'(?<!^)([\u2014\u2013-]+)(?!$)'), '-'),
    'quote': (_c('[`\'"\u2018\u201c\u2019\u201d]'), "'"),
    'hyphenated': (_c('(' + _W + '+)-' + _S + r'*\n' + _S + '*(' + _W + '+)'), r'\1-\2'),
}

# content_helper.rb:45-88 (insertion order is the alternation order of the union)
VARIETAL_WORDS = {
    'acknowledgment': 'acknowledgement', 'analogue': 'analog', 'analyse': 'analyze',
    'artefact': 'artifact', 'authorisation': 'authorization', 'authorised': 'authorized',
    'calibre': 'caliber', 'cancelled': 'canceled', 'capitalisations': 'capitalizations',
    'catalogue': 'catalog', 'categorise': 'categorize', 'centre': 'center',
    'emphasised': 'emphasized', 'favour': 'favor', 'favourite': 'favorite',
    'fulfil': 'fulfill', 'fulfilment': 'fulfillment', 'initialise': 'initialize',
    'judgment': 'judgement', 'labelling': 'labeling', 'labour': 'labor',
    'licence': 'license', 'maximise': 'maximize', 'modelled': 'modeled',
    'modelling': 'modeling', 'offence': 'offense', 'optimise': 'optimize',
    'organisation': 'organization', 'organise': 'organize', 'practise': 'practice',
    'programme': 'program', 'realise': 'realize', 'recognise': 'recognize',
    'signalling': 'signaling', 'sub-license': 'sublicense', 'sub license': 'sublicense',
    'utilisation': 'utilization', 'whilst': 'while', 'wilful': 'wilfull',
    'non-commercial': 'noncommercial', 'per cent': 'percent', 'copyright owner': 'copyright holder',
}

# content_helper.rb:89-105
STRIP_METHODS = (
    'bom', 'cc_optional', 'cc0_optional', 'unlicense_optional', 'borders', 'title', 'version',
    'url', 'copyright', 'title', 'block_markup', 'developed_by', 'end_of_terms', 'whitespace',
    'mit_optional',
)

# wordset scan, content_helper.rb:109  -- (?:[\w/-](?:'s|(?<=s)')?)+
WORDSET_REGEX = re.compile(r"(?:[A-Za-z0-9_/-](?:'s|(?<=s)')?)+")

# license_field.rb:50 with keys from vendor/choosealicense.com/_data/fields.yml:7-26 (file order)
FIELD_KEYS = ('fullname', 'login', 'email', 'project', 'description', 'year', 'projecturl')
FIELD_REGEX = re.compile(r'\[(' + '|'.join(re.escape(k) for k in FIELD_KEYS) + r')\]')


def ruby_regexp_escape(s: str) -> str:
    """``Regexp.escape`` (escapes space as ``\\ `` and ``-``/``#`` too)."""
    out = []
    for ch in s:
        if ch in '[]{}()|-*.\\?+^$#':
            out.append('\\' + ch)
        elif ch == ' ':
            out.append('\\ ')
        elif ch == '\t':
            out.append('\\t')
        elif ch == '\n':
            out.append('\\n')
        elif ch == '\r':
            out.append('\\r')
        elif ch == '\f':
            out.append('\\f')
        elif ch == '\v':
            out.append('\\v')
        else:
            out.append(ch)
    return ''.join(out)


def ruby_strip(s: str) -> str:
    return s.strip(_STRIP_CHARS)


def squeeze_spaces(s: str) -> str:
    return re.sub(' {2,}', ' ', s)


def ruby_split_lines(s: str) -> List[str]:
    """``String#split("\\n")``: trailing empty fields are dropped."""
    parts = s.split('\n')
    while parts and parts[-1] == '':
        parts.pop()
    return parts


# Copyright::REGEX, lib/licensee/matchers/copyright.rb:8-11
_COPYRIGHT_SYMBOLS = r'(?:(?i:copyright)|(?i:\(c\))|\u00a9|\u00a9)'
_MAIN_LINE = r'(?i:[_*\- \t\n\v\f\r]*' + _COPYRIGHT_SYMBOLS + r'.*$)'
_OPTIONAL_LINE = r'(?i:[_*\- \t\n\v\f\r]*with Reserved Font Name.*$)'
COPYRIGHT_REGEX_SRC = START_REGEX_SRC + '((?:' + _MAIN_LINE + _OPTIONAL_LINE + '*)+)$'
COPYRIGHT_REGEX = _c(COPYRIGHT_REGEX_SRC, re.I)
# copyright.rb:14 -- /#{REGEX}+\z/io on content.strip
COPYRIGHT_MATCH_REGEX = _c('(?:' + COPYRIGHT_REGEX_SRC + r')+\Z', re.I)
# content_helper.rb:255 -- Regexp.union(Copyright::REGEX, REGEXES[:all_rights_reserved])
_STRIP_COPYRIGHT_REGEX = _c('(?:' + COPYRIGHT_REGEX_SRC + ')|(?:' + START_REGEX_SRC
                            + r'(?i:all rights reserved\.?$))', re.I)

_SPELLING_REGEX = _c(r'\b(?:' + '|'.join(ruby_regexp_escape(k) for k in VARIETAL_WORDS) + r')\b')
_BULLET_PAREN_REGEX = _c(r'\)' + _S + r'+\(')
_HRS_LINE = REGEXES['hrs']


# --------------------------------------------------------------------------------------
# Title regex (license.rb:144-175, content_helper.rb:199-215)
# --------------------------------------------------------------------------------------
def _ruby_sub_replacement(template: str, m: 're.Match[str]') -> str:
    """Expand a Ruby ``sub`` replacement string: ``\\0-\\9`` are group refs, ``\\\\`` a
    backslash; any other backslash pair is kept verbatim."""
    out = []
    i = 0
    while i < len(template):
        ch = template[i]
        if ch == '\\' and i + 1 < len(template):
            nxt = template[i + 1]
            if nxt.isdigit():
                g = m.group(int(nxt))
                out.append(g or '')
                i += 2
                continue
            if nxt == '\\':
                out.append('\\')
                i += 2
                continue
            out.append(ch + nxt)
            i += 2
            continue
        out.append(ch)
        i += 1
    return ''.join(out)


def ruby_sub(pattern: 're.Pattern[str]', replacement: str, s: str) -> str:
    """``String#sub`` (first match only) with Ruby replacement-string semantics."""
    m = pattern.search(s)
    if not m:
        return s
    return s[:m.start()] + _ruby_sub_replacement(replacement, m) + s[m.end():]


def _translate_ruby_classes(src: str) -> str:
    """Translate ``\\s``/``\\d`` in a generated Ruby regexp source to ASCII classes."""
    out = []
    i = 0
    while i < len(src):
        if src[i] == '\\' and i + 1 < len(src):
            nxt = src[i + 1]
            if nxt == 's':
                out.append(_S)
            elif nxt == 'd':
                out.append(_D)
            else:
                out.append(src[i:i + 2])
            i += 2
            continue
        out.append(src[i])
        i += 1
    return ''.join(out)


def name_without_version(name: str) -> str:
    """license.rb:140-142 -- /(.+?)(( v?\\d\\.\\d)|$)/.match(name)[1]"""
    return re.match(r'(.+?)(( v?[0-9]\.[0-9])|$)', name, re.M | re.S).group(1)


def license_title_regex_src(name: str, key: str, nickname: Optional[str]) -> str:
    """Python source of ``License#title_regex`` (license.rb:144-175), flags scoped."""
    string = name.lower().replace('*', 'u', 1)
    simple = string
    string = re.sub(r'\Athe ', '', string, count=1, flags=re.I)
    string = re.sub(r',? version ', ' ', string, count=1)
    string = ruby_sub(re.compile(r'v([0-9]+\.[0-9]+)'), r'\1', string)
    string = ruby_regexp_escape(string)
    string = ruby_sub(re.compile(r'\\ licen[sc]e', re.I), r'(?:\ licen[sc]e)?', string)
    version_match = re.search(r'[0-9]+\\.([0-9]+)', string)
    if version_match:
        if version_match.group(1) == '0':
            vsub = r',?\s+(?:version\ |v(?:\. )?)?\1(\2)?'
        else:
            vsub = r',?\s+(?:version\ |v(?:\. )?)?\1\2'
        string = ruby_sub(re.compile(r'\\ ([0-9]+)(\\.[0-9]+)'), vsub, string)
    string = ruby_sub(re.compile(r'\bgnu\\ '), '(?:GNU )?', string)
    title = _translate_ruby_classes(string)

    kstr = key.replace('-', '[- ]', 1)
    kstr = kstr.replace('.', '\\.', 1)
    kstr += r'(?:\ licen[sc]e)?'

    parts = ['(?i:' + simple + ')', '(?i:' + title + ')', '(?i:' + kstr + ')']
    if nickname:
        nick = ruby_sub(re.compile(r'\bGNU ', re.I), '(?:GNU )?', nickname)
        parts.append('(?-i:' + nick + ')')
    return '(?:' + '|'.join(parts) + ')'


def build_title_regex(licenses) -> 're.Pattern[str]':
    """``ContentHelper.title_regex`` over ``License.all(hidden: true, psuedo: false)``
    (content_helper.rb:199-215). ``licenses`` are key-sorted objects exposing
    ``name``, ``key``, ``title`` and ``nickname``."""
    titles = [license_title_regex_src(l.name, l.key, l.nickname) for l in licenses]
    for l in licenses:
        nwv = name_without_version(l.name)
        if l.title == nwv:
            continue
        titles.append('(?i:' + ruby_regexp_escape(nwv) + ')')
    src = '(?-i:' + START_REGEX_SRC + r')\(?(?:the )?(?:' + '|'.join(titles) + ').*?$'
    return _c(src, re.I)


# --------------------------------------------------------------------------------------
# ContentHelper mixin
# --------------------------------------------------------------------------------------
class ContentHelper:
    """Mixin restating ``Licensee::ContentHelper``. Hosts provide ``content`` (str or None),
    optionally ``filename`` and, for templates, ``spdx_alt_segments()``; the process-wide
    title regex comes from ``title_regex_provider()`` (License corpus)."""

    DIGEST = hashlib.sha1

    # -- public API (content_helper.rb:108-168) -----------------------------------------
    def wordset(self):
        if not hasattr(self, '_wordset'):
            cn = self.content_normalized()
            self._wordset = None if cn is None else frozenset(WORDSET_REGEX.findall(cn))
        return self._wordset

    def wordset_list(self):
        """Distinct words in first-occurrence order (Ruby ``Set`` preserves insertion order)."""
        cn = self.content_normalized()
        if cn is None:
            return None
        seen = {}
        for w in WORDSET_REGEX.findall(cn):
            seen.setdefault(w, None)
        return list(seen)

    def length(self) -> int:
        cn = self.content_normalized()
        return 0 if cn is None else len(cn)

    def length_delta(self, other) -> int:
        return abs(self.length() - other.length())

    def content_hash(self) -> Optional[str]:
        cn = self.content_normalized()
        if cn is None:
            return None
        return hashlib.sha1(cn.encode('utf-8')).hexdigest()

    def content_without_title_and_version(self):
        if not hasattr(self, '_cwtv'):
            self._content_state = None
            for op in ('html', 'hrs', 'comments', 'markdown_headings', 'link_markup', 'title', 'version'):
                self._strip(op)
            self._cwtv = self._cur()
        return self._cwtv

    def content_normalized(self, wrap: Optional[int] = None):
        if not hasattr(self, '_content_normalized'):
            base = self.content_without_title_and_version()
            if base is None:
                self._content_normalized = None
            else:
                self._content_state = base.lower()
                for op in ('lists', 'https', 'ampersands', 'dashes', 'quote', 'hyphenated',
                           'spelling', 'span_markup', 'bullets'):
                    self._normalize(op)
                for op in STRIP_METHODS:
                    self._strip(op)
                self._content_normalized = self._cur()
        if wrap is None:
            return self._content_normalized
        return wrap_text(self._content_normalized, wrap)

    def wordset_fieldless(self):
        if not hasattr(self, '_wordset_fieldless'):
            self._wordset_fieldless = self.wordset() - self.fields_normalized_set()
        return self._wordset_fieldless

    def fields_normalized(self) -> List[str]:
        if not hasattr(self, '_fields_normalized'):
            self._fields_normalized = FIELD_REGEX.findall(self.content_normalized())
        return self._fields_normalized

    def fields_normalized_set(self):
        return frozenset(self.fields_normalized())

    def has_spdx_alt_segments(self) -> bool:
        return hasattr(self, 'spdx_alt_segments')

    def similarity(self, other) -> float:
        """content_helper.rb:128-133 for any two ContentHelper objects, scored on the GPU
        (``dice.pair_similarity``); a non-License self uses the simple length delta (:343)."""
        from .dice import pair_similarity
        return pair_similarity(self, other)

    def variation_adjusted_length_delta(self, other) -> int:
        """content_helper.rb:337-347"""
        delta = self.length_delta(other)
        if not self.has_spdx_alt_segments():
            return delta
        adjusted = delta - max(len(self.fields_normalized()), self.spdx_alt_segments()) * 5
        return adjusted if adjusted > 0 else 0

    # -- private machinery (content_helper.rb:219-321) ------------------------------------
    def _cur(self):
        """``_content``: ``@_content ||= content.to_s.dup.strip``"""
        if getattr(self, '_content_state', None) is None:
            self._content_state = ruby_strip(_to_s(self.content))
        return self._content_state

    def _strip(self, regex_or_sym):
        if self._cur() is None:
            return
        if isinstance(regex_or_sym, str):
            meth = getattr(self, '_strip_' + regex_or_sym, None)
            if meth is not None:
                return meth()
            if regex_or_sym not in REGEXES:
                raise ValueError(f'{regex_or_sym} is an invalid regex reference')
            regex_or_sym = REGEXES[regex_or_sym]
        self._content_state = ruby_strip(squeeze_spaces(regex_or_sym.sub(' ', self._cur())))

    def _strip_title(self):
        tr = self.title_regex_provider()
        while tr.search(self._cur()):
            self._strip(tr)

    def _strip_borders(self):
        self._normalize_with(REGEXES['border_markup'], r'\1')

    def _strip_comments(self):
        lines = ruby_split_lines(self._cur())
        if len(lines) == 1:
            return
        if not all(REGEXES['comment_markup'].search(line) for line in lines):
            return
        self._strip('comment_markup')

    def _strip_copyright(self):
        while _STRIP_COPYRIGHT_REGEX.search(self._cur()):
            self._strip(_STRIP_COPYRIGHT_REGEX)

    def _strip_cc0_optional(self):
        if 'associating cc0' not in self._cur():
            return
        self._strip(REGEXES['cc_legal_code'])
        self._strip(REGEXES['cc0_info'])
        self._strip(REGEXES['cc0_disclaimer'])

    def _strip_cc_optional(self):
        if 'creative commons' not in self._cur():
            return
        self._strip(REGEXES['cc_dedication'])
        self._strip(REGEXES['cc_wiki'])

    def _strip_unlicense_optional(self):
        if 'unlicense' not in self._cur():
            return
        self._strip(REGEXES['unlicense_info'])

    def _strip_end_of_terms(self):
        m = END_OF_TERMS_REGEX.search(self._cur())
        if m:
            self._content_state = self._cur()[:m.start()]

    def _strip_link_markup(self):
        self._normalize_with(REGEXES['link_markup'], r'\1')

    def _strip_html(self):
        filename = getattr(self, 'filename', None)
        if not filename:
            return
        ext = _ruby_extname(filename)
        if re.search(r'\.html?', ext, re.I):
            raise NotImplementedError('HTML license files need the reverse_markdown gem '
                                      '(content_helper.rb:293-299); not supported')

    def _normalize(self, key):
        if key in NORMALIZATIONS:
            frm, to = NORMALIZATIONS[key]
            self._normalize_with(frm, to)
        elif key == 'spelling':
            self._content_state = _SPELLING_REGEX.sub(lambda m: VARIETAL_WORDS[m.group(0)], self._cur())
        elif key == 'span_markup':
            self._normalize_with(REGEXES['span_markup'], r'\1')
        elif key == 'bullets':
            self._content_state = REGEXES['bullet'].sub('\n\n- ', self._cur())
            self._content_state = _BULLET_PAREN_REGEX.sub(')(', self._cur())
        else:
            raise ValueError(f'{key} is an invalid normalization')

    def _normalize_with(self, frm, to):
        if isinstance(frm, str):
            self._content_state = self._cur().replace(frm, to)
        else:
            self._content_state = frm.sub(to, self._cur())


def _to_s(content) -> str:
    return '' if content is None else str(content)


def _ruby_extname(filename: str) -> str:
    """``File.extname``: extension of the basename, '' for dotfiles."""
    base = filename.rsplit('/', 1)[-1]
    stripped = base.lstrip('.')
    if '.' not in stripped:
        return ''
    ext = '.' + stripped.rsplit('.', 1)[-1]
    return '' if ext == '.' else ext


def wrap_text(text: Optional[str], line_width: int = 80) -> Optional[str]:
    """``ContentHelper.wrap`` (content_helper.rb:177-193)."""
    if text is None:
        return None
    text = REGEXES['bullet'].sub(lambda m: '\n' + m.group(0) + '\n', text)
    text = re.sub(r'([^\n])\n([^\n])', r'\1 \2', text)
    line_re = re.compile('(.{1,%d})(%s+|$)' % (line_width, _S), re.M)
    out = []
    for line in ruby_split_lines(text):
        if _HRS_LINE.search(line) or len(line) <= line_width:
            out.append(line)
        else:
            out.append(ruby_strip(line_re.sub(lambda m: m.group(1) + '\n', line)))
    return ruby_strip('\n'.join(out))


def format_percent(value: float) -> str:
    """content_helper.rb:195-197"""
    return '%.2f%%' % value
