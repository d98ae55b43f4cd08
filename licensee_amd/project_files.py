"""Candidate files: restates ``Licensee::ProjectFiles::ProjectFile`` / ``LicenseFile``.

    ProjectFile#initialize (decode)     lib/licensee/project_files/project_file.rb:37-45
    ProjectFile#matcher/confidence      project_file.rb:69-80
    LicenseFile::CC_FALSE_POSITIVE_REGEX license_file.rb:63-65 (here 173-175 of the concatenated view)
    LicenseFile#possible_matchers       license_file.rb:67-69
    LicenseFile#potential_false_positive? license_file.rb:80-82
    LicenseFile#license                 license_file.rb:92-98 (falls back to License 'other')
"""
from __future__ import annotations

import re
from typing import Optional, Union

from .content_helper import ContentHelper, ruby_strip
from .license import License

CC_FALSE_POSITIVE_REGEX = re.compile(r'^(creative commons )?Attribution-(NonCommercial|NoDerivatives)',
                                     re.I | re.M)


def decode_content(content: Union[str, bytes]) -> str:
    """project_file.rb:38-41: force UTF-8, drop invalid bytes, universal newline."""
    if isinstance(content, bytes):
        text = content.decode('utf-8', errors='ignore')
    else:
        text = content
    return text.replace('\r\n', '\n').replace('\r', '\n')


class ProjectFile:
    def __init__(self, content: Union[str, bytes], metadata=None):
        self.content = decode_content(content)
        if isinstance(metadata, str):
            metadata = {'name': metadata}
        self._data = metadata or {}

    @property
    def filename(self) -> Optional[str]:
        return self._data.get('name')

    path = filename

    def possible_matchers(self):
        raise NotImplementedError

    def matcher(self):
        if not hasattr(self, '_matcher'):
            self._matcher = None
            for cls in self.possible_matchers():
                m = cls(self)
                if m.match():
                    self._matcher = m
                    break
        return self._matcher

    def confidence(self):
        m = self.matcher()
        return None if m is None else m.confidence()

    def matched_license(self):
        lic = self.license()
        return None if lic is None else lic.spdx_id


class LicenseFile(ContentHelper, ProjectFile):
    def __init__(self, content: Union[str, bytes], metadata=None):
        ProjectFile.__init__(self, content, metadata)

    @staticmethod
    def title_regex_provider():
        return License.title_regex()

    def possible_matchers(self):
        from .matchers import Copyright, Dice, Exact
        return [Copyright, Exact, Dice]

    def potential_false_positive(self) -> bool:
        return CC_FALSE_POSITIVE_REGEX.search(ruby_strip(self.content)) is not None

    def license(self) -> License:
        m = self.matcher()
        if m is not None and m.match():
            return m.match()
        return License.find('other')

    match = license

    def similarity(self, other) -> float:
        from .dice import pair_similarity
        return pair_similarity(self, other)
