import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE = os.environ.get('LICENSEE_REFERENCE', '/root/reference')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a gfx950 GPU (run on the MI355X box)')


@pytest.fixture(scope='session')
def reference_root():
    if not os.path.isdir(os.path.join(REFERENCE, 'spec', 'fixtures')):
        pytest.skip('reference checkout not present (GPU box / CI without /root/reference)')
    return REFERENCE
