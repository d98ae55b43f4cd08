import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE = os.environ.get('LICENSEE_REFERENCE', '/root/reference')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a gfx950 GPU (run on the MI355X box)')


def pytest_sessionstart(session):
    """GPU sessions: let torch's HIP runtime initialize before liblicensee_dice.so loads, as bench.py
    does. Both resolve the same libamdhip64 soname; when the library (built against /opt/rocm)
    loads it first, torch's later device query can find no GPU, and the tests that use torch for
    streams, graphs or pinned memory would fail depending on test order."""
    markexpr = getattr(session.config.option, 'markexpr', '') or ''
    if 'gpu' in markexpr and 'not gpu' not in markexpr:
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.init()
        except Exception:
            pass


@pytest.fixture(scope='session')
def reference_root():
    if not os.path.isdir(os.path.join(REFERENCE, 'spec', 'fixtures')):
        pytest.skip('reference checkout not present (GPU box / CI without /root/reference)')
    return REFERENCE
