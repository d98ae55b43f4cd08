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
    """GPU sessions: initialize torch's HIP runtime up front. The library shares it either way
    (licensee_amd._native maps torch's runtime before liblicensee_dice.so; tests/test_runtime.py
    checks the library-first order), so this only moves torch's device start-up out of the first
    test's time limit."""
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
