import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'tests')):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP device); run with -m gpu')


@pytest.fixture(scope='session')
def oracle_lib():
    from oracle import trigger
    return trigger.lib()


@pytest.fixture(scope='session')
def gpu():
    """Skip-free GPU guard: a -m gpu run on a box without a GPU must fail loudly."""
    import torch
    assert torch.cuda.is_available(), 'gpu tests need a HIP device'
    from mkids_sdr_amd import _lib
    _lib.load()
    return 0
