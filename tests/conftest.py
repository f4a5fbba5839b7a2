import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'jalil-saboorizadeh-multi-speaker-neural-vocoder_amd')
GOLDEN = os.path.join(ROOT, 'tests', 'golden')
for p in (ROOT, PKG, os.path.join(ROOT, 'oracle'), GOLDEN):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs through the HIP C-ABI)')
    config.addinivalue_line('markers', 'slow: long-running CPU test')


def golden(name):
    import numpy as np
    return np.load(os.path.join(GOLDEN, name + '.npz'))


@pytest.fixture(scope='session')
def hip():
    """The product HIP library; GPU tests fail loudly if it cannot be loaded."""
    import torch
    assert torch.cuda.is_available(), 'gpu test needs a GPU'
    import samplernn_hip
    samplernn_hip.lib()  # raises if the .so is missing
    return samplernn_hip
