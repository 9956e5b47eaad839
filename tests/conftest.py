import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, 'pose-unsupervised_amd', 'lib')
for p in (LIB, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs the HIP kernels)')


@pytest.fixture(scope='session')
def golden():
    import numpy as np

    def load(name):
        with np.load(os.path.join(GOLDEN, name)) as z:
            return {k: z[k] for k in z.files}
    return load


@pytest.fixture(scope='session')
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail('GPU test selected but no GPU is visible')
    return torch.device('cuda', 0)
