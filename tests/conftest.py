import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: test needs an MI355X (HIP device) and the native HIP kernels')
    config.addinivalue_line('markers', 'slow: long-running test')


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason='no GPU available')
    for item in items:
        if 'gpu' in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True)
def _seed_everything():
    """Every test starts from the same RNG state (numpy, python, torch via mx.random.seed),
    like the reference's @with_seed() decorator (tests/python/unittest/common.py)."""
    import random
    import numpy as np
    random.seed(1234)
    np.random.seed(1234)
    import mxnet_maintenance_amd as mx
    mx.random.seed(1234)
    yield
