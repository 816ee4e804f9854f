import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a ROCm GPU (MI355X) and the built libonetrans_hip.so')
    config.addinivalue_line('markers', 'slow: long-running')


@pytest.fixture(scope='session')
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.fail('gpu-marked test run without a ROCm GPU')
    return torch.device('cuda', 0)


def release_device_cache():
    """Return the memory this process's caching allocator holds to the device (multi-rank GPU tests
    spawn processes that allocate their own full-size tables on the same GPU)."""
    import gc
    import torch
    gc.collect()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
