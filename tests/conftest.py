import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the native extension")
    config.addinivalue_line("markers", "slow: long-running test")
    config.addinivalue_line(
        "markers", "gpu_shared: several processes whose kernels wait on each other on ONE GPU "
        "(K11 / persistent rehearsals); skipped unless DALGO_GPU_SHARED_TESTS=1")


def pytest_collection_modifyitems(config, items):
    if os.environ.get("DALGO_GPU_SHARED_TESTS", "0") == "1":
        return
    skip = pytest.mark.skip(reason="cross-process spin-waits on one GPU: opt-in via "
                                   "DALGO_GPU_SHARED_TESTS=1")
    for item in items:
        if "gpu_shared" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dalgo.ops import _ext
    assert _ext.load(), "native extension failed to load on a GPU host"
    return torch.device("cuda", 0)
