import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REF = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture
def ref_resource():
    def _p(name):
        p = os.path.join(REF, "resource", name)
        if os.path.exists(p):
            return p
        # vendored copies of the small reference configs / schemas (GPU boxes have no reference)
        v = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", name)
        if os.path.exists(v):
            return v
        pytest.skip(f"reference resource {name} not mounted")
    return _p


def pytest_collection_modifyitems(config, items):
    """``gpu``-marked tests skip (rather than fail) on a host without a HIP device."""
    if gpu_available():
        return
    skip = pytest.mark.skip(reason="no HIP GPU on this host")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture
def cuda():
    if not gpu_available():
        pytest.skip("no GPU")
    import torch
    return torch.device("cuda")
