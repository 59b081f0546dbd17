"""Test configuration: the `gpu` marker and import paths.

`-m "not gpu"` runs here (no GPU): the oracle against the reference's golden
fixtures, host logic, and that the C-ABI library loads and exports every
symbol include/tropical_hip.h declares.  `-m gpu` runs on an MI355X: the HIP
path against the goldens and the oracle.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tropical-nerf.pytorch_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running CPU oracle case")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible ROCm GPU")
    return torch.device("cuda", 0)
