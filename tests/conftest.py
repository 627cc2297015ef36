"""pytest configuration: the `gpu` marker and import paths.

CPU tests (-m "not gpu") exercise the oracle against the golden vectors, host
logic and the C-ABI library's exports.  GPU tests (-m gpu) are the parity tests
proper: they call the product through the C-ABI and compare with the oracle.
"""
import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "oracle", ROOT / "rram-caffe-simulation_amd" / "python"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def device():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a machine without a GPU (run with -m 'not gpu')")
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle
