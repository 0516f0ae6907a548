import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long CPU test")


def pytest_sessionstart(session):
    """On a GPU box, bring up torch's HIP runtime before the engine's: torch ships its own
    libamdhip64, and once the engine (linked against /opt/rocm's) has initialised the
    device, torch's lazy init reports "No HIP GPUs are available".  Tests use torch only
    as HBM plumbing (device buffers for the *_async entry points)."""
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle
    oracle.lib()
    return oracle
