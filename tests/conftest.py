import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def pytest_sessionstart(session):
    # Two HIP runtimes share a test process: torch's bundled one and /opt/rocm's, which libscotty_mi355x.so links.
    # torch's must open the device first, or it reports "no ROCm-capable device" once the library has; tests that use
    # only the C-ABI can run before any torch test, so torch's runtime is initialised up front (no-op without a GPU).
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass
