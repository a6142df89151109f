"""pytest configuration: `gpu` marker + import paths.

-m "not gpu": oracle vs golden fixtures, host logic, C-ABI load/export checks
              (no kernel launches; runs in the CPU build container).
-m gpu      : parity of the HIP kernels (through libainp.so) against the oracle.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ml-audio-inpainting_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
