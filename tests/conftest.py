"""pytest configuration: the `gpu` marker and shared fixtures.

`-m "not gpu"` runs on the CPU-only build container (oracle vs golden fixtures, host logic, ABI
exports, gloo multi-process plumbing); `-m gpu` runs the HIP parity tests on an MI355X.
"""
import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libimgrec.so")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not gpu_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    from image_recommender_amd import _lib
    _lib.load()
    return True
