"""Shared test setup: import paths, the ``gpu`` marker, and common fixtures.

``-m "not gpu"`` tests run on the CPU-only dev container (oracle vs golden fixtures, host
logic, C-ABI exports, gloo data-parallel); ``-m gpu`` tests are the HIP parity tests and
need an MI355X (they call the kernels through libfs2_hip.so).
"""
import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
PKG = os.path.join(ROOT, "fine-grained-emotional-control-of-tts_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels through libfs2_hip.so)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def cfg_all():
    from fastspeech2 import load_config
    return load_config()


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from fastspeech2 import _native
    _native.load()   # fail loudly if the HIP library is missing on a GPU box
    return torch.device("cuda")
