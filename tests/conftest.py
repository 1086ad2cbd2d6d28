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


# Observed parity errors recorded by GPU tests (``parity_log`` fixture): written at session end
# to gpurun_out/parity_observed.json so a GPU run's numbers can be committed under profiles/
# and quoted in DESIGN.md section 2 next to the asserted tolerances.
_PARITY = {}


@pytest.fixture(scope="session")
def parity_log():
    return _PARITY


def pytest_sessionfinish(session, exitstatus):
    if _PARITY:
        import json
        out = os.path.join(ROOT, "gpurun_out")
        os.makedirs(out, exist_ok=True)
        path = os.path.join(out, "parity_observed.json")
        old = {}
        if os.path.exists(path):
            try:
                old = json.load(open(path))
            except ValueError:
                old = {}
        old.update(_PARITY)
        json.dump(old, open(path, "w"), indent=1, sort_keys=True)


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
