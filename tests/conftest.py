import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parent.parent
PKG_ROOT = REPO / "lit-llama-ja_amd"
GOLDEN = Path(__file__).resolve().parent / "golden"

for p in (str(REPO), str(PKG_ROOT)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box with -m gpu)")


@pytest.fixture(scope="session")
def golden():
    cache = {}

    def load(name):
        if name not in cache:
            cache[name] = dict(np.load(GOLDEN / f"{name}.npz"))
        return cache[name]

    return load


@pytest.fixture(scope="session")
def hip():
    """The in-tree HIP library; GPU tests must run through it (no fallback)."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from lit_llama import _hip

    return _hip.lib()
