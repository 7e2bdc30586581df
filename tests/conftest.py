import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "face-inpainting-diffusion-models_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def meta():
    with open(os.path.join(GOLDEN, "meta.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def evals():
    return dict(np.load(os.path.join(GOLDEN, "unet_evals.npz")))


@pytest.fixture(scope="session")
def loops():
    return dict(np.load(os.path.join(GOLDEN, "loops.npz")))


@pytest.fixture(scope="session")
def layers():
    return dict(np.load(os.path.join(GOLDEN, "layers.npz")))
