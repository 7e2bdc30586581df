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
def meta_full():
    with open(os.path.join(GOLDEN, "full", "meta_full.json")) as f:
        return json.load(f)


def golden_full(name):
    return dict(np.load(os.path.join(GOLDEN, "full", f"{name}.npz")))


_RECORDED = {}


@pytest.fixture(scope="session")
def record():
    """record(key, **numbers): measured parity errors, written at session end to
    $IFD_PARITY_JSON (default gpurun_out/parity.json when gpurun_out/ exists) so the numbers the
    gates check are kept, not only printed."""
    def rec(key, **vals):
        _RECORDED[key] = {k: (float(v) if isinstance(v, (int, float, np.floating)) else v) for k, v in vals.items()}
        print(key, _RECORDED[key])
    yield rec
    path = os.environ.get("IFD_PARITY_JSON")
    if not path and os.path.isdir(os.path.join(ROOT, "gpurun_out")):
        path = os.path.join(ROOT, "gpurun_out", "parity.json")
    if path and _RECORDED:
        old = {}
        if os.path.exists(path):
            with open(path) as f:
                old = json.load(f)
        old.update(_RECORDED)
        with open(path, "w") as f:
            json.dump(old, f, indent=1, sort_keys=True)
