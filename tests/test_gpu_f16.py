"""The reduced-precision sampler mode (precision="f16", include/ifd.h IFD_PREC_F16; SURVEY §8f rank 4,
the reference's `.half()` experiment code/test_quant.py:390-409), reported separately from the
fp32-class modes. Its error is measured against the reference fixtures and recorded; the gates are
f16-class: relative L2 error of one UNet eval < 1e-2, and the C2 DDIM-100 loop's pixel values
within 0.1 of the reference's (images in [-1, 1]).
"""
import numpy as np
import pytest
import torch

from conftest import golden_full
from ifd.manifest import make_state_dict
from ifd.topology import FULL

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


@pytest.fixture(scope="module")
def f16_model():
    from ifd.model import DiffusionInpaintingModel
    m = DiffusionInpaintingModel(FULL, device=DEV, precision="f16")
    m.load_state_dict(make_state_dict(FULL, seed=1))
    return m.eval()


def test_f16_unet_eval(evals, f16_model, record):
    x, gt, mask = (_t(evals[f"full/{k}"]).to(DEV) for k in ("x", "gt", "mask"))
    with torch.no_grad():
        y = f16_model(x, torch.tensor([999], device=DEV), masked_image=gt * (1 - mask), mask=mask)
    ref = _t(evals["full_t999/y"]).to(DEV)
    rel = float((y - ref).norm() / ref.norm())
    record("unet_full_t999/f16", maxabs=float((y - ref).abs().max()), rel_l2=rel)
    assert torch.isfinite(y).all() and rel < 1e-2


def test_f16_c2_loop(meta_full, f16_model, record):
    from test_gpu_full import _script_loop
    name = "c2_cos100_eta0.75"
    g = golden_full(name)
    y = _script_loop(f16_model, meta_full["loops"][name], _t(g["gt"]), _t(g["mask"]))
    d = (y.cpu().double() - _t(g["y"]).double()).abs()
    record(f"{name}/f16", maxabs=float(d.max()), mean=float(d.mean()), p999=float(d.flatten().quantile(0.999)))
    assert torch.isfinite(y).all() and float(d.max()) < 0.1
