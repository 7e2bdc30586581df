"""End-to-end drop-in: a checkpoint file on disk -> dropin create_model_and_diffusion -> forward on
the GPU, compared with the reference's own output for the same weights (golden full eval)."""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DROPIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                      "face-inpainting-diffusion-models_amd", "dropin")


def test_dropin_factory_checkpoint_roundtrip(tmp_path, evals):
    from ifd.manifest import make_state_dict
    from ifd.topology import FULL
    ck = tmp_path / "best_model.pt"
    torch.save({"model_state_dict": make_state_dict(FULL, seed=1), "epoch": 3}, ck)
    sys.path.insert(0, DROPIN)
    try:
        import train_inpainting
        model, diffusion, info = train_inpainting.create_model_and_diffusion(str(ck), torch.device("cuda:0"), 256)
    finally:
        sys.path.remove(DROPIN)
    assert not info["missing_keys"] and not info["unexpected_keys"]
    assert diffusion.num_timesteps == 1000
    dev = torch.device("cuda:0")
    x, gt, mask = (torch.from_numpy(evals[f"full/{k}"]).to(dev) for k in ("x", "gt", "mask"))
    with torch.no_grad():
        y = model(x, torch.tensor([999], device=dev), masked_image=gt * (1 - mask), mask=mask)
    err = float((y.cpu().double() - torch.from_numpy(evals["full_t999/y"]).double()).abs().max())
    assert err <= 2e-5, err
