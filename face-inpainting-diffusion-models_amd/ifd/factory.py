"""`create_model_and_diffusion` (code/train_inpainting.py:199-262, code/train_inpainting_ddpm.py:199-262).

Same signature and return value `(model, diffusion, {'missing_keys', 'unexpected_keys'})`.
Differences, all deliberate:
  * checkpoints are read with `torch.load(..., weights_only=True)` (state-dict checkpoints load
    the same; arbitrary pickles are refused);
  * `checkpoint_path=None` gives the seeded synthetic weights of `ifd.manifest` (no checkpoints
    exist offline);
  * a base (3-channel) checkpoint is widened to 9 input channels as DiffusionInpaintingModel does
    (code/unet.py:184-195): RGB weights copied to channels 0:3, zeros in 3:9, and the new conv's
    bias default-initialised from the global torch RNG (U(+-1/sqrt(fan_in)), as nn.Conv2d does —
    the exact RNG stream of the reference's module construction is not reproduced).
  * `noise_schedule` / `steps` are keyword overrides (defaults = the reference factory's).
  * `precision` selects the conv arithmetic: "3xf16" (the default) or "fp32"; the IFD_PRECISION
    environment variable overrides the default, so the reference's scripts switch without edits. The
    active mode is logged (logger "ifd") when the model is created.
    Why 3xf16 is the default: it is the MORE accurate of the two against exact arithmetic. Its products
    are exact and its hi x hi sums go into one fp32 accumulator while the correction products go into a
    second one, so per UNet eval its error against an fp64 UNet is within ~1.2x of the
    reference's own fp32 (oneDNN) error (tests/test_gpu_full.py::test_c1_eval_error_vs_fp64). "fp32" runs
    v_mfma_f32_32x32x2_f32, an fp32 FMA chain over K = 9 Cin terms with one rounding per product: ~2.6x
    the reference's error (tools/diag/acc_model.py reproduces both ratios on the CPU). Out-of-range
    split operands trip the range guard and the eval is recomputed in fp32.
"""
from __future__ import annotations

import logging
import math
import os

import torch

from .manifest import make_state_dict
from .model import DiffusionInpaintingModel
from .schedules import create_gaussian_diffusion
from .topology import UNetConfig


def _unwrap(ckpt):
    if isinstance(ckpt, dict):
        for k in ("state_dict", "model", "model_state_dict"):
            if k in ckpt and isinstance(ckpt[k], dict):
                return ckpt[k]
    return ckpt


def create_model_and_diffusion(checkpoint_path, device, img_size=256, *, steps=1000, noise_schedule="quadratic",
                               model_channels=128, seed=1, precision=None):
    cfg = UNetConfig(image_size=img_size, model_channels=model_channels)
    precision = precision or os.environ.get("IFD_PRECISION", "3xf16")
    logging.getLogger("ifd").info("create_model_and_diffusion: conv arithmetic %s (IFD_PRECISION)", precision)
    model = DiffusionInpaintingModel(cfg, device=device, precision=precision)
    if checkpoint_path is None:
        sd = make_state_dict(cfg, seed=seed, prefix="base_model.")
    else:
        sd = _unwrap(torch.load(checkpoint_path, map_location="cpu", weights_only=True))
        sd = {(k if k.startswith("base_model.") else "base_model." + k): v for k, v in sd.items()}
        w_key = "base_model.input_blocks.0.0.weight"
        if w_key in sd and sd[w_key].shape[1] == 3:
            w3 = sd[w_key]
            w9 = torch.zeros(w3.shape[0], 9, *w3.shape[2:], dtype=w3.dtype)
            w9[:, :3] = w3
            sd[w_key] = w9
            bound = 1.0 / math.sqrt(9 * w3.shape[2] * w3.shape[3])
            sd["base_model.input_blocks.0.0.bias"] = torch.empty(w3.shape[0]).uniform_(-bound, bound)
    missing, unexpected = model.load_state_dict(sd, strict=False)
    model.eval()
    diffusion = create_gaussian_diffusion(steps=steps, learn_sigma=True, noise_schedule=noise_schedule, use_kl=False,
                                          predict_xstart=False, rescale_timesteps=False)
    return model, diffusion, {"missing_keys": missing, "unexpected_keys": unexpected}
