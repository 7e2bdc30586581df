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
  * `precision` selects the conv arithmetic ("3xf16": the split mode, DESIGN.md §3a, whose error
    against exact arithmetic matches the reference's own fp32 — tests/test_gpu_full.py — and whose
    range guard recomputes any out-of-range eval in fp32; "fp32": the plain fp32 MFMA chain);
    default from the IFD_PRECISION environment variable, else "fp32" (the reference's own
    arithmetic class, bit-comparable with earlier fp32 runs), so the reference's scripts can opt into
    "3xf16" without edits. The active mode is logged (logger "ifd") when the model is created.
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
    precision = precision or os.environ.get("IFD_PRECISION", "fp32")
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
