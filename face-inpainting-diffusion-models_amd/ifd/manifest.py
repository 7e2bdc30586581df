"""Seeded synthetic weights for the 9-channel UNet (no checkpoints exist offline).

Every parameter of `state_dict_spec(cfg)` is drawn from its own torch CPU generator,
seeded from (seed, index in state-dict order), so the same weights regenerate bit-identically
on any host with the same torch build. Rules (PyTorch-default-like scale, *all* layers
non-zero so the zero-initialised layers of code/nn.py:176,254 and code/unet.py:151 do not
make the model output exactly 0):

  conv / linear weight, fan_in = prod(shape[1:]):   U(-1/sqrt(fan_in), 1/sqrt(fan_in)) * gain
  conv / linear bias:                               U(-1/sqrt(fan_in), 1/sqrt(fan_in))
  GroupNorm weight / bias (1-D, GN keys):           1 + U(-0.1, 0.1) / U(-0.1, 0.1)

`gain` is 1 except for the layers the reference zero-initialises (out_layers.3, proj_out,
out.2), which get 0.5 to keep the residual stream O(1) over 30 ResBlocks.
"""
from __future__ import annotations

import math

import torch

from .topology import UNetConfig, FULL, state_dict_spec

_GN_TAGS = ("in_layers.0.", "out_layers.0.", ".norm.", "out.0.")
_ZERO_INIT_TAGS = ("out_layers.3.", "proj_out.", "out.2.")


def _is_gn(key):
    return any(tag in key for tag in _GN_TAGS) or key.startswith("out.0.") or ".out.0." in key


def _gen(seed, index):
    return torch.Generator().manual_seed(int(seed) * 1_000_003 + index)


def make_state_dict(cfg: UNetConfig = FULL, seed: int = 1, prefix: str = "base_model."):
    spec = state_dict_spec(cfg, prefix)
    fan_in = {}
    for key, shape in spec:
        if key.endswith(".weight") and len(shape) >= 2:
            fan_in[key[: -len(".weight")]] = math.prod(shape[1:])
    sd = {}
    for i, (key, shape) in enumerate(spec):
        g = _gen(seed, i)
        u = torch.rand(shape, generator=g, dtype=torch.float32) * 2 - 1
        stem = key.rsplit(".", 1)[0]
        if len(shape) == 1 and _is_gn(key):
            t = (1 + 0.1 * u) if key.endswith(".weight") else 0.1 * u
        else:
            bound = 1.0 / math.sqrt(fan_in[stem])
            gain = 0.5 if any(tag in key for tag in _ZERO_INIT_TAGS) and key.endswith(".weight") else 1.0
            t = u * (bound * gain)
        sd[key] = t.contiguous()
    return sd


def checksums(sd):
    """Per-tensor (sum, sum of squares) in float64, for cross-host regeneration checks."""
    return {k: (float(v.double().sum()), float((v.double() ** 2).sum())) for k, v in sd.items()}
