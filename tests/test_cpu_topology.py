"""Host logic: state-dict spec, manifest regeneration, schedules, DDIM sequences, coefficients."""
import math

import numpy as np
import pytest
import torch

from ifd.topology import FULL, REDUCED, state_dict_spec, gflop_per_image
from ifd.manifest import make_state_dict, checksums
from ifd.schedules import get_named_beta_schedule, create_gaussian_diffusion


@pytest.mark.parametrize("name,cfg", [("reduced", REDUCED), ("full", FULL)])
def test_state_dict_spec_matches_reference(meta, name, cfg):
    ours = [[k, list(s)] for k, s in state_dict_spec(cfg)]
    assert ours == meta[f"keys_{name}"]


def test_param_count():
    assert sum(math.prod(s) for _, s in state_dict_spec(FULL)) == 93570822


@pytest.mark.parametrize("name,cfg", [("reduced", REDUCED)])
def test_manifest_regenerates(meta, name, cfg):
    cs = checksums(make_state_dict(cfg, seed=1))
    ref = meta[f"checksums_{name}"]
    for k, (s, s2) in cs.items():
        assert s == pytest.approx(ref[k][0], rel=0, abs=1e-9) and s2 == pytest.approx(ref[k][1], rel=0, abs=1e-9), k


def test_gflop_per_image():
    # 388.84 GFLOP per image per UNet eval (2*MAC, convs + attention + qkv/proj)
    assert gflop_per_image(FULL) == pytest.approx(388.84, abs=0.05)


def test_ddim_sequences(meta):
    from ifd.sampler import InpaintingSampler
    for key, seq in meta["ddim_sequences"].items():
        T, n = map(int, key.split("_"))
        assert [int(v) for v in InpaintingSampler.create_ddim_timestep_sequence(T, n)] == seq


def test_schedules(meta):
    for key, vals in meta["alphas_cumprod_samples"].items():
        sched, T = key.rsplit("_", 1)
        T = int(T)
        d = create_gaussian_diffusion(steps=T, learn_sigma=True, noise_schedule=sched)
        got = [float(d.alphas_cumprod[i]) for i in (0, 1, T // 2, T - 2, T - 1)]
        assert got == vals  # bit-exact float64


def test_ddim_coeffs_follow_torch_float64_semantics():
    """ifd.sampler.ddim_coeffs == the fp32 values torch produces from float64 0-dim tensors."""
    from ifd.sampler import ddim_coeffs, InpaintingSampler
    ac = create_gaussian_diffusion(steps=1000, learn_sigma=True, noise_schedule="cosine").alphas_cumprod
    seq = InpaintingSampler.create_ddim_timestep_sequence(1000, 10)
    one = torch.ones(1, dtype=torch.float32)
    for k, tau in enumerate(seq):
        eta = 0.9
        c = ddim_coeffs(ac, seq, k, eta)
        a_t = torch.tensor(ac[tau])
        a_p = torch.tensor(ac[seq[k + 1]]) if k < len(seq) - 1 else torch.tensor(1.0)
        sigma = eta * torch.sqrt((1 - a_p) / (1 - a_t)) * torch.sqrt(1 - a_t / a_p)
        assert float(one * torch.sqrt(1 - a_t)) == c.c_sqrt_1m_at
        assert float(one * torch.sqrt(a_t)) == c.c_sqrt_at
        assert float(one * torch.sqrt(a_p)) == c.c_sqrt_ap
        assert float(one * torch.sqrt(1 - a_p - sigma ** 2)) == c.c_dir
        assert float(one * sigma) == c.c_sigma
