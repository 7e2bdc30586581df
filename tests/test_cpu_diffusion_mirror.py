"""The host `GaussianDiffusion` mirror (ifd/diffusion.py) against the reference class itself
(code/gaussian_diffusion.py:172-614), bit for bit, on the vectors tests/golden/make_golden_diffusion.py
recorded by importing the reference: p_mean_variance (all four dict entries, clip on/off), q_sample,
q_mean_variance, q_posterior_mean_variance, _predict_xstart_from_eps, _predict_eps_from_xstart and
training_losses (with the injection's GT-noise cache), schedules linear / cosine / quadratic, t pairs
[tau, 999 - tau] for tau in {0, 1, 500, 999}. CPU tensors: these are the reference's torch algebra
(the GPU loops fuse it into kernels, tested in tests/test_gpu_*.py)."""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden_diffusion as mk  # noqa: E402

GOLD = dict(np.load(os.path.join(HERE, "golden", "diffusion_mirror.npz")))


@pytest.mark.parametrize("schedule", mk.SCHEDULES)
@pytest.mark.parametrize("tau", mk.TAUS)
def test_diffusion_mirror_bit_exact(schedule, tau):
    from ifd.schedules import create_gaussian_diffusion
    diff = create_gaussian_diffusion(steps=1000, learn_sigma=True, noise_schedule=schedule)
    x, x0, noise, out6, mask = mk.inputs()
    got = mk.record(diff, out6, x, x0, noise, mask, tau)
    keys = [k for k in GOLD if k.startswith(f"{schedule}/t{tau}/")]
    assert len(keys) == len(got) >= 17
    for k in keys:
        name = k.split("/", 2)[2]
        assert np.array_equal(got[name], GOLD[k]), (k, float(np.abs(got[name] - GOLD[k]).max()))


def test_p_mean_variance_dict_and_shapes():
    """The returned dict has exactly the reference's keys; a wrong model-output width is rejected
    (code/gaussian_diffusion.py:238-242 asserts)."""
    from ifd.schedules import create_gaussian_diffusion
    diff = create_gaussian_diffusion(steps=1000, learn_sigma=True, noise_schedule="cosine")
    x, x0, noise, out6, mask = mk.inputs()
    t = torch.tensor([3, 4])
    pm = diff.p_mean_variance(lambda xx, tt, **kw: out6, x, t)
    assert set(pm) == {"mean", "variance", "log_variance", "pred_xstart"}
    with pytest.raises(AssertionError):
        diff.p_mean_variance(lambda xx, tt, **kw: out6[:, :3], x, t)
