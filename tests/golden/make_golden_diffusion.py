"""Golden vectors for the host `GaussianDiffusion` mirror (ifd/diffusion.py), made by importing the
reference's own class (code/gaussian_diffusion.py) in the build container.

Run here (not on the GPU box — /root/reference does not travel):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_diffusion.py

For each schedule (linear / cosine / quadratic, T=1000, LEARNED_RANGE, EPSILON, MSE, the factory's
create_gaussian_diffusion, code/utils/schedules.py:69-106) and each timestep pair t = [tau, 999 - tau]
with tau in {0, 1, 500, 999}, on seeded CPU inputs (B=2, 3x8x8) and a stub model that returns a fixed
seeded [B,6,H,W] output, records the reference's
  * p_mean_variance (:213-298): mean, variance, log_variance, pred_xstart (clip_denoised True/False)
  * q_sample (:172-189), q_mean_variance, q_posterior_mean_variance (:191-211)
  * _predict_xstart_from_eps (:300-305), _predict_eps_from_xstart (:316-319)
  * training_losses (:540-614) with injection (its GT-noise cache drawn after torch.manual_seed)
into golden/diffusion_mirror.npz. tests/test_cpu_diffusion_mirror.py compares ifd's mirror bit for bit.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/code"
SCHEDULES = ("linear", "cosine", "quadratic")
TAUS = (0, 1, 500, 999)


def inputs():
    g = torch.Generator().manual_seed(2024)
    x = torch.randn(2, 3, 8, 8, generator=g)
    x0 = torch.rand(2, 3, 8, 8, generator=g) * 2 - 1
    noise = torch.randn(2, 3, 8, 8, generator=g)
    out6 = torch.cat([torch.randn(2, 3, 8, 8, generator=g), torch.rand(2, 3, 8, 8, generator=g) * 2 - 1], 1)
    mask = (torch.rand(2, 1, 8, 8, generator=g) > 0.5).float()
    return x, x0, noise, out6, mask


def record(diff, out6, x, x0, noise, mask, tau):
    """Every recorded quantity of one (diffusion, tau) case, as name -> fp32 numpy array."""
    t = torch.tensor([tau, 999 - tau], dtype=torch.int64)

    def model(xx, tt, **kw):
        return out6.clone()
    res = {}
    for clip in (True, False):
        pm = diff.p_mean_variance(model, x, t, clip_denoised=clip, model_kwargs={"gt": x0})
        for k in ("mean", "variance", "log_variance", "pred_xstart"):
            res[f"pmv_clip{int(clip)}/{k}"] = pm[k]
    res["q_sample"] = diff.q_sample(x0, t, noise=noise)
    for k, v in zip(("mean", "variance", "log_variance"), diff.q_mean_variance(x0, t)):
        res[f"qmv/{k}"] = v
    for k, v in zip(("mean", "variance", "log_variance"), diff.q_posterior_mean_variance(x0, x, t)):
        res[f"qpost/{k}"] = v
    res["xstart_from_eps"] = diff._predict_xstart_from_eps(x, t, out6[:, :3])
    res["eps_from_xstart"] = diff._predict_eps_from_xstart(x, t, x0)
    diff.clear_gt_noise_cache()
    torch.manual_seed(77 + tau)
    tl = diff.training_losses(model, x0, t, model_kwargs={"mask": mask, "masked_image": x0 * (1 - mask)},
                              noise=noise)
    res["training_losses/loss"] = tl["loss"].reshape(1)
    return {k: v.detach().to(torch.float32).numpy() for k, v in res.items()}


def main():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    from utils import schedules as r_sched
    x, x0, noise, out6, mask = inputs()
    out = {}
    for sch in SCHEDULES:
        diff = r_sched.create_gaussian_diffusion(steps=1000, learn_sigma=True, noise_schedule=sch)
        for tau in TAUS:
            for k, v in record(diff, out6, x, x0, noise, mask, tau).items():
                out[f"{sch}/t{tau}/{k}"] = v
    np.savez_compressed(os.path.join(HERE, "diffusion_mirror.npz"), **out)
    print(f"wrote {len(out)} arrays")


if __name__ == "__main__":
    main()
