"""Beta schedules and the diffusion factory (mirror of code/utils/schedules.py:9-106).

Host-side float64 numpy, exactly the reference's formulas (the tables feed float64 -> fp32
coefficients; nothing here runs per pixel).
"""
from __future__ import annotations

import math

import numpy as np


def get_named_beta_schedule(schedule_name, num_diffusion_timesteps):
    """code/utils/schedules.py:9-46."""
    T = num_diffusion_timesteps
    if schedule_name == "linear":
        scale = 1000 / T
        return np.linspace(scale * 0.0001, scale * 0.02, T, dtype=np.float64)
    if schedule_name == "cosine":
        return betas_for_alpha_bar(T, lambda t: math.cos((t + 0.008) / 1.008 * math.pi / 2) ** 2)
    if schedule_name == "quadratic":
        scale = 1000 / T
        lo, hi = scale * 0.0001, scale * 0.02
        return lo + (hi - lo) * np.linspace(0, 1, T, dtype=np.float64) ** 2
    if schedule_name in ("sqrt_linear", "sqrt"):
        return np.sqrt(np.linspace(0.0001, 0.02, T, dtype=np.float64))
    raise NotImplementedError(f"unknown beta schedule: {schedule_name}")


def betas_for_alpha_bar(num_diffusion_timesteps, alpha_bar, max_beta=0.999):
    """code/utils/schedules.py:49-66."""
    out = []
    for i in range(num_diffusion_timesteps):
        t1, t2 = i / num_diffusion_timesteps, (i + 1) / num_diffusion_timesteps
        out.append(min(1 - alpha_bar(t2) / alpha_bar(t1), max_beta))
    return np.array(out)


def create_gaussian_diffusion(*, steps=1000, learn_sigma=False, sigma_small=False, noise_schedule="linear",
                              use_kl=False, predict_xstart=False, rescale_timesteps=False,
                              rescale_learned_sigmas=False, timestep_respacing=""):
    """code/utils/schedules.py:69-106 (timestep_respacing is accepted and ignored, as there)."""
    from .diffusion import GaussianDiffusion
    from .losses import LossType, ModelMeanType, ModelVarType

    betas = get_named_beta_schedule(noise_schedule, steps)
    if use_kl:
        loss_type = LossType.RESCALED_KL if rescale_learned_sigmas else LossType.KL
    else:
        loss_type = LossType.RESCALED_MSE if rescale_learned_sigmas else LossType.MSE
    return GaussianDiffusion(
        betas=betas,
        model_mean_type=ModelMeanType.START_X if predict_xstart else ModelMeanType.EPSILON,
        model_var_type=(ModelVarType.LEARNED_RANGE if learn_sigma
                        else (ModelVarType.FIXED_SMALL if sigma_small else ModelVarType.FIXED_LARGE)),
        loss_type=loss_type,
        rescale_timesteps=rescale_timesteps,
    )
