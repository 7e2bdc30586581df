"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference's diffusion arithmetic on the inpainting hot path:
beta schedules, the float64 coefficient tables, `p_mean_variance` (LEARNED_RANGE / EPSILON),
the script DDIM / DDPM loops with post-update known-region re-injection, the library
`ddim_sample_loop` / `p_sample_loop` with pre-model injection, and the final blend.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.

Reference citations (paths relative to the reference repository root):
  code/utils/schedules.py:9-66        get_named_beta_schedule, betas_for_alpha_bar
  code/gaussian_diffusion.py:12-24    _extract_into_tensor (index float64, then .float())
  code/gaussian_diffusion.py:41-83    coefficient tables
  code/gaussian_diffusion.py:85-157   get_gt_noised / apply_inpainting_injection
  code/gaussian_diffusion.py:172-189  q_sample
  code/gaussian_diffusion.py:191-305  q_posterior_mean_variance, p_mean_variance, x0-from-eps
  code/gaussian_diffusion.py:357-538  p_sample(_loop), ddim_sample(_loop)
  code/test_inp_ddim_50.py:373-385    model_fn
  code/test_inp_ddim_50.py:387-400    create_ddim_timestep_sequence
  code/test_inp_ddim_50.py:402-468    inpainting_p_sample_loop (script DDPM)
  code/test_inp_ddim_50.py:470-576    inpainting_ddim_sample_loop (script DDIM)
  code/test_inp_ddim_50.py:692-696    final blend

RNG: every draw uses the global torch CPU generator in exactly the reference's call order,
so fixtures regenerate bit-identically from a seed. Draws are always fp32 (`_randn`), so an fp64
model (the error-envelope fixtures) sees the same noise values as the fp32 reference.
"""
from __future__ import annotations

import math

import numpy as np
import torch


def get_named_beta_schedule(name, T):
    """code/utils/schedules.py:9-46."""
    if name == "linear":
        s = 1000 / T
        return np.linspace(s * 0.0001, s * 0.02, T, dtype=np.float64)
    if name == "cosine":
        f = lambda u: math.cos((u + 0.008) / 1.008 * math.pi / 2) ** 2
        return np.array([min(1 - f((i + 1) / T) / f(i / T), 0.999) for i in range(T)])
    if name == "quadratic":
        s = 1000 / T
        b0, b1 = s * 0.0001, s * 0.02
        u = np.linspace(0, 1, T, dtype=np.float64)
        return b0 + (b1 - b0) * u ** 2
    if name in ("sqrt_linear", "sqrt"):
        return np.sqrt(np.linspace(0.0001, 0.02, T, dtype=np.float64))
    raise NotImplementedError(name)


class Tables:
    """float64 tables of code/gaussian_diffusion.py:47-80."""

    def __init__(self, betas):
        b = np.array(betas, dtype=np.float64)
        self.betas = b
        self.T = len(b)
        a = 1.0 - b
        self.ac = np.cumprod(a)
        self.ac_prev = np.append(1.0, self.ac[:-1])
        self.sqrt_ac = np.sqrt(self.ac)
        self.sqrt_1m_ac = np.sqrt(1.0 - self.ac)
        self.sqrt_recip_ac = np.sqrt(1.0 / self.ac)
        self.sqrt_recipm1_ac = np.sqrt(1.0 / self.ac - 1)
        self.post_var = b * (1.0 - self.ac_prev) / (1.0 - self.ac)
        self.post_logvar_clipped = np.log(np.append(self.post_var[1], self.post_var[1:]))
        self.coef1 = b * np.sqrt(self.ac_prev) / (1.0 - self.ac)
        self.coef2 = (1.0 - self.ac_prev) * np.sqrt(a) / (1.0 - self.ac)
        self.log_betas = np.log(b)


def extract(arr, t, shape):
    """code/gaussian_diffusion.py:12-24: float64 gather, then fp32, broadcast."""
    res = torch.from_numpy(arr)[t].float()
    while res.dim() < len(shape):
        res = res[..., None]
    return res.expand(shape)


def q_sample(tb, x0, t, noise):
    """code/gaussian_diffusion.py:172-189."""
    return extract(tb.sqrt_ac, t, x0.shape) * x0 + extract(tb.sqrt_1m_ac, t, x0.shape) * noise


def p_mean_variance(tb, model, x, t, clip=True, model_kwargs=None):
    """code/gaussian_diffusion.py:213-298 for EPSILON mean, LEARNED_RANGE variance."""
    model_kwargs = model_kwargs or {}
    B, C = x.shape[:2]
    out = model(x, t, **model_kwargs)
    eps, v = torch.split(out, C, dim=1)
    min_log = extract(tb.post_logvar_clipped, t, x.shape)
    max_log = extract(tb.log_betas, t, x.shape)
    frac = (v + 1) / 2
    logvar = frac * max_log + (1 - frac) * min_log
    x0 = extract(tb.sqrt_recip_ac, t, x.shape) * x - extract(tb.sqrt_recipm1_ac, t, x.shape) * eps
    if clip:
        x0 = x0.clamp(-1, 1)
    mean = extract(tb.coef1, t, x.shape) * x0 + extract(tb.coef2, t, x.shape) * x
    return {"mean": mean, "variance": torch.exp(logvar), "log_variance": logvar, "pred_xstart": x0}


def model_fn_factory(unet_call):
    """code/test_inp_ddim_50.py:373-385: build masked image / inpaint mask from gt, keep."""
    def model_fn(x, t, gt=None, gt_keep_mask=None, **kw):
        masked = gt * gt_keep_mask + torch.zeros_like(gt) * (1 - gt_keep_mask)
        return unet_call(x, t, masked, 1 - gt_keep_mask)
    return model_fn


def ddim_timestep_sequence(T, n):
    """code/test_inp_ddim_50.py:387-400."""
    c = T // n
    seq = np.asarray(list(range(0, T, c)))
    if seq[-1] != T - 1:
        seq = np.append(seq, T - 1)
    return seq[::-1]


def _randn(like):
    """torch.randn_like for an fp32 tensor; fp32 draws cast up for an fp64 one."""
    return torch.randn(like.shape).to(like.dtype)


def script_ddim_loop(tb, model_fn, shape, gt, masks, ddim_steps, clip=True, eta=0.0):
    """code/test_inp_ddim_50.py:470-576 (post-update injection at alpha_prev, fresh noise)."""
    img = torch.randn(*shape)
    seq = ddim_timestep_sequence(tb.T, ddim_steps)
    keep = 1 - masks
    for k, tau in enumerate(seq):
        t = torch.tensor([tau] * shape[0])
        out = model_fn(img, t, gt=gt, gt_keep_mask=keep)
        eps = out[:, :3] if out.shape[1] == 6 else out
        a_t = torch.tensor(tb.ac[tau])                       # float64 0-dim tensors (:533-534)
        a_p = torch.tensor(tb.ac[seq[k + 1]]) if k < len(seq) - 1 else torch.tensor(1.0)
        x0 = (img - torch.sqrt(1 - a_t) * eps) / torch.sqrt(a_t)
        if clip:
            x0 = torch.clamp(x0, -1, 1)
        sigma = eta * torch.sqrt((1 - a_p) / (1 - a_t)) * torch.sqrt(1 - a_t / a_p)
        pred_dir = torch.sqrt(1 - a_p - sigma ** 2) * eps
        noise = _randn(img) if tau > 0 and eta > 0 else torch.zeros_like(img)
        img = torch.sqrt(a_p) * x0 + pred_dir + sigma * noise
        if tau > 0:
            known = _randn(gt)
            img = img * masks + (torch.sqrt(a_p) * gt + torch.sqrt(1 - a_p) * known) * keep
    return img


def script_ddpm_loop(tb, model_fn, shape, gt, masks, clip=True):
    """code/test_inp_ddim_50.py:402-468 (script DDPM, injection at alpha_cumprod[i-1])."""
    img = torch.randn(*shape)
    keep = 1 - masks
    for i in range(tb.T)[::-1]:
        t = torch.tensor([i] * shape[0])
        out = p_mean_variance(tb, model_fn, img, t, clip, {"gt": gt, "gt_keep_mask": keep})
        noise = _randn(img)
        nonzero = (t != 0).float().view(-1, 1, 1, 1)
        img = out["mean"] + nonzero * torch.exp(0.5 * out["log_variance"]) * noise
        if i > 0:
            a = torch.tensor(tb.ac[i - 1])
            known = _randn(gt)
            img = img * masks + (torch.sqrt(a) * gt + torch.sqrt(1 - a) * known) * keep
    return img


def final_blend(result, gt, masks):
    """code/test_inp_ddim_50.py:692-696."""
    return result * masks + gt * (1 - masks)


# ---- library loops (code/gaussian_diffusion.py:85-157, 357-538) ----

class LibraryState:
    def __init__(self, tb):
        self.tb = tb
        self.cache = {}

    def gt_noised(self, gt, tau):
        key = (tuple(gt.shape), tau)
        if key not in self.cache:
            self.cache[key] = _randn(gt)
        t = torch.tensor([tau]).expand(gt.shape[0])
        return q_sample(self.tb, gt, t, self.cache[key])

    def inject(self, x, t, gt, keep, schedule="all", cumulative=True):
        tau = int(t[0].item())
        T = self.tb.T
        if schedule == "high" and tau < T // 2:
            return x
        if schedule == "low" and tau >= T // 2:
            return x
        if cumulative:
            w = self.gt_noised(gt, tau)
        else:
            ac = extract(self.tb.ac, t, x.shape)
            w = torch.sqrt(ac) * gt + torch.sqrt(1 - ac) * _randn(gt)
        if keep.shape[1] == 1 and x.shape[1] > 1:
            keep = keep.repeat(1, x.shape[1], 1, 1)
        return keep * w + (1 - keep) * x


def library_ddim_loop(tb, model, shape, model_kwargs, eta=0.0, clip=True, injection=True,
                      schedule="all", cumulative=True, noise=None):
    st = LibraryState(tb)
    img = noise if noise is not None else torch.randn(*shape)
    for i in range(tb.T)[::-1]:
        t = torch.tensor([i] * shape[0])
        x = img
        if injection and model_kwargs:
            x = st.inject(x, t, model_kwargs["gt"], model_kwargs["gt_keep_mask"], schedule, cumulative)
        out = p_mean_variance(tb, model, x, t, clip, model_kwargs)
        eps = (extract(tb.sqrt_recip_ac, t, x.shape) * x - out["pred_xstart"]) / extract(tb.sqrt_recipm1_ac, t, x.shape)
        ab = extract(tb.ac, t, x.shape)
        abp = extract(tb.ac_prev, t, x.shape)
        sigma = eta * torch.sqrt((1 - abp) / (1 - ab)) * torch.sqrt(1 - ab / abp)
        nz = _randn(x)
        mean = out["pred_xstart"] * torch.sqrt(abp) + torch.sqrt(1 - abp - sigma ** 2) * eps
        nonzero = (t != 0).float().view(-1, 1, 1, 1)
        img = mean + nonzero * sigma * nz
    return img


def library_ddpm_loop(tb, model, shape, model_kwargs, clip=True, injection=True,
                      schedule="all", cumulative=True, noise=None):
    st = LibraryState(tb)
    img = noise if noise is not None else torch.randn(*shape)
    for i in range(tb.T)[::-1]:
        t = torch.tensor([i] * shape[0])
        x = img
        if injection and model_kwargs:
            x = st.inject(x, t, model_kwargs["gt"], model_kwargs["gt_keep_mask"], schedule, cumulative)
        out = p_mean_variance(tb, model, x, t, clip, model_kwargs)
        nz = _randn(x)
        nonzero = (t != 0).float().view(-1, 1, 1, 1)
        img = out["mean"] + nonzero * torch.exp(0.5 * out["log_variance"]) * nz
    return img
