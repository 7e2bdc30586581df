"""`GaussianDiffusion` with the reference's API (code/gaussian_diffusion.py:27-700).

Tables are float64 numpy (same formulas as code/gaussian_diffusion.py:47-80); per-timestep values
are gathered in float64 and rounded to fp32 once (`_extract_into_tensor`,
code/gaussian_diffusion.py:12-24).
The library loops (p_sample_loop / ddim_sample_loop and their _progressive forms) run each step's
algebra as two HIP kernels on GPU tensors (include/ifd.h ifd_lib_inject / ifd_lib_update): the
known-region injection before the model call and the DDIM / DDPM update after it, with the
step's coefficients taken on the host from the loop's own timestep, so there is no
`int(t[0].item())` sync per step. Direct calls of the per-step API (ddim_sample, p_sample,
apply_inpainting_injection, p_mean_variance, ...) with arbitrary t keep the reference's torch algebra.
The headline path (the scripts' DDIM / DDPM loops) does NOT go through here: it is fused into the
UNet's last conv by `ifd.sampler` (ifd_ddim_step / ifd_ddpm_step).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .losses import LossType, ModelMeanType, ModelVarType


def _f32(v):
    return float(np.float32(v))


def _extract_into_tensor(arr, timesteps, broadcast_shape):
    """float64 gather on the timesteps' device, then fp32 (code/gaussian_diffusion.py:12-24)."""
    res = torch.from_numpy(np.ascontiguousarray(arr)).to(device=timesteps.device)[timesteps].float()
    while res.dim() < len(broadcast_shape):
        res = res[..., None]
    return res.expand(broadcast_shape)


class GaussianDiffusion:
    def __init__(self, *, betas, model_mean_type, model_var_type, loss_type, rescale_timesteps=False):
        self.model_mean_type = model_mean_type
        self.model_var_type = model_var_type
        self.loss_type = loss_type
        self.rescale_timesteps = rescale_timesteps
        b = np.array(betas, dtype=np.float64)
        assert b.ndim == 1 and (b > 0).all() and (b <= 1).all()
        self.betas = b
        self.num_timesteps = int(b.shape[0])
        a = 1.0 - b
        ac = np.cumprod(a, axis=0)
        self.alphas_cumprod = ac
        self.alphas_cumprod_prev = np.append(1.0, ac[:-1])
        self.alphas_cumprod_next = np.append(ac[1:], 0.0)
        self.sqrt_alphas_cumprod = np.sqrt(ac)
        self.sqrt_one_minus_alphas_cumprod = np.sqrt(1.0 - ac)
        self.log_one_minus_alphas_cumprod = np.log(1.0 - ac)
        self.sqrt_recip_alphas_cumprod = np.sqrt(1.0 / ac)
        self.sqrt_recipm1_alphas_cumprod = np.sqrt(1.0 / ac - 1)
        self.posterior_variance = b * (1.0 - self.alphas_cumprod_prev) / (1.0 - ac)
        self.posterior_log_variance_clipped = np.log(np.append(self.posterior_variance[1], self.posterior_variance[1:]))
        self.posterior_mean_coef1 = b * np.sqrt(self.alphas_cumprod_prev) / (1.0 - ac)
        self.posterior_mean_coef2 = (1.0 - self.alphas_cumprod_prev) * np.sqrt(a) / (1.0 - ac)
        self._gt_noises_cache = {}
        # RNG placement: None draws on the tensors' device in the reference's order; a device
        # (e.g. "cpu") draws there in the same order and copies (reproduces CPU golden fixtures).
        self.noise_device = None

    def _randn_like(self, x):
        if self.noise_device is None or torch.device(self.noise_device) == x.device:
            return torch.randn_like(x)
        return torch.randn(x.shape, device=self.noise_device, dtype=x.dtype).to(x.device)

    def _randn(self, shape, device):
        if self.noise_device is None or torch.device(self.noise_device) == torch.device(device):
            return torch.randn(*shape, device=device)
        return torch.randn(*shape, device=self.noise_device).to(device)

    # ---- known-region injection (code/gaussian_diffusion.py:85-157) --------------------------
    def _gt_noise(self, gt, timestep):
        key = (gt.shape, timestep, gt.device)
        noise = self._gt_noises_cache.get(key)
        if noise is None:
            noise = self._randn_like(gt)
            self._gt_noises_cache[key] = noise
        return noise

    def get_gt_noised(self, gt, timestep):
        noise = self._gt_noise(gt, timestep)
        t = torch.tensor([timestep], device=gt.device).expand(gt.shape[0])
        return self.q_sample(gt, t, noise=noise)

    def clear_gt_noise_cache(self):
        self._gt_noises_cache.clear()

    def apply_inpainting_injection(self, x, t, gt, gt_keep_mask, use_cumulative_noise=True, injection_schedule="all",
                                   _tau=None):
        if gt is None or gt_keep_mask is None:
            return x
        tau = int(t[0].item()) if _tau is None else int(_tau)  # the library loops pass their host timestep
        half = self.num_timesteps // 2
        if (injection_schedule == "high" and tau < half) or (injection_schedule == "low" and tau >= half):
            return x
        B, C, H, W = x.shape
        if (_tau is not None and x.is_cuda and x.dtype == torch.float32 and gt.shape == x.shape
                and tuple(gt_keep_mask.shape) in ((B, 1, H, W), (1, 1, H, W))):
            # fused: keep * q_sample(gt) + (1 - keep) * x in one kernel (coefficients as _extract yields them)
            if use_cumulative_noise:
                noise = self._gt_noise(gt, tau)
                ca, cb = _f32(self.sqrt_alphas_cumprod[tau]), _f32(self.sqrt_one_minus_alphas_cumprod[tau])
            else:
                ac = np.float32(self.alphas_cumprod[tau])
                ca, cb = float(np.sqrt(ac)), float(np.sqrt(np.float32(1) - ac))
                noise = self._randn_like(gt)
            keep = gt_keep_mask.to(torch.float32).expand(B, 1, H, W).contiguous()
            out = torch.empty_like(x)
            xc, gc, nc = x.contiguous(), gt.to(torch.float32).contiguous(), noise.contiguous()
            _lib.check(_lib.lib().ifd_lib_inject(_lib.ptr(xc), _lib.ptr(gc), _lib.ptr(keep), _lib.ptr(nc), ca, cb, B, C, H,
                                                 W, _lib.ptr(out), _lib.stream_ptr(x.device)))
            return out
        if use_cumulative_noise:
            weighed = self.get_gt_noised(gt, tau)
        else:
            ac = _extract_into_tensor(self.alphas_cumprod, t, x.shape)
            weighed = torch.sqrt(ac) * gt + torch.sqrt(1 - ac) * self._randn_like(gt)
        keep = gt_keep_mask
        if keep.shape[1] == 1 and x.shape[1] > 1:
            keep = keep.repeat(1, x.shape[1], 1, 1)
        return keep * weighed + (1 - keep) * x

    # ---- forward process ---------------------------------------------------------------------
    def q_mean_variance(self, x_start, t):
        mean = _extract_into_tensor(self.sqrt_alphas_cumprod, t, x_start.shape) * x_start
        var = _extract_into_tensor(1.0 - self.alphas_cumprod, t, x_start.shape)
        logv = _extract_into_tensor(self.log_one_minus_alphas_cumprod, t, x_start.shape)
        return mean, var, logv

    def q_sample(self, x_start, t, noise=None):
        if noise is None:
            noise = self._randn_like(x_start)
        assert noise.shape == x_start.shape
        return (_extract_into_tensor(self.sqrt_alphas_cumprod, t, x_start.shape) * x_start
                + _extract_into_tensor(self.sqrt_one_minus_alphas_cumprod, t, x_start.shape) * noise)

    def q_posterior_mean_variance(self, x_start, x_t, t):
        assert x_start.shape == x_t.shape
        mean = (_extract_into_tensor(self.posterior_mean_coef1, t, x_t.shape) * x_start
                + _extract_into_tensor(self.posterior_mean_coef2, t, x_t.shape) * x_t)
        var = _extract_into_tensor(self.posterior_variance, t, x_t.shape)
        logv = _extract_into_tensor(self.posterior_log_variance_clipped, t, x_t.shape)
        return mean, var, logv

    # ---- reverse process ---------------------------------------------------------------------
    def p_mean_variance(self, model, x, t, clip_denoised=True, denoised_fn=None, model_kwargs=None):
        model_kwargs = model_kwargs or {}
        B, C = x.shape[:2]
        assert t.shape == (B,)
        out = model(x, self._scale_timesteps(t), **model_kwargs)
        if self.model_var_type in (ModelVarType.LEARNED, ModelVarType.LEARNED_RANGE):
            assert out.shape == (B, C * 2, *x.shape[2:])
            out, var_values = torch.split(out, C, dim=1)
            if self.model_var_type == ModelVarType.LEARNED:
                log_var = var_values
            else:
                min_log = _extract_into_tensor(self.posterior_log_variance_clipped, t, x.shape)
                max_log = _extract_into_tensor(np.log(self.betas), t, x.shape)
                frac = (var_values + 1) / 2
                log_var = frac * max_log + (1 - frac) * min_log
            var = torch.exp(log_var)
        else:
            table = {
                ModelVarType.FIXED_LARGE: np.append(self.posterior_variance[1], self.betas[1:]),
                ModelVarType.FIXED_SMALL: self.posterior_variance,
            }[self.model_var_type]
            log_table = {
                ModelVarType.FIXED_LARGE: np.log(np.append(self.posterior_variance[1], self.betas[1:])),
                ModelVarType.FIXED_SMALL: self.posterior_log_variance_clipped,
            }[self.model_var_type]
            var = _extract_into_tensor(table, t, x.shape)
            log_var = _extract_into_tensor(log_table, t, x.shape)

        def process(v):
            if denoised_fn is not None:
                v = denoised_fn(v)
            return v.clamp(-1, 1) if clip_denoised else v

        if self.model_mean_type == ModelMeanType.PREVIOUS_X:
            pred_xstart = process(self._predict_xstart_from_xprev(x_t=x, t=t, xprev=out))
            mean = out
        elif self.model_mean_type in (ModelMeanType.START_X, ModelMeanType.EPSILON):
            pred_xstart = process(out if self.model_mean_type == ModelMeanType.START_X
                                  else self._predict_xstart_from_eps(x_t=x, t=t, eps=out))
            mean, _, _ = self.q_posterior_mean_variance(x_start=pred_xstart, x_t=x, t=t)
        else:
            raise NotImplementedError(self.model_mean_type)
        assert mean.shape == log_var.shape == pred_xstart.shape == x.shape
        return {"mean": mean, "variance": var, "log_variance": log_var, "pred_xstart": pred_xstart}

    def _predict_xstart_from_eps(self, x_t, t, eps):
        assert x_t.shape == eps.shape
        return (_extract_into_tensor(self.sqrt_recip_alphas_cumprod, t, x_t.shape) * x_t
                - _extract_into_tensor(self.sqrt_recipm1_alphas_cumprod, t, x_t.shape) * eps)

    def _predict_xstart_from_xprev(self, x_t, t, xprev):
        assert x_t.shape == xprev.shape
        return (_extract_into_tensor(1.0 / self.posterior_mean_coef1, t, x_t.shape) * xprev
                - _extract_into_tensor(self.posterior_mean_coef2 / self.posterior_mean_coef1, t, x_t.shape) * x_t)

    def _predict_eps_from_xstart(self, x_t, t, pred_xstart):
        return ((_extract_into_tensor(self.sqrt_recip_alphas_cumprod, t, x_t.shape) * x_t - pred_xstart)
                / _extract_into_tensor(self.sqrt_recipm1_alphas_cumprod, t, x_t.shape))

    def _scale_timesteps(self, t):
        return t.float() * (1000.0 / self.num_timesteps) if self.rescale_timesteps else t

    def condition_mean(self, cond_fn, p_mean_var, x, t, model_kwargs=None):
        gradient = cond_fn(x, self._scale_timesteps(t), **(model_kwargs or {}))
        return p_mean_var["mean"].float() + p_mean_var["variance"] * gradient.float()

    def condition_score(self, cond_fn, p_mean_var, x, t, model_kwargs=None):
        alpha_bar = _extract_into_tensor(self.alphas_cumprod, t, x.shape)
        eps = self._predict_eps_from_xstart(x, t, p_mean_var["pred_xstart"])
        eps = eps - (1 - alpha_bar).sqrt() * cond_fn(x, self._scale_timesteps(t), **(model_kwargs or {}))
        out = p_mean_var.copy()
        out["pred_xstart"] = self._predict_xstart_from_eps(x, t, eps)
        out["mean"], _, _ = self.q_posterior_mean_variance(x_start=out["pred_xstart"], x_t=x, t=t)
        return out

    def _maybe_inject(self, x, t, model_kwargs, use_inpainting_injection, injection_schedule, use_cumulative_noise,
                      _tau=None):
        if use_inpainting_injection and model_kwargs:
            gt, keep = model_kwargs.get("gt"), model_kwargs.get("gt_keep_mask")
            if gt is not None and keep is not None:
                return self.apply_inpainting_injection(x, t, gt, keep, use_cumulative_noise=use_cumulative_noise,
                                                       injection_schedule=injection_schedule, _tau=_tau)
        return x

    def _fused_step(self, ddim, model, x, t, tau, clip_denoised, model_kwargs, eta=0.0):
        """One library-loop step's update as one HIP kernel (x and the model output on the GPU, EPSILON
        mean, LEARNED_RANGE variance). Draws the step noise in the reference's order (after the model)."""
        B, C, H, W = x.shape
        out = model(x, self._scale_timesteps(t), **(model_kwargs or {}))
        assert out.shape == (B, C * 2, H, W)
        noise = self._randn_like(x)
        c = _lib.LibCoeffs()
        c.c_recip, c.c_recipm1 = _f32(self.sqrt_recip_alphas_cumprod[tau]), _f32(self.sqrt_recipm1_alphas_cumprod[tau])
        c.c_ab, c.c_abp, c.c_eta = _f32(self.alphas_cumprod[tau]), _f32(self.alphas_cumprod_prev[tau]), _f32(eta)
        c.c_nonzero = 1.0 if tau != 0 else 0.0
        c.c_min_log, c.c_max_log = _f32(self.posterior_log_variance_clipped[tau]), _f32(np.log(self.betas)[tau])
        c.c_coef1, c.c_coef2 = _f32(self.posterior_mean_coef1[tau]), _f32(self.posterior_mean_coef2[tau])
        c.clip = int(bool(clip_denoised))
        xc, oc, nc = x.contiguous(), out.to(torch.float32).contiguous(), noise.contiguous()
        sample, pred = torch.empty_like(xc), torch.empty_like(xc)
        _lib.check(_lib.lib().ifd_lib_update(int(ddim), _lib.ptr(xc), _lib.ptr(oc), _lib.ptr(nc), B, H, W, c,
                                             _lib.ptr(sample), _lib.ptr(pred), _lib.stream_ptr(x.device)))
        return {"sample": sample, "pred_xstart": pred}

    def _can_fuse(self, x, cond_fn, denoised_fn, _tau):
        return (_tau is not None and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and x.shape[1] == 3
                and cond_fn is None and denoised_fn is None and self.model_mean_type == ModelMeanType.EPSILON
                and self.model_var_type == ModelVarType.LEARNED_RANGE)

    def p_sample(self, model, x, t, clip_denoised=True, denoised_fn=None, cond_fn=None, model_kwargs=None,
                 use_inpainting_injection=False, injection_schedule="all", use_cumulative_noise=True, _tau=None):
        x = self._maybe_inject(x, t, model_kwargs, use_inpainting_injection, injection_schedule, use_cumulative_noise,
                               _tau)
        if self._can_fuse(x, cond_fn, denoised_fn, _tau):
            return self._fused_step(False, model, x, t, int(_tau), clip_denoised, model_kwargs)
        out = self.p_mean_variance(model, x, t, clip_denoised=clip_denoised, denoised_fn=denoised_fn,
                                   model_kwargs=model_kwargs)
        noise = self._randn_like(x)
        nonzero = (t != 0).float().view(-1, *([1] * (x.dim() - 1)))
        if cond_fn is not None:
            out["mean"] = self.condition_mean(cond_fn, out, x, t, model_kwargs=model_kwargs)
        return {"sample": out["mean"] + nonzero * torch.exp(0.5 * out["log_variance"]) * noise,
                "pred_xstart": out["pred_xstart"]}

    def _progressive(self, step, model, shape, noise, device, progress, **kw):
        if device is None:
            device = next(model.parameters()).device
        assert isinstance(shape, (tuple, list))
        img = noise if noise is not None else self._randn(shape, device)
        indices = list(range(self.num_timesteps))[::-1]
        if progress:
            from tqdm.auto import tqdm
            indices = tqdm(indices)
        for i in indices:
            t = torch.tensor([i] * shape[0], device=device)
            with torch.no_grad():
                out = step(model, img, t, _tau=i, **kw)
                yield out
                img = out["sample"]

    def p_sample_loop(self, model, shape, noise=None, clip_denoised=True, denoised_fn=None, cond_fn=None,
                      model_kwargs=None, device=None, progress=False, use_inpainting_injection=False,
                      injection_schedule="all", use_cumulative_noise=True):
        self.clear_gt_noise_cache()
        final = None
        for s in self.p_sample_loop_progressive(model, shape, noise=noise, clip_denoised=clip_denoised,
                                                denoised_fn=denoised_fn, cond_fn=cond_fn, model_kwargs=model_kwargs,
                                                device=device, progress=progress,
                                                use_inpainting_injection=use_inpainting_injection,
                                                injection_schedule=injection_schedule,
                                                use_cumulative_noise=use_cumulative_noise):
            final = s
        return final["sample"]

    def p_sample_loop_progressive(self, model, shape, noise=None, clip_denoised=True, denoised_fn=None, cond_fn=None,
                                  model_kwargs=None, device=None, progress=False, use_inpainting_injection=False,
                                  injection_schedule="all", use_cumulative_noise=True):
        yield from self._progressive(self.p_sample, model, shape, noise, device, progress,
                                     clip_denoised=clip_denoised, denoised_fn=denoised_fn, cond_fn=cond_fn,
                                     model_kwargs=model_kwargs, use_inpainting_injection=use_inpainting_injection,
                                     injection_schedule=injection_schedule, use_cumulative_noise=use_cumulative_noise)

    def ddim_sample(self, model, x, t, clip_denoised=True, denoised_fn=None, cond_fn=None, model_kwargs=None, eta=0.0,
                    use_inpainting_injection=False, injection_schedule="all", use_cumulative_noise=True, _tau=None):
        x = self._maybe_inject(x, t, model_kwargs, use_inpainting_injection, injection_schedule, use_cumulative_noise,
                               _tau)
        if self._can_fuse(x, cond_fn, denoised_fn, _tau):
            return self._fused_step(True, model, x, t, int(_tau), clip_denoised, model_kwargs, eta)
        out = self.p_mean_variance(model, x, t, clip_denoised=clip_denoised, denoised_fn=denoised_fn,
                                   model_kwargs=model_kwargs)
        if cond_fn is not None:
            out = self.condition_score(cond_fn, out, x, t, model_kwargs=model_kwargs)
        eps = self._predict_eps_from_xstart(x, t, out["pred_xstart"])
        ab = _extract_into_tensor(self.alphas_cumprod, t, x.shape)
        abp = _extract_into_tensor(self.alphas_cumprod_prev, t, x.shape)
        sigma = eta * torch.sqrt((1 - abp) / (1 - ab)) * torch.sqrt(1 - ab / abp)
        noise = self._randn_like(x)
        mean = out["pred_xstart"] * torch.sqrt(abp) + torch.sqrt(1 - abp - sigma ** 2) * eps
        nonzero = (t != 0).float().view(-1, *([1] * (x.dim() - 1)))
        return {"sample": mean + nonzero * sigma * noise, "pred_xstart": out["pred_xstart"]}

    def ddim_sample_loop(self, model, shape, noise=None, clip_denoised=True, denoised_fn=None, cond_fn=None,
                         model_kwargs=None, device=None, progress=False, eta=0.0, use_inpainting_injection=False,
                         injection_schedule="all", use_cumulative_noise=True):
        self.clear_gt_noise_cache()
        final = None
        for s in self.ddim_sample_loop_progressive(model, shape, noise=noise, clip_denoised=clip_denoised,
                                                   denoised_fn=denoised_fn, cond_fn=cond_fn,
                                                   model_kwargs=model_kwargs, device=device, progress=progress,
                                                   eta=eta, use_inpainting_injection=use_inpainting_injection,
                                                   injection_schedule=injection_schedule,
                                                   use_cumulative_noise=use_cumulative_noise):
            final = s
        return final["sample"]

    def ddim_sample_loop_progressive(self, model, shape, noise=None, clip_denoised=True, denoised_fn=None,
                                     cond_fn=None, model_kwargs=None, device=None, progress=False, eta=0.0,
                                     use_inpainting_injection=False, injection_schedule="all",
                                     use_cumulative_noise=True):
        yield from self._progressive(self.ddim_sample, model, shape, noise, device, progress,
                                     clip_denoised=clip_denoised, denoised_fn=denoised_fn, cond_fn=cond_fn,
                                     model_kwargs=model_kwargs, eta=eta,
                                     use_inpainting_injection=use_inpainting_injection,
                                     injection_schedule=injection_schedule, use_cumulative_noise=use_cumulative_noise)

    def training_losses(self, model, x_start, t, model_kwargs=None, noise=None, use_injection=True,
                        injection_schedule="all", use_cumulative_noise=True):
        """Masked eps-MSE (code/gaussian_diffusion.py:540-614) with any model callable (forward only;
        the HIP training step with its backward is ifd.train.UNetTrainer.train_step)."""
        model_kwargs = model_kwargs or {}
        if noise is None:
            noise = self._randn_like(x_start)
        mask = model_kwargs.get("mask")
        masked_image = model_kwargs.get("masked_image")
        if mask is None:
            mask = torch.ones(x_start.shape[0], 1, x_start.shape[2], x_start.shape[3], device=x_start.device)
        x_t = self.q_sample(x_start, t, noise=noise)
        if use_injection and masked_image is not None:
            x_t = self.apply_inpainting_injection(x=x_t, t=t, gt=x_start, gt_keep_mask=1 - mask,
                                                  use_cumulative_noise=use_cumulative_noise,
                                                  injection_schedule=injection_schedule)
        if self.loss_type not in (LossType.MSE, LossType.RESCALED_MSE):
            raise NotImplementedError(f"Loss type {self.loss_type} not implemented for masking")
        out = model(x_t, self._scale_timesteps(t), **model_kwargs)
        if self.model_var_type in (ModelVarType.LEARNED, ModelVarType.LEARNED_RANGE):
            B, C = x_t.shape[:2]
            assert out.shape == (B, C * 2, *x_t.shape[2:])
            out, _ = torch.split(out, C, dim=1)
        m3 = mask.repeat(1, 3, 1, 1)
        area = torch.clamp(m3.sum(dim=[2, 3], keepdim=True), min=1.0)
        mse = (((noise - out) ** 2) * m3).sum(dim=[2, 3], keepdim=True) / area
        mse = mse.mean()
        if self.loss_type == LossType.RESCALED_MSE:
            mse = mse * self.num_timesteps
        return {"mse": mse, "loss": mse}

    def sample_with_advanced_inpainting(self, model, shape, gt=None, gt_keep_mask=None, use_ddim=True, eta=0.0,
                                        progress=True, device=None, injection_schedule="all",
                                        use_cumulative_noise=True):
        """code/gaussian_diffusion.py:640-700."""
        if device is None:
            device = next(model.parameters()).device
        model_kwargs = {}
        use_injection = False
        if gt is not None and gt_keep_mask is not None:
            model_kwargs = {"gt": gt, "gt_keep_mask": gt_keep_mask, "masked_image": gt * gt_keep_mask,
                            "mask": 1 - gt_keep_mask}
            use_injection = True
        fn = self.ddim_sample_loop if use_ddim else self.p_sample_loop
        kw = dict(eta=eta) if use_ddim else {}
        return fn(model=model, shape=shape, device=device, progress=progress, model_kwargs=model_kwargs,
                  use_inpainting_injection=use_injection, injection_schedule=injection_schedule,
                  use_cumulative_noise=use_cumulative_noise, **kw)
