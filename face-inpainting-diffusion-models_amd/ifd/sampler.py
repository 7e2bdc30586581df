"""The scripts' inpainting sampler (code/test_inp_ddim_50.py:288-698) on the fused HIP path.

`InpaintingSampler.inpainting_ddim_sample_loop` / `inpainting_p_sample_loop` keep the reference's
signatures, RNG draw order and arithmetic. When `model_fn` is this sampler's own `model_fn` and
the model is the HIP `DiffusionInpaintingModel`, each iteration is ONE library call
(`ifd_ddim_step` / `ifd_ddpm_step`): input assembly (model_fn), the UNet, and the DDIM / DDPM
update + known-region re-injection fused into the epilogue of the final conv, updating `img` in
place. Otherwise the model output is computed by `model_fn` and the update runs as one fused
elementwise kernel (`ifd_ddim_update` / `ifd_ddpm_update`).

Coefficients follow torch's semantics in the reference loop: float64 0-dim tensors combined in
float64, rounded to fp32 once when they meet an fp32 tensor.

RNG: every draw happens in reference order on `noise_device` (default: the sampling device, as
the reference does); `noise_device="cpu"` draws from the global CPU generator and uploads, which
reproduces CPU-generated golden fixtures bit-for-bit in the noise. `noise_shard=(lo, hi, B)` is
the multi-GPU parity mode: every draw is made for the FULL batch of B images in
reference order and rows lo:hi are kept, so a rank's images see exactly the noise they would in an
unsharded run (results independent of the GPU count).

Shapes: gt must be [B,3,H,W] and masks [B,1,H,W] (1 = hole), or broadcastable to them along the
batch (a [1,...] tensor is expanded); anything else raises ValueError before a kernel is launched.
"""
from __future__ import annotations

import math
from types import SimpleNamespace

import numpy as np
import torch

from . import _lib
from .model import DiffusionInpaintingModel


def _f32(v):
    return float(np.float32(v))


def ddim_coeffs(alphas_cumprod, seq, k, eta, clip=True):
    """Per-step DDIM coefficients of code/test_inp_ddim_50.py:523-571 as an ifd_step_coeffs."""
    tau = int(seq[k])
    a_t = float(alphas_cumprod[tau])
    last = k >= len(seq) - 1
    a_p = 1.0 if last else float(alphas_cumprod[int(seq[k + 1])])
    sigma = eta * math.sqrt((1 - a_p) / (1 - a_t)) * math.sqrt(1 - a_t / a_p)
    c = _lib.StepCoeffs()
    c.c_sqrt_1m_at = _f32(math.sqrt(1 - a_t))
    c.c_sqrt_at = _f32(math.sqrt(a_t))
    c.c_sqrt_ap = _f32(math.sqrt(a_p))
    c.c_dir = _f32(math.sqrt(1 - a_p - sigma ** 2))
    c.c_sigma = _f32(sigma)
    c.use_noise = int(tau > 0 and eta > 0)
    c.inject = int(tau > 0)
    c.c_inj_a = _f32(math.sqrt(a_p))
    c.c_inj_b = _f32(math.sqrt(1 - a_p))
    c.clip = int(bool(clip))
    return c


def ddpm_coeffs(diffusion, i, clip=True):
    """Per-step DDPM coefficients: p_mean_variance (code/gaussian_diffusion.py:241-286, LEARNED_RANGE,
    EPSILON) + the script update and injection (code/test_inp_ddim_50.py:442-466)."""
    c = _lib.StepCoeffs()
    c.c_min_log = _f32(diffusion.posterior_log_variance_clipped[i])
    c.c_max_log = _f32(np.log(diffusion.betas)[i])
    c.c_recip = _f32(diffusion.sqrt_recip_alphas_cumprod[i])
    c.c_recipm1 = _f32(diffusion.sqrt_recipm1_alphas_cumprod[i])
    c.c_coef1 = _f32(diffusion.posterior_mean_coef1[i])
    c.c_coef2 = _f32(diffusion.posterior_mean_coef2[i])
    c.c_nonzero = 1.0 if i != 0 else 0.0
    c.inject = int(i > 0)
    if i > 0:
        a = float(diffusion.alphas_cumprod[i - 1])
        c.c_inj_a = _f32(math.sqrt(a))
        c.c_inj_b = _f32(math.sqrt(1 - a))
    c.use_noise = 1
    c.clip = int(bool(clip))
    return c


def prepare_gt_mask(gt, masks, B, H, W, device):
    """gt -> contiguous fp32 [B,3,H,W], masks -> [B,1,H,W] on `device`; a batch-1 tensor is
    expanded (the reference broadcasts it). The kernels index exactly these shapes."""
    gt = torch.as_tensor(gt)
    masks = torch.as_tensor(masks)
    if gt.dim() != 4 or gt.shape[1:] != (3, H, W) or gt.shape[0] not in (1, B):
        raise ValueError(f"gt must be [{B},3,{H},{W}] (or batch 1), got {tuple(gt.shape)}")
    if masks.dim() != 4 or masks.shape[1:] != (1, H, W) or masks.shape[0] not in (1, B):
        raise ValueError(f"masks must be [{B},1,{H},{W}] (or batch 1), got {tuple(masks.shape)}")
    gt = gt.to(device=device, dtype=torch.float32).expand(B, 3, H, W).contiguous()
    masks = masks.to(device=device, dtype=torch.float32).expand(B, 1, H, W).contiguous()
    return gt, masks


class InpaintingSampler:
    """Sampling core of the reference's `InpaintingSampler` (no dataset / metrics / IO)."""

    def __init__(self, model, diffusion, ddim_timesteps=100, device=None, noise_device=None, args=None,
                 noise_shard=None):
        self.model = model
        self.diffusion = diffusion
        self.args = args if args is not None else SimpleNamespace(ddim_timesteps=ddim_timesteps)
        self.device = device if device is not None else next(model.parameters()).device
        self.noise_device = noise_device
        if noise_shard is not None:
            lo, hi, gb = (int(v) for v in noise_shard)
            if not 0 <= lo < hi <= gb:
                raise ValueError(f"noise_shard must satisfy 0 <= lo < hi <= B, got {noise_shard}")
            noise_shard = (lo, hi, gb)
        self.noise_shard = noise_shard

    # code/test_inp_ddim_50.py:373-385
    def model_fn(self, x, t, gt=None, gt_keep_mask=None, **kwargs):
        if gt is None or gt_keep_mask is None:
            raise ValueError("Ground truth and mask required for inpainting")
        masked_image = gt * gt_keep_mask + torch.zeros_like(gt) * (1 - gt_keep_mask)
        return self.model(x, t, masked_image=masked_image, mask=1 - gt_keep_mask)

    # code/test_inp_ddim_50.py:387-400
    @staticmethod
    def create_ddim_timestep_sequence(total_timesteps, ddim_timesteps):
        c = total_timesteps // ddim_timesteps
        seq = np.asarray(list(range(0, total_timesteps, c)))
        if seq[-1] != total_timesteps - 1:
            seq = np.append(seq, total_timesteps - 1)
        return seq[::-1]

    # ---- RNG in reference order -------------------------------------------------------------
    def _randn(self, shape, device):
        nd = self.noise_device
        if self.noise_shard is not None:
            lo, hi, gb = self.noise_shard
            if shape[0] != hi - lo:
                raise ValueError(f"batch {shape[0]} does not match noise_shard rows {lo}:{hi}")
            full = torch.randn(gb, *shape[1:], device=nd if nd is not None else device)
            return full[lo:hi].to(device).contiguous()
        if nd is None or torch.device(nd) == torch.device(device):
            return torch.randn(*shape, device=device)
        return torch.randn(*shape, device=nd).to(device, non_blocking=True)

    def _fused(self, model_fn):
        return (getattr(model_fn, "__self__", None) is self and getattr(model_fn, "__func__", None)
                is InpaintingSampler.model_fn and isinstance(self.model, DiffusionInpaintingModel))

    def _guarded(self, model_fn, device, run):
        """The fused loops in 3xf16 mode: one range-guard check at the end of the loop (one sync);
        if an operand reached the f16 range, the RNG state is rewound and the loop re-run in exact
        fp32, so the returned sample is what the fp32 path would give for the same seed."""
        if not (self._fused(model_fn) and self.model.precision != "fp32"):
            return run()
        dev = torch.device(device)
        states = [(None, torch.get_rng_state())]
        if dev.type == "cuda":
            states.append((dev, torch.cuda.get_rng_state(dev)))

        def rewind():
            for d, st in states:
                if d is None:
                    torch.set_rng_state(st)
                else:
                    torch.cuda.set_rng_state(st, d)
        return self.model.run_guarded(self.model.handle(dev), dev, run, before_retry=rewind)

    # ---- script DDIM (code/test_inp_ddim_50.py:470-576) -------------------------------------
    def inpainting_ddim_sample_loop(self, model_fn, shape, gt_images, masks, clip_denoised=True, device=None,
                                    progress=False, eta=0.0):
        if device is None:
            device = next(self.model.parameters()).device
        return self._guarded(model_fn, device, lambda: self._ddim_loop(model_fn, shape, gt_images, masks,
                                                                       clip_denoised, device, progress, eta))

    def _ddim_loop(self, model_fn, shape, gt_images, masks, clip_denoised, device, progress, eta):
        assert isinstance(shape, (tuple, list))
        B, _, H, W = shape
        gt, mk = prepare_gt_mask(gt_images, masks, B, H, W, device)
        img = self._randn(shape, device).contiguous()
        seq = self.create_ddim_timestep_sequence(self.diffusion.num_timesteps, self.args.ddim_timesteps)
        it = enumerate(seq)
        if progress:
            from tqdm import tqdm
            it = tqdm(it, total=len(seq), desc=f"DDIM inpainting ({self.args.ddim_timesteps} steps)")
        fused = self._fused(model_fn)
        L = _lib.lib()
        h = self.model.handle(torch.device(device)) if fused else None
        keep = None if fused else 1 - mk
        # every step's timestep vector in one host-to-device copy (rows are contiguous views)
        t_tab = torch.as_tensor(np.repeat(np.asarray(seq, dtype=np.int64)[:, None], B, 1)).to(device)
        for k, tau in it:
            tau = int(tau)
            c = ddim_coeffs(self.diffusion.alphas_cumprod, seq, k, eta, clip_denoised)
            t = t_tab[k]
            with torch.no_grad():
                out = None if fused else model_fn(img, t, gt=gt, gt_keep_mask=keep)
                noise = self._randn(shape, device) if c.use_noise else None
                known = self._randn(gt.shape, device) if c.inject else None
                if fused:
                    _lib.check(L.ifd_ddim_step(h.h, _lib.ptr(t), B, H, W, _lib.ptr(img), _lib.ptr(gt), _lib.ptr(mk),
                                               _lib.ptr(noise), _lib.ptr(known), c, _lib.stream_ptr(device)))
                else:
                    out = out.to(torch.float32).contiguous()
                    if out.dim() != 4 or out.shape[0] != B or out.shape[1] not in (3, 6) or out.shape[2:] != (H, W):
                        raise ValueError(f"Unexpected model output shape: {tuple(out.shape)}")
                    if out.shape[1] == 3:
                        out = torch.cat([out, torch.zeros_like(out)], 1)
                    _lib.check(L.ifd_ddim_update(_lib.ptr(out), B, H, W, _lib.ptr(img), _lib.ptr(gt), _lib.ptr(mk),
                                                 _lib.ptr(noise), _lib.ptr(known), c, _lib.stream_ptr(device)))
                del noise, known
        return img

    # ---- script DDPM (code/test_inp_ddim_50.py:402-468) -------------------------------------
    def inpainting_p_sample_loop(self, model_fn, shape, gt_images, masks, clip_denoised=True, device=None,
                                 progress=False):
        if device is None:
            device = next(self.model.parameters()).device
        return self._guarded(model_fn, device, lambda: self._ddpm_loop(model_fn, shape, gt_images, masks,
                                                                       clip_denoised, device, progress))

    def _ddpm_loop(self, model_fn, shape, gt_images, masks, clip_denoised, device, progress):
        assert isinstance(shape, (tuple, list))
        B, _, H, W = shape
        gt, mk = prepare_gt_mask(gt_images, masks, B, H, W, device)
        img = self._randn(shape, device).contiguous()
        indices = list(range(self.diffusion.num_timesteps))[::-1]
        if progress:
            from tqdm import tqdm
            indices = tqdm(indices, desc="DDPM inpainting with injection")
        fused = self._fused(model_fn)
        L = _lib.lib()
        h = self.model.handle(torch.device(device)) if fused else None
        keep = None if fused else 1 - mk
        T = self.diffusion.num_timesteps
        t_tab = torch.as_tensor(np.repeat(np.arange(T, dtype=np.int64)[:, None], B, 1)).to(device)
        for i in indices:
            c = ddpm_coeffs(self.diffusion, i, clip_denoised)
            t = t_tab[i]
            with torch.no_grad():
                out = None if fused else model_fn(img, t, gt=gt, gt_keep_mask=keep)
                noise = self._randn(shape, device)
                known = self._randn(gt.shape, device) if i > 0 else None
                if fused:
                    _lib.check(L.ifd_ddpm_step(h.h, _lib.ptr(t), B, H, W, _lib.ptr(img), _lib.ptr(gt), _lib.ptr(mk),
                                               _lib.ptr(noise), _lib.ptr(known), c, _lib.stream_ptr(device)))
                else:
                    out = out.to(torch.float32).contiguous()
                    if tuple(out.shape) != (B, 6, H, W):  # p_mean_variance's LEARNED_RANGE split (:241-243)
                        raise ValueError(f"DDPM needs a [B,6,H,W] model output, got {tuple(out.shape)}")
                    _lib.check(L.ifd_ddpm_update(_lib.ptr(out), B, H, W, _lib.ptr(img), _lib.ptr(gt), _lib.ptr(mk),
                                                 _lib.ptr(noise), _lib.ptr(known), c, _lib.stream_ptr(device)))
                del noise, known
        return img

    @staticmethod
    def final_blend(result, gt_images, masks):
        """code/test_inp_ddim_50.py:692-696 (one HIP kernel)."""
        r = result.to(torch.float32).contiguous()
        if r.dim() != 4 or r.shape[1] != 3:
            raise ValueError(f"result must be [B,3,H,W], got {tuple(r.shape)}")
        B, C, H, W = r.shape
        g, m = prepare_gt_mask(gt_images, masks, B, H, W, r.device)
        out = torch.empty_like(r)
        _lib.check(_lib.lib().ifd_blend(_lib.ptr(r), _lib.ptr(g), _lib.ptr(m), B, C, H, W, _lib.ptr(out),
                                        _lib.stream_ptr(r.device)))
        return out
