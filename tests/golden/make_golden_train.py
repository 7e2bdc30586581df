"""Reference training-step fixtures (BASELINE configs[4] / SURVEY §8f rank 1), made by importing the
reference here. Run in the build container:
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_train.py

Calls the reference's own `train_epoch` (code/train_inpainting.py:15-79) twice, one batch each, on
the reduced config (64x64, 64 channels, B=2) with seeded manifest weights, the reference factory's
diffusion (quadratic T=1000, code/train_inpainting.py:248-255) and AdamW(lr 5e-5, wd 0.01,
betas 0.9/0.999) (:394-399, scripts/train.py:112,142). Inside: t = randint (device RNG = the CPU
generator here), noise = randn_like, the GT-noise cache entry for t[0] (gaussian_diffusion.py:85-108,
never cleared), masked eps-MSE, backward, clip_grad_norm_(1.0), AdamW.step.
Recorded per step: the loss, the gradient norm before clipping; per parameter tensor: the norm of
the (clipped) gradient, the norm of the update, and the values of both at up to 256 fixed indices.
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "face-inpainting-diffusion-models_amd"), HERE]
from ifd.manifest import make_state_dict  # noqa: E402
from ifd.topology import REDUCED  # noqa: E402
import make_golden as mg  # noqa: E402


def sample_idx(n, k=256):
    return np.unique(np.linspace(0, n - 1, min(n, k)).round().astype(np.int64))


def main():
    torch.set_num_threads(8)
    r_unet, r_nn, r_gd, r_sched, r_script = mg.import_reference()
    import train_inpainting as r_train
    sd = make_state_dict(REDUCED, seed=1)
    model, _ = mg.ref_model(r_unet, REDUCED, sd)
    diffusion = r_sched.create_gaussian_diffusion(steps=1000, learn_sigma=True, noise_schedule="quadratic",
                                                  use_kl=False, predict_xstart=False, rescale_timesteps=False)
    opt, _ = r_train.create_optimizer_and_scheduler(model, lr=5e-5, weight_decay=0.01, num_epochs=1,
                                                    scheduler_type="none")
    B, H = 2, 64
    out = {}
    meta = {"config": "reduced", "B": B, "H": H, "lr": 5e-5, "weight_decay": 0.01, "betas": [0.9, 0.999],
            "eps": 1e-8, "max_norm": 1.0, "schedule": "quadratic", "T": 1000, "steps": []}
    names = [k for k, _ in model.named_parameters()]
    params0 = {k: v.detach().clone() for k, v in model.named_parameters()}
    for step, seed in enumerate((2024, 2025)):
        g = torch.Generator().manual_seed(100 + step)
        images = torch.rand(B, 3, H, H, generator=g) * 2 - 1
        masks = torch.zeros(B, 1, H, H)
        masks[0, :, 16:48, 8:40] = 1
        masks[1, :, 4:30, 20:60] = 1
        masked = images * (1 - masks)  # data/dataset.py:286
        batch = [{"image": images, "masked_image": masked, "mask": masks}]
        torch.manual_seed(seed)
        # the same draws train_epoch makes, replayed to record them (t first: train_inpainting.py:42)
        t_rec = torch.randint(0, diffusion.num_timesteps, (B,)).long()
        torch.manual_seed(seed)
        norms = {}
        orig_clip = torch.nn.utils.clip_grad_norm_

        def clip_rec(params, max_norm, *a, **k):
            total = orig_clip(params, max_norm, *a, **k)
            norms["total"] = float(total)
            return total
        r_train.torch.nn.utils.clip_grad_norm_ = clip_rec
        try:
            loss = r_train.train_epoch(model, batch, opt, diffusion, torch.device("cpu"), epoch=1)
        finally:
            r_train.torch.nn.utils.clip_grad_norm_ = orig_clip
        rec = {"seed": seed, "t": [int(v) for v in t_rec], "loss": float(loss), "grad_norm": norms["total"]}
        out[f"s{step}/images"] = images.numpy()
        out[f"s{step}/masks"] = masks.numpy()
        for k, p in model.named_parameters():
            gflat = p.grad.detach().flatten()
            dflat = (p.detach() - params0[k]).flatten()
            idx = sample_idx(gflat.numel())
            out[f"s{step}/g/{k}"] = gflat[idx].numpy()
            out[f"s{step}/d/{k}"] = dflat[idx].numpy()
            rec.setdefault("gnorm", {})[k] = float(gflat.double().norm())
            rec.setdefault("dnorm", {})[k] = float(dflat.double().norm())
        params0 = {k: v.detach().clone() for k, v in model.named_parameters()}
        meta["steps"].append(rec)
        print(f"[train golden] step {step}: t={rec['t']} loss={rec['loss']:.6f} grad_norm={rec['grad_norm']:.4f}",
              flush=True)
    meta["param_names"] = names
    np.savez_compressed(os.path.join(HERE, "train_steps.npz"), **out)
    with open(os.path.join(HERE, "train_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
