"""GPU parity of the training step (BASELINE configs[4]) against the reference's
own `train_epoch` (code/train_inpainting.py:15-79): two steps on the reduced config, fp32, same
weights, batches and RNG draws (t, noise, the t[0]-keyed GT-noise cache). Fixtures:
tests/golden/make_golden_train.py (train_meta.json, train_steps.npz).

Tolerances (written here):
  * loss:                         relative 1e-5
  * global gradient norm:         relative 1e-4 (clip_grad_norm_'s total norm, step 1 clips at 2.68)
  * per-tensor clipped gradient:  ||g - g_ref|| <= 1e-3 ||g_ref|| on the recorded indices, and the
                                  norm of the whole tensor within 1e-3 relative
  * per-tensor AdamW update:      |d - d_ref| <= 1e-3 lr + 2 ulp(p) where |g_ref| >= 1e-3 max|g_ref|
                                  (d = p_new - p_old carries p's own rounding; elsewhere the first
                                  steps' update ~ lr sign(g) may flip with rounding: <= 2.2 lr)
"""
import json
import os

import numpy as np
import pytest
import torch

from ifd.manifest import make_state_dict
from ifd.topology import REDUCED

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _sample_idx(n, k=256):
    return np.unique(np.linspace(0, n - 1, min(n, k)).round().astype(np.int64))


@pytest.fixture(scope="module")
def golden_train():
    meta = json.load(open(os.path.join(GOLDEN, "train_meta.json")))
    return meta, dict(np.load(os.path.join(GOLDEN, "train_steps.npz")))


def test_train_steps_match_reference(golden_train, record):
    from ifd.schedules import create_gaussian_diffusion
    from ifd.train import UNetTrainer
    meta, z = golden_train
    tr = UNetTrainer(REDUCED, device=DEV, lr=meta["lr"], weight_decay=meta["weight_decay"], betas=tuple(meta["betas"]),
                     eps=meta["eps"], max_norm=meta["max_norm"])
    tr.load_state_dict(make_state_dict(REDUCED, seed=1))
    diff = create_gaussian_diffusion(steps=meta["T"], learn_sigma=True, noise_schedule=meta["schedule"])
    lr = meta["lr"]
    prev = tr.flat.clone()
    worst = {}
    for step, rec in enumerate(meta["steps"]):
        images = torch.from_numpy(z[f"s{step}/images"])
        masks = torch.from_numpy(z[f"s{step}/masks"])
        masked = images * (1 - masks)
        torch.manual_seed(rec["seed"])
        t = torch.randint(0, diff.num_timesteps, (images.shape[0],)).long()
        assert t.tolist() == rec["t"]
        loss = tr.train_step(diff, images.to(DEV), masked.to(DEV), masks.to(DEV), t.to(DEV), noise_device="cpu")
        torch.cuda.synchronize()
        loss = float(loss)
        gnorm = float(tr.norm_coef[0])
        rel_loss = abs(loss - rec["loss"]) / abs(rec["loss"])
        rel_gn = abs(gnorm - rec["grad_norm"]) / rec["grad_norm"]
        g_rel, n_rel, d_err, d_frac = 0.0, 0.0, 0.0, 1.0
        for name in meta["param_names"]:
            key = name[len("base_model."):]
            g = tr.g(key).flatten()
            d = (tr.p(key) - prev[tr.offsets[key][0]: tr.offsets[key][0] + g.numel()].view(tr.p(key).shape)).flatten()
            idx = torch.from_numpy(_sample_idx(g.numel())).to(DEV)
            gs, ds = g[idx].double().cpu(), d[idx].double().cpu()
            ulp2 = 2.0 ** -22 * tr.p(key).flatten()[idx].double().abs().cpu()
            gr = torch.from_numpy(z[f"s{step}/g/{name}"]).double()
            dr = torch.from_numpy(z[f"s{step}/d/{name}"]).double()
            ref_n = rec["gnorm"][name]
            if ref_n > 0:
                g_rel = max(g_rel, float((gs - gr).norm() / max(gr.norm(), 1e-30)))
                n_rel = max(n_rel, abs(float(g.double().norm()) - ref_n) / ref_n)
            else:
                assert float(g.abs().max()) == 0.0, name
            big = gr.abs() >= 1e-3 * float(gr.abs().max()) if float(gr.abs().max()) > 0 else torch.ones_like(gr, dtype=bool)
            if big.any():
                d_err = max(d_err, float(((ds - dr).abs() - ulp2)[big].max()) / lr)
            d_frac = min(d_frac, float(((ds - dr).abs() <= 1e-3 * lr).double().mean()))
            assert float((ds - dr).abs().max()) <= 2.2 * lr, (step, name)
        worst[step] = dict(loss=loss, loss_ref=rec["loss"], rel_loss=rel_loss, grad_norm=gnorm,
                           grad_norm_ref=rec["grad_norm"], rel_grad_norm=rel_gn, max_tensor_grad_rel=g_rel,
                           max_tensor_norm_rel=n_rel, max_update_err_over_lr=d_err, min_update_frac_within=d_frac)
        prev = tr.flat.clone()
        assert rel_loss <= 1e-5 and rel_gn <= 1e-4, worst[step]
        assert g_rel <= 1e-3 and n_rel <= 1e-3, worst[step]
        assert d_err <= 1e-3, worst[step]
    record("train_steps_reduced/fp32", **{f"step{k}": v for k, v in worst.items()})


def test_train_step_deterministic():
    """Two identical steps from identical state give bit-identical parameters (no atomics anywhere)."""
    from bench import synth_inputs
    from ifd.schedules import create_gaussian_diffusion
    from ifd.train import UNetTrainer
    diff = create_gaussian_diffusion(steps=1000, learn_sigma=True, noise_schedule="quadratic")
    gt, mask = synth_inputs(2, 64, seed=3, device=DEV)
    outs = []
    for _ in range(2):
        tr = UNetTrainer(REDUCED, device=DEV)
        tr.load_state_dict(make_state_dict(REDUCED, seed=1))
        torch.manual_seed(9)
        t = torch.randint(0, 1000, (2,), device=DEV)
        tr.train_step(diff, gt, gt * (1 - mask), mask, t)
        torch.cuda.synchronize()
        outs.append(tr.flat.clone())
    assert torch.equal(outs[0], outs[1])
