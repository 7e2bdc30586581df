"""Generate the committed golden fixtures by importing the reference in the build container.

Run here (not on the GPU box — /root/reference does not travel):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What it does
  1. Imports the reference modules from /root/reference/code (unet, nn, gaussian_diffusion,
     utils.schedules and the sampling script test_inp_ddim_50 with its IO/metric-only imports
     torchvision / lpips / skimage stubbed — they are not installed and are off the hot path).
  2. Checks our state-dict spec (ifd.topology) against the reference model's state_dict.
  3. Loads seeded manifest weights (ifd.manifest) into the reference model and records
     outputs of: per-layer modules, whole UNet evals (reduced 64x64 config and the full 256x256
     config), the script DDIM / DDPM loops (InpaintingSampler.inpainting_*_sample_loop called on
     the real class), and the library ddim_sample_loop / p_sample_loop with injection.
  4. Checks the oracle (oracle/ref_*.py) against every reference output it restates.

RNG convention for every loop fixture: torch.manual_seed(seed) on the CPU generator
immediately before the loop call; all draws come from that generator in reference order.
Inputs: gt ~ U(-1,1) from Generator(seed 7); mask 1 = hole.
"""
from __future__ import annotations

import json
import os
import sys
import time
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "face-inpainting-diffusion-models_amd"))
REF = "/root/reference/code"
OUT = os.path.dirname(os.path.abspath(__file__))

from ifd.topology import FULL, REDUCED, state_dict_spec  # noqa: E402
from ifd.manifest import make_state_dict, checksums  # noqa: E402
from oracle import ref_unet, ref_diffusion  # noqa: E402


def _stub_modules():
    """torchvision / lpips / skimage are imported at the top of the reference scripts for IO and
    metrics only; they are not installed here. Empty stand-ins let the sampler class import."""
    tv = types.ModuleType("torchvision")
    tv.transforms = types.ModuleType("torchvision.transforms")
    tv.utils = types.ModuleType("torchvision.utils")
    tv.utils.save_image = lambda *a, **k: None
    for name in ("Compose", "Resize", "ToTensor", "Normalize", "Grayscale"):
        setattr(tv.transforms, name, lambda *a, **k: None)
    sys.modules.update({"torchvision": tv, "torchvision.transforms": tv.transforms, "torchvision.utils": tv.utils})
    lp = types.ModuleType("lpips")
    lp.LPIPS = lambda *a, **k: None
    sys.modules["lpips"] = lp
    sk = types.ModuleType("skimage")
    sk.metrics = types.ModuleType("skimage.metrics")
    sk.metrics.structural_similarity = lambda *a, **k: 0.0
    sys.modules.update({"skimage": sk, "skimage.metrics": sk.metrics})


def import_reference():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    _stub_modules()
    import unet as r_unet
    import nn as r_nn
    import gaussian_diffusion as r_gd
    from utils import schedules as r_sched
    import test_inp_ddim_50 as r_script
    return r_unet, r_nn, r_gd, r_sched, r_script


def ref_model(r_unet, cfg, sd):
    base = r_unet.UNetModel(
        image_size=cfg.image_size, in_channels=3, model_channels=cfg.model_channels, out_channels=6,
        num_res_blocks=cfg.num_res_blocks, attention_resolutions=cfg.attention_resolutions,
        channel_mult=cfg.channel_mult, conv_resample=True, dims=2, use_checkpoint=False, use_fp16=False,
        num_heads=4, num_head_channels=cfg.num_head_channels, use_scale_shift_norm=True, resblock_updown=True)
    m = r_unet.DiffusionInpaintingModel(base, in_channels=9)
    ref_keys = [(k, tuple(v.shape)) for k, v in m.state_dict().items()]
    ours = [(k, tuple(s)) for k, s in state_dict_spec(cfg)]
    assert ref_keys == ours, "state-dict spec mismatch"
    m.load_state_dict(sd, strict=True)
    m.eval()
    return m, ref_keys


def gt_and_mask(B, H, seed_gt=7, kind="center"):
    g = torch.Generator().manual_seed(seed_gt)
    gt = torch.rand(B, 3, H, H, generator=g) * 2 - 1
    mask = torch.zeros(B, 1, H, H)
    if kind == "center":
        q = H // 4
        mask[:, :, q:H - q, q:H - q] = 1.0
    else:  # seeded random rectangles covering roughly 5-60 % (README.md:93)
        for b in range(B):
            for _ in range(3):
                h0, w0 = [int(v) for v in torch.randint(0, H // 2, (2,), generator=g)]
                hh, ww = [int(v) for v in torch.randint(H // 8, H // 2, (2,), generator=g)]
                mask[b, :, h0:h0 + hh, w0:w0 + ww] = 1.0
    return gt, mask


def maxabs(a, b):
    return float((a.double() - b.double()).abs().max())


def main():
    t0 = time.time()
    torch.set_num_threads(8)
    r_unet, r_nn, r_gd, r_sched, r_script = import_reference()
    meta = {"generated_by": "tests/golden/make_golden.py", "torch": torch.__version__, "checks": {}}

    # ---------- 1. state-dict spec + manifest checksums ----------
    sds = {}
    for name, cfg in (("reduced", REDUCED), ("full", FULL)):
        sd = make_state_dict(cfg, seed=1)
        sds[name] = sd
        model, keys = ref_model(r_unet, cfg, sd)
        meta[f"keys_{name}"] = [[k, list(s)] for k, s in keys]
        meta[f"checksums_{name}"] = checksums(sd)
    red_model, _ = ref_model(r_unet, REDUCED, sds["reduced"])
    full_model, _ = ref_model(r_unet, FULL, sds["full"])
    sd_red = ref_unet.strip_prefix(sds["reduced"])
    sd_full = ref_unet.strip_prefix(sds["full"])

    # ---------- 2. per-layer modules (reference classes, manifest-style weights) ----------
    layers = {}
    g = torch.Generator().manual_seed(11)

    def init_module(mod, seed):
        gg = torch.Generator().manual_seed(seed)
        with torch.no_grad():
            for k, p in mod.state_dict().items():
                u = torch.rand(p.shape, generator=gg) * 2 - 1
                if p.dim() == 1 and ("in_layers.0" in k or "out_layers.0" in k or k.startswith("norm")):
                    p.copy_(1 + 0.1 * u if k.endswith("weight") else 0.1 * u)
                else:
                    fan = p.shape[1:].numel() if p.dim() > 1 else None
                    if fan is None:
                        w = mod.state_dict()[k[: -len("bias")] + "weight"]
                        fan = w.shape[1:].numel()
                    p.copy_(u / fan ** 0.5)

    cases = [
        ("res_128_128_r16", dict(cin=128, cout=128), 16, False, False),
        ("res_192_64_r16", dict(cin=192, cout=64), 16, False, False),
        ("res_down_64_r32", dict(cin=64, cout=64), 32, False, True),
        ("res_up_64_r8", dict(cin=64, cout=64), 8, True, False),
    ]
    for i, (name, ch, r, up, down) in enumerate(cases):
        mod = r_nn.ResBlock(ch["cin"], 256, 0.0, out_channels=ch["cout"], use_scale_shift_norm=True, up=up, down=down)
        init_module(mod, 100 + i)
        mod.eval()
        x = torch.randn(2, ch["cin"], r, r, generator=g)
        emb = torch.randn(2, 256, generator=g)
        with torch.no_grad():
            y = mod(x, emb)
            sd = {k: v for k, v in mod.state_dict().items()}
            yo = ref_unet.resblock(sd, "", x, emb, ch["cout"], up=up, down=down)
        meta["checks"][f"oracle_vs_ref_{name}"] = maxabs(y, yo)
        layers[name] = dict(x=x, emb=emb, y=y, **{"w." + k: v for k, v in sd.items()})
    for i, (name, c, r) in enumerate((("attn_512_r8", 512, 8), ("attn_256_r16", 256, 16), ("attn_128_r4", 128, 4))):
        mod = r_nn.AttentionBlock(c, num_heads=4, num_head_channels=64)
        init_module(mod, 200 + i)
        x = torch.randn(2, c, r, r, generator=g)
        with torch.no_grad():
            y = mod(x)
            sd = {k: v for k, v in mod.state_dict().items()}
            yo = ref_unet.attention(sd, "", x, 64)
        meta["checks"][f"oracle_vs_ref_{name}"] = maxabs(y, yo)
        layers[name] = dict(x=x, y=y, **{"w." + k: v for k, v in sd.items()})
    # (round 1 stored these forward-only tensors as layers.npz; the block-level fixtures, forward and
    # backward, are now made by make_golden_blocks.py — only the oracle checks are kept here)
    del layers

    # ---------- 3. whole-UNet evals ----------
    evals = {}
    for name, cfg, model, sdo, B in (("reduced", REDUCED, red_model, sd_red, 2), ("full", FULL, full_model, sd_full, 1)):
        H = cfg.image_size
        gt, mask = gt_and_mask(B, H, kind="center" if name == "full" else "rect")
        keep = 1 - mask
        gx = torch.Generator().manual_seed(42)
        x = torch.randn(B, 3, H, H, generator=gx)
        ts = (999, 500, 10) if name == "reduced" else (999,)
        for tv in ts:
            t = torch.tensor([tv] * B)
            with torch.no_grad():
                y = model(x, t, masked_image=gt * keep, mask=mask)
                yo = ref_unet.inpaint_forward(sdo, x, t, gt * keep, mask, cfg)
            meta["checks"][f"oracle_vs_ref_unet_{name}_t{tv}"] = maxabs(y, yo)
            evals[f"{name}_t{tv}/y"] = y
        evals[f"{name}/x"] = x
        evals[f"{name}/gt"] = gt
        evals[f"{name}/mask"] = mask
        print(f"[golden] unet {name} done {time.time() - t0:.1f}s", flush=True)
    np.savez_compressed(os.path.join(OUT, "unet_evals.npz"), **{k: v.numpy() for k, v in evals.items()})

    # ---------- 4. script loops (real InpaintingSampler methods) ----------
    loops = {}
    loop_meta = {}

    def sampler_for(model, diffusion, ddim_steps):
        s = object.__new__(r_script.InpaintingSampler)
        s.args = types.SimpleNamespace(ddim_timesteps=ddim_steps)
        s.model = model
        s.diffusion = diffusion
        s.device = torch.device("cpu")
        return s

    loop_cases = [
        # name, cfg, model, sd, B, schedule, T, method, steps, eta, mask kind
        ("c1_full_cos10_eta0.9", FULL, full_model, sd_full, 1, "cosine", 1000, "ddim", 10, 0.9, "center"),
        ("c1_full_cos10_eta0", FULL, full_model, sd_full, 1, "cosine", 1000, "ddim", 10, 0.0, "center"),
        ("red_cos10_eta0.9", REDUCED, red_model, sd_red, 2, "cosine", 1000, "ddim", 10, 0.9, "rect"),
        ("red_lin500_ddim10_eta0.9", REDUCED, red_model, sd_red, 2, "linear", 500, "ddim", 10, 0.9, "rect"),
        ("red_quad_ddim30_eta0.9", REDUCED, red_model, sd_red, 2, "quadratic", 1000, "ddim", 30, 0.9, "center"),
        ("red_cos100_eta0.75", REDUCED, red_model, sd_red, 2, "cosine", 1000, "ddim", 100, 0.75, "center"),
        ("red_ddpm_lin1000", REDUCED, red_model, sd_red, 1, "linear", 1000, "ddpm", 0, 0.0, "rect"),
    ]
    for (name, cfg, model, sdo, B, sched, T, method, steps, eta, mk) in loop_cases:
        H = cfg.image_size
        diffusion = r_sched.create_gaussian_diffusion(steps=T, learn_sigma=True, noise_schedule=sched)
        tb = ref_diffusion.Tables(ref_diffusion.get_named_beta_schedule(sched, T))
        assert np.array_equal(tb.ac, diffusion.alphas_cumprod)
        gt, mask = gt_and_mask(B, H, kind=mk)
        s = sampler_for(model, diffusion, steps)
        seed = 1234
        with torch.no_grad():
            torch.manual_seed(seed)
            if method == "ddim":
                y = s.inpainting_ddim_sample_loop(s.model_fn, (B, 3, H, H), gt, mask, clip_denoised=True,
                                                  device=torch.device("cpu"), progress=False, eta=eta)
            else:
                y = s.inpainting_p_sample_loop(s.model_fn, (B, 3, H, H), gt, mask, clip_denoised=True,
                                               device=torch.device("cpu"), progress=False)
            y = ref_diffusion.final_blend(y, gt, mask)
            # oracle restatement, same seed / order
            mf = ref_diffusion.model_fn_factory(lambda x, t, m, k: ref_unet.inpaint_forward(sdo, x, t, m, k, cfg))
            torch.manual_seed(seed)
            if method == "ddim":
                yo = ref_diffusion.script_ddim_loop(tb, mf, (B, 3, H, H), gt, mask, steps, True, eta)
            else:
                yo = ref_diffusion.script_ddpm_loop(tb, mf, (B, 3, H, H), gt, mask, True)
            yo = ref_diffusion.final_blend(yo, gt, mask)
        meta["checks"][f"oracle_vs_ref_loop_{name}"] = maxabs(y, yo)
        loops[f"{name}/y"] = y
        loops[f"{name}/gt"] = gt
        loops[f"{name}/mask"] = mask
        loop_meta[name] = dict(cfg="full" if cfg is FULL else "reduced", B=B, schedule=sched, T=T, method=method,
                               ddim_steps=steps, eta=eta, seed=seed, mask=mk, final_blend=True)
        print(f"[golden] loop {name} done {time.time() - t0:.1f}s maxabs(oracle) {meta['checks'][f'oracle_vs_ref_loop_{name}']:.3g}", flush=True)

    # ---------- 5. library loops with injection (GaussianDiffusion.*_sample_loop) ----------
    for (name, method, sched, T, eta) in (("lib_ddim_lin50_eta0.5", "ddim", "linear", 50, 0.5),
                                          ("lib_ddpm_cos50", "ddpm", "cosine", 50, 0.0)):
        cfg, model, sdo, B = REDUCED, red_model, sd_red, 2
        H = cfg.image_size
        diffusion = r_sched.create_gaussian_diffusion(steps=T, learn_sigma=True, noise_schedule=sched)
        tb = ref_diffusion.Tables(ref_diffusion.get_named_beta_schedule(sched, T))
        gt, mask = gt_and_mask(B, H, kind="rect")
        keep = 1 - mask
        s = sampler_for(model, diffusion, 0)
        kw = {"gt": gt, "gt_keep_mask": keep}
        seed = 99
        with torch.no_grad():
            torch.manual_seed(seed)
            if method == "ddim":
                y = diffusion.ddim_sample_loop(s.model_fn, (B, 3, H, H), clip_denoised=True, model_kwargs=kw,
                                               device=torch.device("cpu"), eta=eta, use_inpainting_injection=True)
            else:
                y = diffusion.p_sample_loop(s.model_fn, (B, 3, H, H), clip_denoised=True, model_kwargs=kw,
                                            device=torch.device("cpu"), use_inpainting_injection=True)
            mf = ref_diffusion.model_fn_factory(lambda x, t, m, k: ref_unet.inpaint_forward(sdo, x, t, m, k, cfg))
            torch.manual_seed(seed)
            if method == "ddim":
                yo = ref_diffusion.library_ddim_loop(tb, mf, (B, 3, H, H), kw, eta=eta)
            else:
                yo = ref_diffusion.library_ddpm_loop(tb, mf, (B, 3, H, H), kw)
        meta["checks"][f"oracle_vs_ref_loop_{name}"] = maxabs(y, yo)
        loops[f"{name}/y"] = y
        loops[f"{name}/gt"] = gt
        loops[f"{name}/mask"] = mask
        loop_meta[name] = dict(cfg="reduced", B=B, schedule=sched, T=T, method="lib_" + method, eta=eta,
                               seed=seed, mask="rect", final_blend=False)
        print(f"[golden] {name} done {time.time() - t0:.1f}s", flush=True)

    np.savez_compressed(os.path.join(OUT, "loops.npz"), **{k: v.numpy() for k, v in loops.items()})
    meta["loops"] = loop_meta
    # timestep sequences (create_ddim_timestep_sequence) for the a1 row
    s = sampler_for(None, None, 0)
    meta["ddim_sequences"] = {f"{T}_{n}": [int(v) for v in s.create_ddim_timestep_sequence(T, n)]
                              for T, n in ((1000, 100), (1000, 50), (1000, 30), (1000, 10), (500, 10), (500, 50))}
    # schedules (float64 alphas_cumprod) for the a17/a18 rows
    meta["alphas_cumprod_samples"] = {}
    for sched in ("linear", "cosine", "quadratic"):
        for T in (1000, 500):
            d = r_sched.create_gaussian_diffusion(steps=T, learn_sigma=True, noise_schedule=sched)
            meta["alphas_cumprod_samples"][f"{sched}_{T}"] = [float(d.alphas_cumprod[i]) for i in (0, 1, T // 2, T - 2, T - 1)]
    meta["elapsed_s"] = time.time() - t0
    with open(os.path.join(OUT, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(json.dumps(meta["checks"], indent=1))


if __name__ == "__main__":
    main()
