"""Full-size (256x256) loop fixtures and fp64 error envelopes, made by importing the reference here.

Run in the build container (the reference does not travel to the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_full.py [case ...]

Cases (each writes tests/golden/full/<case>.npz and merges its record into
tests/golden/full/meta_full.json):
  c2_cos100_eta0.75   the headline workload's loop (BASELINE configs[1]): the real
                      `InpaintingSampler.inpainting_ddim_sample_loop` of code/test_inp_ddim_100.py
                      (:470-576), full 256x256 config, cosine T=1000, DDIM-100, eta 0.75
                      (code/test_inp_ddim_100.py:820), B=1, centre mask, + final blend (:692-696).
                      Also: the oracle (fp32, must equal the reference) and the oracle in fp64 (the
                      error envelope: how far the fp32 reference itself is from exact arithmetic).
  c3_ddpm_lin1000     configs[2]'s loop: the real `inpainting_p_sample_loop` (code/test_inp_ddim_50.py
                      :402-468, the body code/tes_ddpm.py repeats), full config, linear T=1000, B=1,
                      rectangle mask, + final blend.
  c1_fp64             fp64 oracle outputs of the two C1 loops already in loops.npz
                      (c1_full_cos10_eta0 / _eta0.9): the fp32-vs-exact envelope of the reference.
  adv_inpaint         `GaussianDiffusion.sample_with_advanced_inpainting` (code/gaussian_diffusion.py
                      :640-700) at the reduced config: DDIM eta 0.5 / DDPM, injection schedules
                      "all" / "high" / "low", cumulative and fresh-noise injection.

RNG convention (as make_golden.py): torch.manual_seed(seed) on the CPU generator right before the
loop call; every draw in reference order. fp64 envelopes draw the same fp32 noise values
(oracle/ref_diffusion.py `_randn`).
"""
from __future__ import annotations

import json
import os
import sys
import time
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "face-inpainting-diffusion-models_amd"), HERE]
OUT = os.path.join(HERE, "full")

from ifd.manifest import make_state_dict  # noqa: E402
from ifd.topology import FULL, REDUCED  # noqa: E402
from oracle import ref_diffusion, ref_unet  # noqa: E402
import make_golden as mg  # noqa: E402


def _sampler(cls, model, diffusion, ddim_steps):
    s = object.__new__(cls)
    s.args = types.SimpleNamespace(ddim_timesteps=ddim_steps)
    s.model = model
    s.diffusion = diffusion
    s.device = torch.device("cpu")
    return s


def _stats(a, b):
    d = (a.double() - b.double()).abs().flatten()
    return {"max": float(d.max()), "p999": float(d.quantile(0.999)), "mean": float(d.mean())}


def _oracle_ddim(sd, cfg, lm, gt, mask):
    tb = ref_diffusion.Tables(ref_diffusion.get_named_beta_schedule(lm["schedule"], lm["T"]))
    mf = ref_diffusion.model_fn_factory(lambda x, t, m, k: ref_unet.inpaint_forward(sd, x, t, m, k, cfg))
    torch.manual_seed(lm["seed"])
    with torch.no_grad():
        y = ref_diffusion.script_ddim_loop(tb, mf, (lm["B"], 3, cfg.image_size, cfg.image_size), gt, mask,
                                           lm["ddim_steps"], True, lm["eta"])
    return ref_diffusion.final_blend(y, gt, mask)


def case_c2(ref, rec):
    r_unet, r_sched, r_script100 = ref["unet"], ref["sched"], ref["script100"]
    name = "c2_cos100_eta0.75"
    sd = make_state_dict(FULL, seed=1)
    model, _ = mg.ref_model(r_unet, FULL, sd)
    lm = dict(cfg="full", B=1, schedule="cosine", T=1000, method="ddim", ddim_steps=100, eta=0.75, seed=1234,
              mask="center", final_blend=True, script="code/test_inp_ddim_100.py")
    diffusion = r_sched.create_gaussian_diffusion(steps=lm["T"], learn_sigma=True, noise_schedule=lm["schedule"])
    gt, mask = mg.gt_and_mask(1, 256, kind="center")
    s = _sampler(r_script100.InpaintingSampler, model, diffusion, lm["ddim_steps"])
    torch.manual_seed(lm["seed"])
    with torch.no_grad():
        y = s.inpainting_ddim_sample_loop(s.model_fn, (1, 3, 256, 256), gt, mask, clip_denoised=True,
                                          device=torch.device("cpu"), progress=False, eta=lm["eta"])
        y = ref_diffusion.final_blend(y, gt, mask)
    print(f"[full] {name}: reference done", flush=True)
    sdo = ref_unet.strip_prefix(sd)
    yo = _oracle_ddim(sdo, FULL, lm, gt, mask)
    rec["checks"][f"oracle_vs_ref_{name}"] = mg.maxabs(y, yo)
    print(f"[full] {name}: oracle fp32 maxabs {rec['checks'][f'oracle_vs_ref_{name}']:.3g}", flush=True)
    sd64 = {k: v.double() for k, v in sdo.items()}
    y64 = _oracle_ddim(sd64, FULL, lm, gt, mask)
    rec["envelopes"][name] = _stats(y, y64)
    print(f"[full] {name}: fp32 ref vs fp64 {rec['envelopes'][name]}", flush=True)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), y=y.numpy(), y64=y64.numpy(), gt=gt.numpy(),
                        mask=mask.numpy())
    rec["loops"][name] = lm


def case_c3(ref, rec):
    r_unet, r_sched, r_script = ref["unet"], ref["sched"], ref["script50"]
    name = "c3_ddpm_lin1000"
    sd = make_state_dict(FULL, seed=1)
    model, _ = mg.ref_model(r_unet, FULL, sd)
    lm = dict(cfg="full", B=1, schedule="linear", T=1000, method="ddpm", ddim_steps=0, eta=0.0, seed=4321,
              mask="rect", final_blend=True, script="code/test_inp_ddim_50.py (= code/tes_ddpm.py loop body)")
    diffusion = r_sched.create_gaussian_diffusion(steps=lm["T"], learn_sigma=True, noise_schedule=lm["schedule"])
    gt, mask = mg.gt_and_mask(1, 256, kind="rect")
    s = _sampler(r_script.InpaintingSampler, model, diffusion, 0)
    t0 = time.time()
    torch.manual_seed(lm["seed"])
    with torch.no_grad():
        y = s.inpainting_p_sample_loop(s.model_fn, (1, 3, 256, 256), gt, mask, clip_denoised=True,
                                       device=torch.device("cpu"), progress=False)
        y = ref_diffusion.final_blend(y, gt, mask)
    print(f"[full] {name}: reference done {time.time() - t0:.0f}s", flush=True)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), y=y.numpy(), gt=gt.numpy(), mask=mask.numpy())
    rec["loops"][name] = lm


def case_c1_fp64(ref, rec):
    meta = json.load(open(os.path.join(HERE, "meta.json")))
    loops = np.load(os.path.join(HERE, "loops.npz"))
    sd64 = {k: v.double() for k, v in ref_unet.strip_prefix(make_state_dict(FULL, seed=1)).items()}
    arrs = {}
    for name in ("c1_full_cos10_eta0", "c1_full_cos10_eta0.9"):
        lm = meta["loops"][name]
        gt, mask = torch.from_numpy(loops[f"{name}/gt"]), torch.from_numpy(loops[f"{name}/mask"])
        y64 = _oracle_ddim(sd64, FULL, lm, gt, mask)
        rec["envelopes"][name] = _stats(torch.from_numpy(loops[f"{name}/y"]), y64)
        print(f"[full] {name}: fp32 ref vs fp64 {rec['envelopes'][name]}", flush=True)
        arrs[f"{name}/y64"] = y64.numpy()
    np.savez_compressed(os.path.join(OUT, "c1_fp64.npz"), **arrs)


def case_adv(ref, rec):
    r_unet, r_sched = ref["unet"], ref["sched"]
    sd = make_state_dict(REDUCED, seed=1)
    model, _ = mg.ref_model(r_unet, REDUCED, sd)

    def model_kw(x, t, masked_image=None, mask=None, **kw):  # the raw model rejects gt=
        return model(x, t, masked_image=masked_image, mask=mask)

    arrs = {}
    variants = [("adv_ddim_all", True, 0.5, "all", True), ("adv_ddim_high_fresh", True, 0.0, "high", False),
                ("adv_ddpm_low", False, 0.0, "low", True)]
    for (name, use_ddim, eta, sched_inj, cum) in variants:
        diffusion = r_sched.create_gaussian_diffusion(steps=40, learn_sigma=True, noise_schedule="cosine")
        gt, mask = mg.gt_and_mask(2, 64, kind="rect")
        keep = 1 - mask
        torch.manual_seed(77)
        with torch.no_grad():
            y = diffusion.sample_with_advanced_inpainting(model_kw, (2, 3, 64, 64), gt=gt, gt_keep_mask=keep,
                                                          use_ddim=use_ddim, eta=eta, progress=False,
                                                          device=torch.device("cpu"), injection_schedule=sched_inj,
                                                          use_cumulative_noise=cum)
        # the oracle's library loop with the same arguments: fp32 (must equal the reference) and
        # fp64 (the envelope)
        tb = ref_diffusion.Tables(ref_diffusion.get_named_beta_schedule("cosine", 40))
        kw = {"gt": gt, "gt_keep_mask": keep, "masked_image": gt * keep, "mask": 1 - keep}
        for dt, tag in ((torch.float32, "y32"), (torch.float64, "y64")):
            sdo = {k: v.to(dt) for k, v in ref_unet.strip_prefix(sd).items()}

            def omodel(x, t, masked_image=None, mask=None, **_):
                return ref_unet.inpaint_forward(sdo, x, t, masked_image, mask, REDUCED)
            loop = ref_diffusion.library_ddim_loop if use_ddim else ref_diffusion.library_ddpm_loop
            extra = dict(eta=eta) if use_ddim else {}
            torch.manual_seed(77)
            with torch.no_grad():
                yo = loop(tb, omodel, (2, 3, 64, 64), kw, schedule=sched_inj, cumulative=cum, **extra)
            if tag == "y32":
                rec["checks"][f"oracle_vs_ref_{name}"] = mg.maxabs(y, yo)
            else:
                rec["envelopes"][name] = _stats(y, yo)
                arrs[f"{name}/y64"] = yo.numpy()
        print(f"[full] {name}: oracle {rec['checks'][f'oracle_vs_ref_{name}']:.3g} env {rec['envelopes'][name]}")
        arrs[f"{name}/y"] = y.numpy()
        arrs[f"{name}/gt"] = gt.numpy()
        arrs[f"{name}/mask"] = mask.numpy()
        rec["loops"][name] = dict(cfg="reduced", B=2, schedule="cosine", T=40, method="advanced", use_ddim=use_ddim,
                                  eta=eta, injection_schedule=sched_inj, use_cumulative_noise=cum, seed=77,
                                  mask="rect", final_blend=False)
        print(f"[full] {name} done", flush=True)
    np.savez_compressed(os.path.join(OUT, "adv_inpaint.npz"), **arrs)


def case_c1_eval0(ref, rec):
    """The first UNet eval of the C1 loops (t=999 on the seed-1234 x_T): reference fp32 output and
    the fp64 oracle's, so a GPU test can compare its per-eval error distribution with the fp32
    reference's own (the quantity the 10-step loop amplifies ~2e4x at clamp-boundary pixels)."""
    r_unet = ref["unet"]
    meta = json.load(open(os.path.join(HERE, "meta.json")))
    loops = np.load(os.path.join(HERE, "loops.npz"))
    name = "c1_full_cos10_eta0"
    gt, mask = torch.from_numpy(loops[f"{name}/gt"]), torch.from_numpy(loops[f"{name}/mask"])
    torch.manual_seed(meta["loops"][name]["seed"])
    x = torch.randn(1, 3, 256, 256)  # the loop's first draw (code/test_inp_ddim_50.py:481)
    sd = make_state_dict(FULL, seed=1)
    model, _ = mg.ref_model(r_unet, FULL, sd)
    t = torch.tensor([999])
    keep = 1 - mask
    with torch.no_grad():
        y32 = model(x, t, masked_image=gt * keep, mask=1 - keep)
        sd64 = {k: v.double() for k, v in ref_unet.strip_prefix(sd).items()}
        y64 = ref_unet.inpaint_forward(sd64, x, t, gt * keep, 1 - keep, FULL)
    rec["envelopes"]["c1_eval0"] = _stats(y32, y64)
    print(f"[full] c1_eval0: fp32 ref vs fp64 {rec['envelopes']['c1_eval0']}", flush=True)
    np.savez_compressed(os.path.join(OUT, "c1_eval0.npz"), x=x.numpy(), y32=y32.numpy(), y64=y64.numpy())


CASES = {"c1_eval0": case_c1_eval0, "c2_cos100_eta0.75": case_c2, "c3_ddpm_lin1000": case_c3, "c1_fp64": case_c1_fp64,
         "adv_inpaint": case_adv}


def main():
    torch.set_num_threads(int(os.environ.get("GOLDEN_THREADS", "8")))
    os.makedirs(OUT, exist_ok=True)
    todo = sys.argv[1:] or list(CASES)
    r_unet, r_nn, r_gd, r_sched, r_script = mg.import_reference()
    import test_inp_ddim_100 as r_script100
    ref = {"unet": r_unet, "sched": r_sched, "script50": r_script, "script100": r_script100}
    mpath = os.path.join(OUT, "meta_full.json")
    for c in todo:
        rec = {"checks": {}, "envelopes": {}, "loops": {}}
        t0 = time.time()
        CASES[c](ref, rec)
        meta = json.load(open(mpath)) if os.path.exists(mpath) else {"checks": {}, "envelopes": {}, "loops": {}}
        for k in rec:
            meta[k].update(rec[k])
        meta.setdefault("elapsed_s", {})[c] = time.time() - t0
        meta["torch"] = torch.__version__
        with open(mpath, "w") as f:
            json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
