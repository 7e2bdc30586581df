"""Development: per-step model outputs along the C1 eta-0 loop. mode dump: run the 3xf16 loop
(unfused), save each step's input state and 3xf16 output; mode eval: re-evaluate those states with
this library in 3xf16 and fp32 and compare. usage: python tools/diag/c1_states.py dump|eval FILE"""
import os, sys
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "face-inpainting-diffusion-models_amd")]
import json
import numpy as np
import torch
from ifd.manifest import make_state_dict
from ifd.model import DiffusionInpaintingModel
from ifd.topology import FULL
from ifd.sampler import InpaintingSampler
from ifd.schedules import create_gaussian_diffusion
mode, fn = sys.argv[1], sys.argv[2]
DEV = torch.device("cuda:0")
G = os.path.join(ROOT, "tests", "golden")
meta = json.load(open(os.path.join(G, "meta.json")))
loops = np.load(os.path.join(G, "loops.npz"))
name = "c1_full_cos10_eta0"
lm = meta["loops"][name]
sd = make_state_dict(FULL, seed=1)
m = DiffusionInpaintingModel(FULL, device=DEV, precision="3xf16"); m.load_state_dict(sd)
gt = torch.from_numpy(loops[f"{name}/gt"]).to(DEV)
mask = torch.from_numpy(loops[f"{name}/mask"]).to(DEV)
if mode == "dump":
    diff = create_gaussian_diffusion(steps=lm["T"], learn_sigma=True, noise_schedule=lm["schedule"])
    s = InpaintingSampler(m, diff, ddim_timesteps=lm["ddim_steps"], device=DEV, noise_device="cpu")
    rec = {}
    def mf(x, t, **kw):
        o = s.model_fn(x, t, **kw)
        k = len(rec) // 3
        rec[f"x{k}"] = x.cpu().numpy(); rec[f"t{k}"] = t.cpu().numpy(); rec[f"o{k}"] = o.cpu().numpy()
        return o
    torch.manual_seed(lm["seed"])
    with torch.no_grad():
        s.inpainting_ddim_sample_loop(mf, (1, 3, 256, 256), gt, mask, True, DEV, False, lm["eta"])
    np.savez(fn, **rec)
else:
    z = np.load(fn)
    m1 = DiffusionInpaintingModel(FULL, device=DEV, precision="fp32"); m1.load_state_dict(sd)
    keep = 1 - mask
    with torch.no_grad():
        for k in range(len(z.files) // 3):
            x = torch.from_numpy(z[f"x{k}"]).to(DEV); t = torch.from_numpy(z[f"t{k}"]).to(DEV)
            ho = torch.from_numpy(z[f"o{k}"]).to(DEV)
            a = m(x, t, masked_image=gt * keep, mask=mask)
            b = m1(x, t, masked_image=gt * keep, mask=mask)
            f = lambda d: f"max {float(d.abs().max()):.2e} mean {float(d.abs().mean()):.2e}"
            print(f"step {k} t={int(t[0])}: |new-head| {f(a - ho)} |new-fp32| {f(a - b)} |head-fp32| {f(ho - b)}", flush=True)
