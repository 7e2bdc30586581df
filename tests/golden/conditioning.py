"""Conditioning of the 10-step cosine C1 loops (run here; result recorded in conditioning.json).

Replays the oracle's script DDIM loop (bit-exact with the reference, tests/golden/meta.json) with the
UNet output perturbed by a relative N(0, rel) factor drawn from a SEPARATE generator (the sampler's
RNG stream is untouched), and records the max-abs / percentile deviation from the golden output.
This is the spread ANY fp32 UNet whose rounding differs from oneDNN's by ~rel must expect.
"""
import json, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "face-inpainting-diffusion-models_amd")]
from oracle import ref_unet, ref_diffusion
from ifd.manifest import make_state_dict
from ifd.topology import FULL

def main():
    torch.set_num_threads(8)
    here = os.path.dirname(os.path.abspath(__file__))
    meta = json.load(open(os.path.join(here, "meta.json")))
    loops = np.load(os.path.join(here, "loops.npz"))
    sd = ref_unet.strip_prefix(make_state_dict(FULL, seed=1))
    res = {}
    for name in ("c1_full_cos10_eta0", "c1_full_cos10_eta0.9"):
        lm = meta["loops"][name]
        gt, mask = torch.from_numpy(loops[f"{name}/gt"]), torch.from_numpy(loops[f"{name}/mask"])
        gold = torch.from_numpy(loops[f"{name}/y"])
        tb = ref_diffusion.Tables(ref_diffusion.get_named_beta_schedule(lm["schedule"], lm["T"]))
        for rel in (1e-6, 1e-5):
            for rep in range(2):
                pg = torch.Generator().manual_seed(1000 + rep)
                def unet(x, t, m, k):
                    o = ref_unet.inpaint_forward(sd, x, t, m, k, FULL)
                    return o * (1 + rel * torch.randn(o.shape, generator=pg))
                mf = ref_diffusion.model_fn_factory(unet)
                torch.manual_seed(lm["seed"])
                with torch.no_grad():
                    y = ref_diffusion.script_ddim_loop(tb, mf, (1, 3, 256, 256), gt, mask, lm["ddim_steps"], True, lm["eta"])
                y = ref_diffusion.final_blend(y, gt, mask)
                d = (y.double() - gold.double()).abs().flatten()
                key = f"{name}/rel{rel:g}/rep{rep}"
                res[key] = {"max": float(d.max()), "p999": float(d.quantile(0.999)), "frac_gt_1e-4": float((d > 1e-4).double().mean())}
                print(key, res[key], flush=True)
    json.dump(res, open(os.path.join(here, "conditioning.json"), "w"), indent=1)

if __name__ == "__main__":
    main()
