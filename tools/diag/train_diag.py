"""Diagnostic: the training forward against the inference forward and itself (determinism)."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "face-inpainting-diffusion-models_amd")]
import torch
from ifd.manifest import make_state_dict
from ifd.model import DiffusionInpaintingModel
from ifd.topology import REDUCED
from ifd.train import UNetTrainer
from bench import synth_inputs
dev = torch.device("cuda:0")
sd = make_state_dict(REDUCED, seed=1)
tr = UNetTrainer(REDUCED, device=dev)
tr.load_state_dict(sd)
gt, mask = synth_inputs(2, 64, seed=3, device=dev)
g = torch.Generator(device=dev).manual_seed(1)
x = torch.randn(2, 3, 64, 64, device=dev, generator=g)
t = torch.tensor([500, 20], device=dev)
mi = (gt * (1 - mask)).contiguous()
res = {}
with torch.no_grad():
    a = tr.forward(x, t, mi, mask).clone()
    torch.cuda.synchronize()
    sa = {k: {kk: vv.clone() for kk, vv in v.items() if torch.is_tensor(vv)} for k, v in tr._tape["saved"].items()}
    b = tr.forward(x, t, mi, mask).clone()
    torch.cuda.synchronize()
    res["fwd_run_to_run_maxabs"] = float((a - b).abs().max())
    sb = tr._tape["saved"]
    res["saved_diffs"] = {f"{k}/{kk}": float((vv - sb[k][kk]).abs().max()) for k, v in sa.items() for kk, vv in v.items()
                          if float((vv - sb[k][kk]).abs().max()) != 0.0}
    m = DiffusionInpaintingModel(REDUCED, device=dev)
    m.load_state_dict(sd)
    y = m(x, t, masked_image=mi, mask=mask)
    res["fwd_vs_inference_maxabs"] = float((a[..., :6].permute(0, 3, 1, 2) - y).abs().max())
print(json.dumps(res, indent=1))
