"""Bisect the wide-unit kernel's plan (development helper): UNet outputs under option sets vs x3w=0."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "face-inpainting-diffusion-models_amd"))
import torch
from ifd.manifest import make_state_dict
from ifd.model import DiffusionInpaintingModel
from ifd.topology import FULL
dev = torch.device("cuda:0")
sd = make_state_dict(FULL, seed=1)
g = torch.Generator(device=dev).manual_seed(3)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
x = torch.randn(B, 3, 256, 256, device=dev, generator=g)
mk = (torch.rand(B, 1, 256, 256, device=dev, generator=g) > 0.5).float()
t = torch.full((B,), 500, device=dev)
def run(opts):
    m = DiffusionInpaintingModel(FULL, device=dev, precision="3xf16", options=opts)
    m.load_state_dict(sd)
    with torch.no_grad():
        return m(x, t, masked_image=x, mask=mk).double().cpu()
ref = run({"x3w": 0})
for opts in ({"x3w": 256}, {"x3w": 128}, {"x3w": 64}, {"x3w": 256, "gn_fused": 0}, {"x3w": 256, "skip_sep": 0},
             {"x3w": 64, "skip_sep": 0, "gn_fused": 0}):
    y = run(opts)
    print(opts, "maxabs", float((y - ref).abs().max()), "finite", bool(torch.isfinite(y).all()), flush=True)
