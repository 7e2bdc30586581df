"""Development: 3xf16 vs fp32 per-eval error on image-like inputs x_t = sqrt(ab) gt + sqrt(1-ab) n
(the states a DDIM loop visits). usage: python tools/diag/x3_img.py"""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "face-inpainting-diffusion-models_amd")]
import torch
from ifd.manifest import make_state_dict
from ifd.model import DiffusionInpaintingModel
from ifd.topology import FULL
from ifd.schedules import create_gaussian_diffusion
dev = torch.device("cuda:0")
sd = make_state_dict(FULL, seed=1)
m3 = DiffusionInpaintingModel(FULL, device=dev, precision="3xf16"); m3.load_state_dict(sd)
m1 = DiffusionInpaintingModel(FULL, device=dev, precision="fp32"); m1.load_state_dict(sd)
diff = create_gaussian_diffusion(steps=1000, learn_sigma=True, noise_schedule="cosine")
g = torch.Generator().manual_seed(0)
gt = (torch.rand(1, 3, 256, 256, generator=g) * 2 - 1)
n = torch.randn(1, 3, 256, 256, generator=g)
mk = torch.zeros(1, 1, 256, 256); mk[:, :, 64:192, 64:192] = 1
gt, n, mk = gt.to(dev), n.to(dev), mk.to(dev)
with torch.no_grad():
    for tv in (999, 900, 700, 500, 300, 100, 0):
        ab = float(diff.alphas_cumprod[tv])
        x = ab ** 0.5 * gt + (1 - ab) ** 0.5 * n
        t = torch.full((1,), tv, device=dev)
        a = m3(x, t, masked_image=gt * (1 - mk), mask=mk)
        b = m1(x, t, masked_image=gt * (1 - mk), mask=mk)
        d = (a - b).abs()
        print(f"t={tv}: |3xf16-fp32| max {float(d.max()):.3e} mean {float(d.mean()):.3e}", flush=True)
