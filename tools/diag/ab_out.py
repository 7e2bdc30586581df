"""Development: one B=4 UNet eval (3xf16 and fp32) with the library at IFD_LIB_PATH (default in-tree), saved
to argv[1]; with argv[2], compared to that earlier file (bit equality and max-abs).
usage: python tools/diag/ab_out.py OUT.npz [REF.npz]"""
import os, sys
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "face-inpainting-diffusion-models_amd")]
import numpy as np
import torch
from ifd.manifest import make_state_dict
from ifd.model import DiffusionInpaintingModel
from ifd.topology import FULL
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(5)
B = 4
x = torch.randn(B, 3, 256, 256, device=dev, generator=g)
gt = torch.rand(B, 3, 256, 256, device=dev, generator=g) * 2 - 1
mask = (torch.rand(B, 1, 256, 256, device=dev, generator=g) > 0.5).float()
t = torch.tensor([999, 640, 120, 7], device=dev)
out = {}
sd = make_state_dict(FULL, seed=1)
for prec in ("3xf16", "fp32", "f16"):
    m = DiffusionInpaintingModel(FULL, device=dev, precision=prec)
    m.load_state_dict(sd)
    with torch.no_grad():
        out[prec] = m(x, t, masked_image=gt * (1 - mask), mask=mask).cpu().numpy()
    del m
np.savez(sys.argv[1], **out)
if len(sys.argv) > 2:
    ref = np.load(sys.argv[2])
    for k in out:
        print(k, "bit-equal" if np.array_equal(out[k], ref[k]) else "DIFFERENT", float(np.abs(out[k] - ref[k]).max()))
