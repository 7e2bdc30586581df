"""Development: determinism of the split kernels (repeat evals bit-identical?) and their distance to
fp32 mode at several t. usage: python tools/diag/x3_det.py [B]"""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "face-inpainting-diffusion-models_amd")]
import torch
from ifd.manifest import make_state_dict
from ifd.model import DiffusionInpaintingModel
from ifd.topology import FULL
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
dev = torch.device("cuda:0")
sd = make_state_dict(FULL, seed=1)
m3 = DiffusionInpaintingModel(FULL, device=dev, precision="3xf16"); m3.load_state_dict(sd)
m1 = DiffusionInpaintingModel(FULL, device=dev, precision="fp32"); m1.load_state_dict(sd)
g = torch.Generator().manual_seed(0)
x = torch.randn(B, 3, 256, 256, generator=g).to(dev)
gt = (torch.rand(B, 3, 256, 256, generator=g) * 2 - 1).to(dev)
mk = torch.zeros(B, 1, 256, 256); mk[:, :, 64:192, 64:192] = 1; mk = mk.to(dev)
with torch.no_grad():
    for tv in (999, 899, 500, 100, 0):
        t = torch.full((B,), tv, device=dev)
        outs = [m3(x, t, masked_image=gt * (1 - mk), mask=mk).clone() for _ in range(4)]
        ref = m1(x, t, masked_image=gt * (1 - mk), mask=mk)
        same = all(torch.equal(outs[0], o) for o in outs[1:])
        spread = max(float((outs[0] - o).abs().max()) for o in outs[1:])
        print(f"t={tv}: repeat bit-identical={same} spread={spread:.3e} |3xf16-fp32| max={float((outs[0]-ref).abs().max()):.3e}", flush=True)
