"""Development: 3xf16 vs fp32 on the B=3 input of tests/test_gpu_x3.py::test_x3_matches_fp32_batch, under
x3_off masks (1 no 16x16, 2 no split-K, 4 no skip layers, 8 no 8x8, 16 no 1x1). usage: x3_b3.py [B]"""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "face-inpainting-diffusion-models_amd")]
import torch
from ifd.manifest import make_state_dict
from ifd.model import DiffusionInpaintingModel
from ifd.topology import FULL
B = int(sys.argv[1]) if len(sys.argv) > 1 else 3
DEV = torch.device("cuda:0")
sd = make_state_dict(FULL, seed=1)
g = torch.Generator(device=DEV).manual_seed(11)
x = torch.randn(B, 3, 256, 256, device=DEV, generator=g)
gt = torch.rand(B, 3, 256, 256, device=DEV, generator=g) * 2 - 1
mask = (torch.rand(B, 1, 256, 256, device=DEV, generator=g) > 0.5).float()
t = torch.tensor([999, 500, 3, 100][:B], device=DEV)
m32 = DiffusionInpaintingModel(FULL, device=DEV); m32.load_state_dict(sd)
with torch.no_grad():
    y32 = m32(x, t, masked_image=gt * (1 - mask), mask=mask)
    for off in (0, 1, 2, 3, 8, 11, 31):
        m3 = DiffusionInpaintingModel(FULL, device=DEV, precision="3xf16", options={"x3_off": off}); m3.load_state_dict(sd)
        y3 = m3(x, t, masked_image=gt * (1 - mask), mask=mask)
        print(f"B={B} x3_off={off}: maxabs {float((y3 - y32).abs().max()):.3e}", flush=True)
