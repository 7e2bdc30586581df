"""development: one 3xf16 UNet eval (B = 2, fixed inputs) with the library IFD_LIB_PATH names, saved to
gpurun_out/cmp_<name>.npy; with --against NAME also prints max-abs vs that saved output.
usage: IFD_LIB_PATH=tools/abl/libifd_X.so python tools/abl/cmp_lib.py X [--against base]"""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [R, os.path.join(R, "face-inpainting-diffusion-models_amd")]
import numpy as np
import torch
from ifd.manifest import make_state_dict
from ifd.model import DiffusionInpaintingModel
from ifd.topology import FULL
name = sys.argv[1]
out = os.path.join(os.environ.get("GRAFT_REPO_ROOT", R), "gpurun_out")
os.makedirs(out, exist_ok=True)
dev = torch.device("cuda:0")
m = DiffusionInpaintingModel(FULL, device=dev, precision="3xf16")
m.load_state_dict(make_state_dict(FULL, seed=1))
g = torch.Generator().manual_seed(3)
x = torch.randn(2, 3, 256, 256, generator=g).to(dev)
mk = (torch.rand(2, 1, 256, 256, generator=g) > 0.5).float().to(dev)
t = torch.tensor([999, 400], device=dev)
with torch.no_grad():
    y = m(x, t, masked_image=x * (1 - mk), mask=mk).cpu().numpy()
np.save(os.path.join(out, f"cmp_{name}.npy"), y)
if "--against" in sys.argv:
    ref = np.load(os.path.join(out, f"cmp_{sys.argv[sys.argv.index('--against') + 1]}.npy"))
    print(f"{name}: max-abs vs reference lib {np.abs(y - ref).max():.3g}, bit-equal {np.array_equal(y, ref)}")
