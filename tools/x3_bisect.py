"""Development: 3xf16 full-UNet eval vs the golden fixture under the IFD_X3_OFF switches."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "face-inpainting-diffusion-models_amd")]
import numpy as np
import torch
from ifd.manifest import make_state_dict
from ifd.model import DiffusionInpaintingModel
from ifd.topology import FULL
ev = dict(np.load(os.path.join(sys.path[0], "tests", "golden", "unet_evals.npz")))
dev = torch.device("cuda:0")
m = DiffusionInpaintingModel(FULL, device=dev, precision="3xf16")
m.load_state_dict(make_state_dict(FULL, seed=1))
x, gt, mk = (torch.from_numpy(ev[f"full/{k}"]).to(dev) for k in ("x", "gt", "mask"))
with torch.no_grad():
    y = m(x, torch.tensor([999], device=dev), masked_image=gt * (1 - mk), mask=mk)
ref = torch.from_numpy(ev["full_t999/y"])
d = (y.double().cpu() - ref.double()).abs()
print(f"IFD_X3_OFF={os.environ.get('IFD_X3_OFF', '0')} maxabs={float(d.max()):.3g} nan={int(torch.isnan(y).sum())}", flush=True)
