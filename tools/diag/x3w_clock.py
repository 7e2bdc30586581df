"""Shader clock during one wide-unit conv launch (IFD_TRACE build: tools/abl/libifd_trace.so).
usage: IFD_LIB_PATH=... python tools/diag/x3w_clock.py "<layer match>" [B]"""
import os, struct, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "face-inpainting-diffusion-models_amd"))
import numpy as np
import torch
from ifd.manifest import make_state_dict
from ifd.model import DiffusionInpaintingModel
from ifd.topology import FULL
match = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
fn = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "clk.bin")
dev = torch.device("cuda:0")
m = DiffusionInpaintingModel(FULL, device=dev, precision="3xf16"); m.load_state_dict(make_state_dict(FULL, seed=1))
x = torch.randn(B, 3, 256, 256, device=dev); mk = (torch.rand(B, 1, 256, 256, device=dev) > 0.5).float()
t = torch.full((B,), 500, device=dev)
with torch.no_grad():
    m(x, t, masked_image=x, mask=mk)
    os.environ["IFD_TRACE_MATCH"] = match; os.environ["IFD_TRACE_NTH"] = "0"; os.environ["IFD_TRACE_FILE"] = fn
    m(x, t, masked_image=x, mask=mk)
    torch.cuda.synchronize()
a = np.fromfile(fn, dtype=np.uint64).reshape(-1, 64)
a = a[a[:, 0] > 0]
dt, dr = (a[:, 2] - a[:, 0]).astype(np.float64), (a[:, 3] - a[:, 1]).astype(np.float64)
clk = dt / dr * 100e6 / 1e9
print(f"{match}: {len(a)} blocks, launch span {dr.max() / 100:.1f} us, shader clock GHz mean {clk.mean():.3f} min {clk.min():.3f} max {clk.max():.3f}")
