"""Development probe: one fused DDIM step (ifd_ddim_step, B = 16 at 256^2) launched eagerly vs replayed from a
HIP graph captured once (same arguments), to price the GPU-side launch gaps of the ~188 kernels per UNet eval.
usage: python tools/graph_probe.py [steps] [batch]"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "face-inpainting-diffusion-models_amd"))
import numpy as np
import torch
from ifd import _lib
from ifd.manifest import make_state_dict
from ifd.model import DiffusionInpaintingModel
from ifd.sampler import ddim_coeffs
from ifd.schedules import create_gaussian_diffusion
from ifd.topology import FULL

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
dev = torch.device("cuda:0")
m = DiffusionInpaintingModel(FULL, device=dev)
m.load_state_dict(make_state_dict(FULL, seed=1))
diff = create_gaussian_diffusion(steps=1000, learn_sigma=True, noise_schedule="cosine")
seq = np.arange(0, 1000, 10)[::-1]
g = torch.Generator(device=dev).manual_seed(0)
img = torch.randn(B, 3, 256, 256, device=dev, generator=g)
gt = torch.randn(B, 3, 256, 256, device=dev, generator=g)
mk = (torch.rand(B, 1, 256, 256, device=dev, generator=g) > 0.5).float()
noise = torch.randn(B, 3, 256, 256, device=dev, generator=g)
known = torch.randn(B, 3, 256, 256, device=dev, generator=g)
t = torch.full((B,), int(seq[10]), device=dev, dtype=torch.int64)
c = ddim_coeffs(diff.alphas_cumprod, seq, 10, 0.75, True)
L = _lib.lib()
h = m.handle(dev)


def step():
    _lib.check(L.ifd_ddim_step(h.h, _lib.ptr(t), B, 256, 256, _lib.ptr(img), _lib.ptr(gt), _lib.ptr(mk), _lib.ptr(noise),
                               _lib.ptr(known), c, _lib.stream_ptr(dev)))


s = torch.cuda.Stream(device=dev)
with torch.no_grad(), torch.cuda.stream(s):
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(K):
        step()
    e1.record(s)
    torch.cuda.synchronize()
    eager = e0.elapsed_time(e1) / K
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        step()
    torch.cuda.synchronize()
    for _ in range(2):
        gr.replay()
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(K):
        gr.replay()
    e1.record(s)
    torch.cuda.synchronize()
    graph = e0.elapsed_time(e1) / K
print(f"eager {eager:.3f} ms per step, graph replay {graph:.3f} ms per step ({100 * (1 - graph / eager):.2f} % less)")
