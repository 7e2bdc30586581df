"""Per-layer conv profile of one UNet eval (development helper): python tools/layer_prof.py [B]"""
import ctypes, json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "face-inpainting-diffusion-models_amd"))
import torch
from ifd import _lib
from ifd.manifest import make_state_dict
from ifd.model import DiffusionInpaintingModel
from ifd.topology import FULL
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
dev = torch.device("cuda:0")
m = DiffusionInpaintingModel(FULL, device=dev, precision=sys.argv[2] if len(sys.argv) > 2 else "fp32"); m.load_state_dict(make_state_dict(FULL, seed=1))
x = torch.randn(B, 3, 256, 256, device=dev); mk = (torch.rand(B, 1, 256, 256, device=dev) > 0.5).float()
t = torch.full((B,), 500, device=dev)
with torch.no_grad():
    for _ in range(2): m(x, t, masked_image=x, mask=mk)
    h = m.handle(dev); L = _lib.lib()
    _lib.check(L.ifd_profile_enable(h.h, 2))
    for _ in range(3): m(x, t, masked_image=x, mask=mk)
    torch.cuda.synchronize()
buf = ctypes.create_string_buffer(1 << 20)
_lib.check(L.ifd_profile_report(h.h, buf, len(buf)))
k = json.loads(buf.value.decode())["kernels"]
tot = sum(v["ms"] for v in k.values())
for name, v in sorted(k.items(), key=lambda kv: -kv[1]["ms"]):
    tf = v["flops"] / (v["ms"] * 1e-3) / 1e12 if v["flops"] else 0
    print(f"{name:60s} n={v['count']:4d} {v['ms']/3:8.3f} ms/eval {tf:6.1f} TF {100*v['ms']/tot:5.1f}%")
print(f"total {tot/3:.2f} ms/eval")
