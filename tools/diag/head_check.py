"""Development: does the 3xf16 forward run the split-MFMA head? Output of a full-size eval with the head
option on vs off (x3_off bit 32) and the kernel names of one profiled forward."""
import ctypes, json, os, sys
_R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(_R, "face-inpainting-diffusion-models_amd"))
import torch
from ifd import _lib
from ifd.manifest import make_state_dict
from ifd.model import DiffusionInpaintingModel
from ifd.topology import FULL
dev = torch.device("cuda:0")
m = DiffusionInpaintingModel(FULL, device=dev, precision="3xf16")
m.load_state_dict(make_state_dict(FULL, seed=1))
g = torch.Generator().manual_seed(3)
x = torch.randn(2, 3, 256, 256, generator=g).to(dev)
mk = (torch.rand(2, 1, 256, 256, generator=g) > 0.5).float().to(dev)
t = torch.full((2,), 500, device=dev)
h = m.handle(dev)
L = _lib.lib()
outs = []
for off in (0, 32):
    _lib.check(L.ifd_set_option(h.h, b"x3_off", off))
    with torch.no_grad():
        _lib.check(L.ifd_profile_enable(h.h, 1))
        y = m(x, t, masked_image=x * (1 - mk), mask=mk)
        torch.cuda.synchronize()
        buf = ctypes.create_string_buffer(1 << 16)
        _lib.check(L.ifd_profile_report(h.h, buf, len(buf)))
        _lib.check(L.ifd_profile_enable(h.h, 0))
    names = [k for k in json.loads(buf.value.decode())["kernels"] if "head" in k]
    outs.append(y.clone())
    print("x3_off", off, "head kernels", names, flush=True)
print("max |head_x3 - head_fp32| =", float((outs[0] - outs[1]).abs().max()))
