"""Quick timing of one UNet eval at full config (development helper)."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "face-inpainting-diffusion-models_amd"))
import torch
from ifd.manifest import make_state_dict
from ifd.model import DiffusionInpaintingModel
from ifd.topology import FULL, gflop_per_image
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
dev = torch.device("cuda:0")
m = DiffusionInpaintingModel(FULL, device=dev, precision=sys.argv[2] if len(sys.argv) > 2 else "fp32")
m.load_state_dict(make_state_dict(FULL, seed=1))
x = torch.randn(B, 3, 256, 256, device=dev); mk = (torch.rand(B, 1, 256, 256, device=dev) > 0.5).float()
t = torch.full((B,), 500, device=dev)
with torch.no_grad():
    for _ in range(2): y = m(x, t, masked_image=x, mask=mk)
    torch.cuda.synchronize()
    n = int(os.environ.get("QT_N", "5"))
    t0 = time.time()
    for _ in range(n): y = m(x, t, masked_image=x, mask=mk)
    torch.cuda.synchronize()
    dt = (time.time() - t0) / n
print(f"B={B} eval {dt*1e3:.1f} ms  {gflop_per_image()*B/dt/1e3:.1f} TFLOP/s  {dt*1e3/B:.2f} ms/img", flush=True)
