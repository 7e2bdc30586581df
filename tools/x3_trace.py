"""Development: per-interval cycle stamps of one 3xf16 conv launch (IFD_TRACE build).
usage: IFD_LIB_PATH=tools/abl/libifd_trace.so python tools/x3_trace.py '<layer match>' [B]"""
import os, sys
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "face-inpainting-diffusion-models_amd")]
import numpy as np
import torch
from ifd.manifest import make_state_dict
from ifd.model import DiffusionInpaintingModel
from ifd.topology import FULL
match = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
out = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "x3trace.bin")
dev = torch.device("cuda:0")
m = DiffusionInpaintingModel(FULL, device=dev, precision="3xf16")
m.load_state_dict(make_state_dict(FULL, seed=1))
x = torch.randn(B, 3, 256, 256, device=dev); mk = (torch.rand(B, 1, 256, 256, device=dev) > 0.5).float()
t = torch.full((B,), 500, device=dev)
with torch.no_grad():
    m(x, t, masked_image=x, mask=mk)
    torch.cuda.synchronize()
    os.environ["IFD_TRACE_MATCH"] = match
    os.environ["IFD_TRACE_FILE"] = out
    m(x, t, masked_image=x, mask=mk)
    torch.cuda.synchronize()
tr = np.fromfile(out, dtype=np.uint64).reshape(-1, 64).astype(np.int64)
print(open(out + ".json").read().strip())
blk = tr[:256]
cs, ce, pi, ps = blk[:, 0:16], blk[:, 16:32], blk[:, 32:48], blk[:, 48:64]
np.set_printoptions(linewidth=220)
med = lambda a: np.median(a, axis=0).astype(int)
print("interval (consumer start j -> j+1):", med(np.diff(cs, axis=1)))
print("consumer issue (start -> MFMAs issued):", med(ce - cs))
# the producer stamps cover intervals 0..7 only (slots 32..39 and 48..55; 40..47 and 56..63 hold the fill
# and the consumer's first-epilogue stamps). Producer interval j starts with the consumer's chunk j.
pi, ps = pi[:, :8], ps[:, :8]
print("producer: interval start -> LDS writes of the next chunk done (j = 0..7):", med(ps - cs[:, :8]))
print("producer: interval start -> DMA + loads issued (j = 0..7):", med(pi - cs[:, :8]))
print("producer: issued -> next interval start (its wait at the barrier):", med(cs[:, 1:9] - pi))
print("first epilogue: start after chunk 0 start", int(np.median(blk[:, 43] - cs[:, 0])),
      "; phases from its start (values [+ stores] issued, statistics [+ stores] issued, epilogue end):",
      [int(np.median(blk[:, k] - blk[:, 43])) for k in (44, 45, 63)])
