"""Where a short 3xf16 conv launch spends its time (IFD_TRACE build of conv_x3.hip): per block the
entry (real-time clock, 100 MHz), the first chunk's start, the chunk intervals and the consumer's end.
usage: IFD_LIB_PATH=<trace build> python tools/diag/x3_span.py "<layer match>" [B] [nth]"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "face-inpainting-diffusion-models_amd"))
import numpy as np
import torch
from ifd.manifest import make_state_dict
from ifd.model import DiffusionInpaintingModel
from ifd.topology import FULL

match = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
nth = sys.argv[3] if len(sys.argv) > 3 else "0"
fn = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "span.bin")
dev = torch.device("cuda:0")
m = DiffusionInpaintingModel(FULL, device=dev, precision="3xf16")
m.load_state_dict(make_state_dict(FULL, seed=1))
x = torch.randn(B, 3, 256, 256, device=dev)
mk = (torch.rand(B, 1, 256, 256, device=dev) > 0.5).float()
t = torch.full((B,), 500, device=dev)
with torch.no_grad():
    m(x, t, masked_image=x, mask=mk)
    os.environ["IFD_TRACE_MATCH"] = match
    os.environ["IFD_TRACE_NTH"] = nth
    os.environ["IFD_TRACE_FILE"] = fn
    m(x, t, masked_image=x, mask=mk)
    torch.cuda.synchronize()
print(open(fn + ".json").read().strip())
a = np.fromfile(fn, dtype=np.uint64).reshape(-1, 64).astype(np.int64)
a = a[a[:, 59] > 0]
rt0 = a[:, 59].min()
ent_us = (a[:, 59] - rt0) / 100.0
end_us = (a[:, 60] - rt0) / 100.0
cyc = a[:, 62] - a[:, 61]
clk = cyc / ((a[:, 60] - a[:, 59]) / 100e6) / 1e9
first = a[:, 0] - a[:, 61]
iv = np.diff(a[:, 0:16], axis=1)
iv = np.where((iv > 0) & (iv < 10**6), iv, np.nan)
q = lambda v: np.percentile(v, [0, 50, 90, 100]).round(1)
print(f"blocks {len(a)}  launch span {end_us.max():.1f} us (first entry -> last consumer end)")
print("entry after first entry, us  [min med p90 max]:", q(ent_us))
print("consumer end, us             [min med p90 max]:", q(end_us))
print("block duration, us           [min med p90 max]:", q(end_us - ent_us))
print("shader clock, GHz            [min med p90 max]:", np.percentile(clk, [0, 50, 90, 100]).round(3))
print("entry -> chunk 0 start, cyc  [min med p90 max]:", q(first))
print("chunk interval, cyc (median per position):", np.nanmedian(iv, axis=0).round(0))
print("first epilogue (start -> end incl. drain), cyc med:", np.median(a[:, 63] - a[:, 43]))
rel = lambda k: np.median(a[:, k] - a[:, 61])
print("fill, cycles after entry (medians): producer chunk 0 issued %d, chunk 1 issued %d, chunk 0 stored %d, "
      "barrier passed %d; consumer at its barrier %d; chunk 0 start %d" % (rel(46), rel(47), rel(56), rel(57), rel(58), rel(0)))
