"""Development: 3xf16 training step vs fp32 at the full config (B=4): loss, grad norm and the worst
per-tensor gradient errors, for forward-only (x3_dgrad=False) and forward + dgrad at several loss scales."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
_R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(_R, "tests"))
sys.path.insert(0, os.path.join(_R, "face-inpainting-diffusion-models_amd"))
import numpy as np
import torch
from test_gpu_train import _full_step

tr32, l32 = _full_step("fp32")
g32 = tr32.grad.clone(); n32 = float(tr32.norm_coef[0]); offs = tr32.offsets
del tr32
for kw in (dict(x3_dgrad=False, x3_wgrad=False), dict(x3_wgrad=False), dict(x3_loss_scale_log2=14), dict(x3_loss_scale_log2=20), dict(x3_loss_scale_log2=24)):
    tr, l = _full_step("3xf16", **kw)
    errs = []
    for k, (o, shape) in offs.items():
        n = int(np.prod(shape)); a, b = tr.grad[o:o + n].double(), g32[o:o + n].double()
        bn = float(b.norm())
        if bn > 0: errs.append((float((a - b).norm()) / bn, k))
    errs.sort(reverse=True)
    print(kw, "trips", tr.guard_trips, "rel_loss %.2e" % (abs(l - l32) / abs(l32)),
          "rel_gn %.2e" % (abs(float(tr.norm_coef[0]) - n32) / n32), "worst", ["%.2e %s" % e for e in errs[:4]],
          "median %.2e" % errs[len(errs) // 2][0], flush=True)
    del tr
