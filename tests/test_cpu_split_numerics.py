"""CPU check of the 3xf16 split arithmetic (csrc/conv_x3.hip) on the reduced UNet.

Every conv of the oracle UNet is replaced by the split kernel's exact arithmetic:
    a_hi = f16(a), a_lo = f16(a - a_hi); w_hi = f16(w), w_lo' = f16((w - w_hi) 2^11)
    conv(a, w) = [conv(a_hi, w_hi 2^11) + conv(a_hi, w_lo') + conv(a_lo, w_hi 2^11)] 2^-11
(f16 x f16 products are exact in fp32, so fp32 convs of f16-valued tensors reproduce them; only the
accumulation order differs from the MFMA's). The claim tested: against an fp64 evaluation of the
same UNet, the split model's error is of the same size as the plain fp32 model's (bound: 2x), and
the two fp32-class results agree to fp32 accumulation noise. Oracle used as the checker only.
"""
import importlib.util
import os
import sys
import types

import torch
import torch.nn.functional as F

from ifd.manifest import make_state_dict
from oracle import ref_unet

S = 2048.0


def _split_conv(fn, x, w, b, **kw):
    xh = x.half().float()
    xl = (x - xh).half().float()
    wh = w.half().float()
    wl = ((w - wh) * S).half().float()
    y = fn(xh, wh * S, None, **kw) + fn(xh, wl, None, **kw) + fn(xl, wh * S, None, **kw)
    return y / S + b.view(1, -1, *([1] * (x.dim() - 2)))


def _f64_module():
    """The oracle UNet module re-instantiated with .float() -> .double() (fp64 reference)."""
    src = open(ref_unet.__file__).read().replace(".float()", ".double()")
    mod = types.ModuleType("ref_unet_f64")
    sys.modules["ref_unet_f64"] = mod
    exec(compile(src, "ref_unet_f64", "exec"), mod.__dict__)
    return mod


def test_split_conv_matches_fp32_error_level():
    torch.manual_seed(0)
    cfg = ref_unet.REDUCED
    sd = ref_unet.strip_prefix(make_state_dict(cfg, seed=1))
    g = torch.Generator().manual_seed(0)
    R = cfg.image_size
    x = torch.randn(1, 3, R, R, generator=g)
    gt = torch.rand(1, 3, R, R, generator=g) * 2 - 1
    mask = torch.zeros(1, 1, R, R)
    mask[:, :, R // 4:3 * R // 4, R // 4:3 * R // 4] = 1
    t = torch.tensor([999])
    m64 = _f64_module()
    sd64 = {k: v.double() for k, v in sd.items()}
    ref64 = m64.inpaint_forward(sd64, x.double(), t, (gt * (1 - mask)).double(), mask.double(),
                                m64.UNetConfig(**cfg.__dict__))
    y32 = ref_unet.inpaint_forward(sd, x, t, gt * (1 - mask), mask, cfg)
    fw = types.SimpleNamespace(**{k: getattr(F, k) for k in dir(F) if not k.startswith("__")})
    fw.conv2d = lambda a, w, b, padding=0: _split_conv(F.conv2d, a, w, b, padding=padding)
    fw.conv1d = lambda a, w, b: _split_conv(F.conv1d, a, w, b)
    ref_unet.F = fw
    try:
        ys = ref_unet.inpaint_forward(sd, x, t, gt * (1 - mask), mask, cfg)
    finally:
        ref_unet.F = F
    e32 = float((y32.double() - ref64).abs().max())
    es = float((ys.double() - ref64).abs().max())
    print(f"fp32 vs fp64 {e32:.3g}, 3xf16 vs fp64 {es:.3g}")
    assert es <= 2 * e32
    assert float((ys - y32).abs().max()) <= 4 * e32
