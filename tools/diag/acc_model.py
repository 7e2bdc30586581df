"""Accumulation-order model of the conv kernels' rounding (CPU, diagnostic only).

Every conv of the oracle UNet is replaced by an emulation of how the MFMA kernels round:
  * fp32chain: v_mfma_f32_32x32x2_f32 = one fp32 rounding per product, K sequential (the exact-fp32 mode);
  * x3one:     3xf16 split, the three products of every tap in ONE fp32 accumulator, each
               v_mfma_f32_32x32x16_f16 = two groups of 8 exact products, one rounding per group;
  * x3sep:     the same, with the two correction products (hi*lo', lo*hi) in a SECOND accumulator,
               added to the main one once per output;
  * x3wino:    Winograd F(2x2,3x3) for the 3x3 convs (round 6): the input transform B^T d B in fp32
               (adds only, as a producer wave would stage it), the weight transform G g G^T in fp64 then split
               like the weights above, the 16 elementwise GEMMs over K = Cin on the x3sep arithmetic, the output
               transform A^T M A in fp32 (1x1 convs stay x3sep); x3wino1: the same with the correction products
               in the main accumulator (no second accumulator set: half the registers);
  * ref:       torch's fp32 conv (the reference's arithmetic class).
and compared against the fp64 UNet. Usage: python tools/diag/acc_model.py [reduced|full] [t]
"""
import sys
import types

import torch
import torch.nn.functional as F

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/face-inpainting-diffusion-models_amd")
from ifd.manifest import make_state_dict  # noqa: E402
from oracle import ref_unet  # noqa: E402

S = 2048.0


def _split(v):
    h = v.half().float()
    return h, (v - h).half().float()


_BT = torch.tensor([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], dtype=torch.float64)
_G = torch.tensor([[1, 0, 0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0, 0, 1]], dtype=torch.float64)
_AT = torch.tensor([[1, 1, 1, 0], [0, 1, -1, -1]], dtype=torch.float64)


def wino_emul(x, w, b, sep=True):
    """F(2x2,3x3), padding 1, even H and W: Y = A^T [ (G g G^T) . (B^T d B) ] A per 2x2 output tile."""
    n, c, _, _ = w.shape
    B, _, H, W = x.shape
    cp = (c + 15) // 16 * 16
    xp = F.pad(x, (1, 1, 1, 1, 0, cp - c))
    wp = F.pad(w, (0, 0, 0, 0, 0, cp - c))
    th, tw = H // 2, W // 2
    d = xp.unfold(2, 4, 2).unfold(3, 4, 2)  # [B, cp, th, tw, 4, 4], fp32
    bt = _BT.float()
    v = torch.einsum("ia,zctuae->zctuie", bt, d)  # B^T d (each entry a sum of two fp32 values)
    v = torch.einsum("zctuia,ja->zctuij", v, bt)  # (B^T d) B
    v = v.reshape(B, cp, th * tw, 16).permute(0, 1, 3, 2).contiguous()  # [B, cp, xi, T]
    u = torch.einsum("ia,ncab,jb->ncij", _G, wp.double(), _G).reshape(n, cp, 16).permute(2, 0, 1)  # [xi, n, cp]
    vh, vl = _split(v)
    uh = u.float().half().float()
    ul = ((u - uh.double()) * S).half().float()
    uhs, ulv = uh.double() * S, ul.double()
    acc = torch.zeros(B, n, 16, th * tw, dtype=torch.float32)
    accl = torch.zeros_like(acc)
    for c0 in range(0, cp, 16):
        for (ua, va, lo) in ((uhs, vh, False), (ulv, vh, True), (uhs, vl, True)):
            for g in range(2):
                cs = slice(c0 + 8 * g, c0 + 8 * g + 8)
                s = torch.einsum("xnk,bkxt->bnxt", ua[:, :, cs], va[:, cs].double())
                if lo and sep:
                    accl = (accl.double() + s).float()
                else:
                    acc = (acc.double() + s).float()
    m = ((acc + accl) / S).view(B, n, 4, 4, th, tw)
    at = _AT.float()
    y = torch.einsum("ia,znaetu->znietu", at, m)
    y = torch.einsum("znietu,je->znijtu", y, at)  # [B, n, 2, 2, th, tw]
    y = y.permute(0, 1, 4, 2, 5, 3).reshape(B, n, H, W)
    return y + b.view(1, -1, 1, 1)


def conv_emul(mode, x, w, b, padding=0):
    if mode == "ref":
        return F.conv2d(x, w, b, padding=padding)
    if mode in ("x3wino", "x3wino1"):
        if w.shape[-1] == 3 and padding == 1 and x.shape[-1] % 2 == 0 and x.shape[-2] % 2 == 0:
            return wino_emul(x, w, b, sep=mode == "x3wino")
        mode = "x3sep"
    n, c, kh, kw = w.shape
    T = kh * kw
    B, _, H, W = x.shape
    cp = (c + 15) // 16 * 16
    xp = F.pad(x, (0, 0, 0, 0, 0, cp - c))
    wp = F.pad(w, (0, 0, 0, 0, 0, cp - c))
    if mode == "fp32chain":
        xu = F.unfold(xp.double(), (kh, kw), padding=padding).view(B, cp, T, -1)
        wv = wp.double().view(n, cp, T)
        acc = torch.zeros(B, n, xu.shape[-1], dtype=torch.float32)
        for c0 in range(0, cp, 8):
            for tap in range(T):
                for ci in range(c0, c0 + 8):
                    acc = (acc.double() + wv[:, ci, tap][None, :, None] * xu[:, ci, tap][:, None, :]).float()
    else:
        xh, xl = _split(xp)
        wh = wp.half().float()
        wl = ((wp - wh) * S).half().float()
        uh = F.unfold(xh.double(), (kh, kw), padding=padding).view(B, cp, T, -1)
        ul = F.unfold(xl.double(), (kh, kw), padding=padding).view(B, cp, T, -1)
        whs = (wh.double() * S).view(n, cp, T)
        wlv = wl.double().view(n, cp, T)
        acc = torch.zeros(B, n, uh.shape[-1], dtype=torch.float32)
        accl = torch.zeros_like(acc)
        for c0 in range(0, cp, 16):
            for tap in range(T):
                for (wa, ua, lo) in ((whs, uh, False), (wlv, uh, True), (whs, ul, True)):
                    for g in range(2):
                        cs = slice(c0 + 8 * g, c0 + 8 * g + 8)
                        s = torch.einsum("nk,bkm->bnm", wa[:, cs, tap], ua[:, cs, tap])
                        if mode == "x3sep" and lo:
                            accl = (accl.double() + s).float()
                        else:
                            acc = (acc.double() + s).float()
        if mode == "x3sep":
            acc = acc + accl
        acc = acc / S
    y = acc.view(B, n, H + 2 * padding - kh + 1, W + 2 * padding - kw + 1)
    return y + b.view(1, -1, 1, 1)


def _f64_module():
    src = open(ref_unet.__file__).read().replace(".float()", ".double()")
    mod = types.ModuleType("ref_unet_f64")
    sys.modules["ref_unet_f64"] = mod
    exec(compile(src, "ref_unet_f64", "exec"), mod.__dict__)
    return mod


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "reduced"
    tt = int(sys.argv[2]) if len(sys.argv) > 2 else 999
    modes = sys.argv[3].split(",") if len(sys.argv) > 3 else ["ref", "x3one", "x3sep", "x3wino", "fp32chain"]
    cfg = ref_unet.REDUCED if which == "reduced" else ref_unet.FULL
    torch.manual_seed(0)
    sd = ref_unet.strip_prefix(make_state_dict(cfg, seed=1))
    g = torch.Generator().manual_seed(0)
    R = cfg.image_size
    x = torch.randn(1, 3, R, R, generator=g)
    gt = torch.rand(1, 3, R, R, generator=g) * 2 - 1
    mask = torch.zeros(1, 1, R, R)
    mask[:, :, R // 4:3 * R // 4, R // 4:3 * R // 4] = 1
    t = torch.tensor([tt])
    m64 = _f64_module()
    sd64 = {k: v.double() for k, v in sd.items()}
    y64 = m64.inpaint_forward(sd64, x.double(), t, (gt * (1 - mask)).double(), mask.double(),
                              m64.UNetConfig(**cfg.__dict__))
    for mode in modes:
        fw = types.SimpleNamespace(**{k: getattr(F, k) for k in dir(F) if not k.startswith("__")})
        fw.conv2d = lambda a, w, b, padding=0, _m=mode: conv_emul(_m, a, w, b, padding)
        fw.conv1d = lambda a, w, b, _m=mode: conv_emul(_m, a[..., None], w[..., None], b)[..., 0]
        ref_unet.F = fw
        try:
            y = ref_unet.inpaint_forward(sd, x, t, gt * (1 - mask), mask, cfg)
        finally:
            ref_unet.F = F
        d = (y.double() - y64).abs().flatten()
        print(f"{which} t={tt} {mode:10s} max {float(d.max()):.3e} p999 {float(d.quantile(0.999)):.3e} "
              f"mean {float(d.mean()):.3e}", flush=True)


if __name__ == "__main__":
    main()
