"""The wide-unit split kernel (conv_x3w.hip, through ifd_tr_conv_x3w) on single 3x3 convs against an
fp64 torch reference of the same op: out = conv3x3(act(xform(cat(x0, x1)))) + bias [+ residual], the
prologue act = silu(A v + B) / A v + B / identity (code/nn.py ResBlock in_layers / out_layers with
the GroupNorm folded into per-(image, channel) A, B), xform = nearest-up x2 (code/nn.py Upsample /
ResBlock h_upd), zero padding after act (torch pads the activated tensor).

The split arithmetic is fp32-class: error bound 2e-5 x (max|ref| + 1) at these fan-ins (fp32's own
accumulation over K = 9 Cin terms is ~1e-6 relative). The granule statistics are checked against the
output's own (mean, M2) per (image, channel quad, 8x16 tile).
"""
import ctypes

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")

CASES = [  # N, H(out), c0, c1, cout, act, xform, res (0 none, 1 same size, 2 upsampled)
    (2, 32, 128, 0, 128, 0, 0, 0),
    (2, 32, 128, 0, 128, 2, 0, 1),
    (1, 64, 64, 64, 256, 2, 0, 0),
    (2, 32, 128, 0, 128, 1, 1, 2),
    (1, 16, 256, 128, 128, 2, 0, 1),
]


@pytest.mark.parametrize("case", CASES, ids=[f"n{c[0]}_h{c[1]}_{c[2]}+{c[3]}to{c[4]}_a{c[5]}_x{c[6]}_r{c[7]}" for c in CASES])
def test_conv_x3w_vs_fp64(case, record):
    from ifd import _lib
    from ifd.train import P, chk, lib

    N, H, c0, c1, cout, act, xf, res = case
    Hin = H // 2 if xf else H
    cin = c0 + c1
    g = torch.Generator().manual_seed(sum(case))
    x0 = torch.randn(N, Hin, Hin, c0, generator=g) + 0.3
    x1 = torch.randn(N, Hin, Hin, c1, generator=g) if c1 else None
    w = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    b = 0.3 * torch.randn(cout, generator=g)
    A = 1 + 0.3 * torch.randn(N, cin, generator=g)
    B = 0.3 * torch.randn(N, cin, generator=g)
    rH = H // 2 if res == 2 else H
    r = torch.randn(N, rH, rH, cout, generator=g) if res else None

    # fp64 reference (NCHW)
    x = torch.cat([x0, x1], -1) if c1 else x0
    v = x.double().permute(0, 3, 1, 2)
    if act:
        v = A.double()[:, :, None, None] * v + B.double()[:, :, None, None]
        if act == 2:
            v = v * torch.sigmoid(v)
    if xf:
        v = F.interpolate(v, scale_factor=2, mode="nearest")
    ref = F.conv2d(v, w.double(), b.double(), padding=1)
    if res:
        rr = r.double().permute(0, 3, 1, 2)
        if res == 2:
            rr = F.interpolate(rr, scale_factor=2, mode="nearest")
        ref = rr + ref
    ref = ref.permute(0, 2, 3, 1)

    s = _lib.stream_ptr(DEV)
    guard = torch.zeros(4, device=DEV, dtype=torch.int32)
    wd = w.to(DEV)
    wx = torch.empty(lib().ifd_tr_x3w_pack_bytes(cout, cin) // 4, device=DEV)
    chk(lib().ifd_tr_pack_conv_x3w(P(wd), cout, cin, cin, P(wx), P(guard), s))
    d = {k: (t.to(DEV).contiguous() if t is not None else None) for k, t in
         dict(x0=x0, x1=x1, b=b, A=A, B=B, r=r).items()}
    out = torch.empty(N, H, H, cout, device=DEV)
    gf = N * (cout // 4) * (H * H // 128) * 2
    gstat = torch.empty(gf, device=DEV)
    E, cnt = ctypes.c_int(0), ctypes.c_float(0.0)
    chk(lib().ifd_tr_conv_x3w(P(d["x0"]), c0, P(d["x1"]), c1, N, H, xf, P(wx), P(d["b"]), cin, cout, act,
                              P(d["A"]), P(d["B"]), P(d["r"]), 1 if res == 2 else 0, P(out), P(guard), P(gstat), gf,
                              ctypes.byref(E), ctypes.byref(cnt), s))
    torch.cuda.synchronize()
    y = out.double().cpu()
    err = float((y - ref).abs().max())
    scale = float(ref.abs().max()) + 1
    record(f"conv_x3w/{'_'.join(map(str, case))}", maxabs=err, ref_max=scale - 1)
    assert int(guard.cpu()[0]) == 0
    assert err <= 2e-5 * scale, (err, scale)
    # granule statistics: entry e = tile (y0 / 8) * (W / 16) + x0 / 16, 4 channels x 128 pixels
    assert E.value == H * H // 128 and cnt.value == 512.0
    gs = gstat.double().cpu().view(N, cout // 4, E.value, 2)
    t = y.view(N, H // 8, 8, H // 16, 16, cout // 4, 4).permute(0, 5, 1, 3, 2, 4, 6).reshape(N, cout // 4, E.value, 512)
    mean = t.mean(-1)
    m2 = ((t - mean[..., None]) ** 2).sum(-1)
    assert float((gs[..., 0] - mean).abs().max()) <= 1e-5 * scale
    assert float(((gs[..., 1] - m2).abs() / (m2 + 1e-3)).max()) <= 1e-4
