"""The split weight gradient (ifd_tr_conv_wgrad_x3, csrc/train_ops.hip: wgrad_ws_kernel for 3x3, wgrad_x3_kernel
for 1x1) against the fp32 weight gradient (ifd_tr_conv_wgrad, fp32 MFMA) and a float64 torch reference on the
same inputs: the training backward's dW[co][ci][tap] = sum_p dY[p][co] X[p + off(tap)][ci] (code/nn.py conv
layers' autograd) and dB = column sums of dY.

Shapes cover 32-wide chunks (W >= 32), 8 x 8 maps (one chunk = whole images), output / input channel
tiles that are partly filled (cout 8, cin 96), an odd batch, and the 1x1 kernel.
Gates (3xf16: three f16 products per MAC, fp32 accumulation): rel-L2 vs float64 <= 2e-6 and within
2x the fp32 kernel's own rel-L2 + 1e-7; the bias gradient rel-L2 <= 1e-6.
"""
import ctypes

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")

CASES = [  # N, H, cin, cout, taps
    (2, 32, 128, 128, 9),
    (3, 64, 64, 128, 9),
    (4, 8, 256, 512, 9),
    (2, 16, 96, 8, 9),
    (2, 32, 256, 128, 1),
]


def _ref(dy, x, taps):
    """float64 dW [cout][cin][taps], dB [cout] from NHWC fp32 tensors."""
    xd = x.double().permute(0, 3, 1, 2)
    dyd = dy.double().permute(0, 3, 1, 2)
    k = 3 if taps == 9 else 1
    w = torch.zeros(dy.shape[-1], x.shape[-1], k, k, dtype=torch.float64, device=x.device, requires_grad=True)
    y = F.conv2d(xd, w, padding=k // 2)
    (y * dyd).sum().backward()
    return w.grad.reshape(w.shape[0], w.shape[1], taps), dyd.sum(dim=(0, 2, 3))


@pytest.mark.parametrize("N,H,cin,cout,taps", CASES)
def test_wgrad_x3_vs_fp64(N, H, cin, cout, taps, record):
    from ifd import _lib
    from ifd.train import P, chk, lib

    s = _lib.stream_ptr(DEV)
    g = torch.Generator().manual_seed(N * 1000 + H + cin + cout)
    x = (torch.randn(N, H, H, cin, generator=g) * 0.8 + 0.2).to(DEV)
    dy = torch.randn(N, H, H, cout, generator=g).to(DEV)
    P_ = N * H * H
    S = ctypes.c_int()
    need = lib().ifd_tr_wgrad_part_floats(cout, cin, taps, P_, ctypes.byref(S))
    part = torch.empty(need, device=DEV)
    colpart = torch.empty(((P_ + 1023) // 1024) * cout, device=DEV)
    guard = torch.zeros(4, device=DEV, dtype=torch.int32)
    out = {}
    for kind in ("fp32", "x3"):
        dw, db = torch.zeros(cout * cin * taps, device=DEV), torch.zeros(cout, device=DEV)
        if kind == "x3":
            chk(lib().ifd_tr_conv_wgrad_x3(P(dy), cout, P(x), cin, None, 0, N, H, taps, P(dw), P(db), P(part), need,
                                           P(colpart), colpart.numel(), P(guard), 3, s))
        else:
            chk(lib().ifd_tr_conv_wgrad(P(dy), cout, P(x), cin, None, 0, N, H, taps, P(dw), P(db), P(part), need,
                                        P(colpart), colpart.numel(), s))
        out[kind] = (dw.view(cout, cin, taps), db)
    torch.cuda.synchronize()
    assert int(guard.max()) == 0
    rw, rb = _ref(dy, x, taps)
    rel = {k: float((v[0].double() - rw).norm() / rw.norm()) for k, v in out.items()}
    relb = float((out["x3"][1].double() - rb).norm() / rb.norm())
    record(f"wgrad_x3/{N}x{H}x{cin}->{cout}/t{taps}", rel_x3=rel["x3"], rel_fp32=rel["fp32"], rel_bias=relb)
    assert rel["x3"] <= 2e-6 and rel["x3"] <= 2 * rel["fp32"] + 1e-7, rel
    assert relb <= 1e-6, relb


@pytest.mark.parametrize("N,H,c0,c1,cout", [(2, 64, 256, 128, 128), (3, 32, 128, 128, 128), (1, 128, 256, 0, 128),
                                             (2, 16, 512, 0, 1536), (4, 16, 256, 256, 256)])
def test_wgrad_wide_1x1_vs_fp64(N, H, c0, c1, cout, record):
    """The wide-tile 1x1 weight gradient (wgrad1x1_wide_kernel: 128 x 128 channel tiles; the skip connections, the
    qkv 512 -> 1536 and proj_out) on a concat input x = cat(x0[c0], x1[c1]) (or one tensor), with the bias gradient's
    column sums fused (the trainer's column-sum workspace): rel-L2 vs float64 as test_wgrad_x3_vs_fp64."""
    from ifd import _lib
    from ifd.train import P, chk, lib

    s = _lib.stream_ptr(DEV)
    cin = c0 + c1
    g = torch.Generator().manual_seed(N * 100 + H + c0 + cout)
    x0 = (torch.randn(N, H, H, c0, generator=g) * 0.8 + 0.2).to(DEV)
    x1 = (torch.randn(N, H, H, c1, generator=g) * 0.5 - 0.1).to(DEV) if c1 else None
    dy = torch.randn(N, H, H, cout, generator=g).to(DEV)
    P_ = N * H * H
    S = ctypes.c_int()
    need = lib().ifd_tr_wgrad_part_floats(cout, cin, 1, P_, ctypes.byref(S))
    part = torch.empty(need, device=DEV)
    colpart = torch.empty(max((P_ + 1023) // 1024, S.value) * cout, device=DEV)
    guard = torch.zeros(4, device=DEV, dtype=torch.int32)
    dw, db = torch.zeros(cout * cin, device=DEV), torch.zeros(cout, device=DEV)
    chk(lib().ifd_tr_conv_wgrad_x3(P(dy), cout, P(x0), c0, P(x1), c1, N, H, 1, P(dw), P(db), P(part), need,
                                   P(colpart), colpart.numel(), P(guard), 3, s))
    torch.cuda.synchronize()
    assert int(guard.max()) == 0
    x = torch.cat([x0, x1], -1) if c1 else x0
    rw, rb = _ref(dy, x, 1)
    rel = float((dw.view(cout, cin, 1).double() - rw).norm() / rw.norm())
    relb = float((db.double() - rb).norm() / rb.norm())
    record(f"wgrad_wide/{N}x{H}x{c0}+{c1}->{cout}", rel_x3=rel, rel_bias=relb)
    assert rel <= 2e-6, rel
    assert relb <= 1e-6, relb
