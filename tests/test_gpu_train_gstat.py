"""GroupNorm statistics from the split conv's granules (ifd_tr_conv_x3_gstat + ifd_tr_gn_fwd_gstat,
csrc/train_ops.hip) vs the statistics pass over the same conv output (ifd_tr_gn_fwd): single-image
256-pixel tiles, a split-K map, a conv with a residual, and a concat of two conv outputs (the output
blocks' cat(h, skip), code/unet.py:170) whose granules come from both sources.

Both paths read the same fp32 tensor; they differ only in summation order (granule merges in fp32 then
fp64 vs fp64 sums), so mean within 1e-6 x (|mean| + std), rstd within 1e-5 relative, the normalised
output within 1e-5 x max|out|.
"""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")

CASES = [  # N, H, cin, cout, residual
    (2, 32, 128, 128, False),
    (2, 16, 256, 256, True),
    (4, 8, 256, 512, False),
    (2, 64, 64, 128, True),
]


def _conv(N, H, cin, cout, res, seed):
    from ifd import _lib
    from ifd.train import P, chk, lib

    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(N, H, H, cin, generator=g) + 0.5).to(DEV)
    w = (torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)).to(DEV)
    b = (0.3 * torch.randn(cout, generator=g)).to(DEV)
    r = (torch.randn(N, H, H, cout, generator=g) * 2 + 1).to(DEV) if res else None
    s = _lib.stream_ptr(DEV)
    guard = torch.zeros(4, device=DEV, dtype=torch.int32)
    wx3 = torch.empty(cout * cin * 9, device=DEV)
    chk(lib().ifd_tr_pack_conv_x3(P(w), cout, cin, 9, cin, cout, 0, P(wx3), P(guard), s))
    pf = lib().ifd_tr_conv_x3_part_floats(N, H, cin, cout)
    part = torch.empty(max(pf, 1), device=DEV)
    gf = lib().ifd_tr_gstat_floats(N, H, cout)
    gstat = torch.empty(gf, device=DEV)
    out = torch.empty(N, H, H, cout, device=DEV)
    E, cnt = ctypes.c_int(0), ctypes.c_float(0.0)
    chk(lib().ifd_tr_conv_x3_gstat(P(x), cin, None, 0, N, H, P(wx3), P(b), cin, cout, P(r), P(out), P(part), pf,
                                   P(guard), 9, P(gstat), gf, ctypes.byref(E), ctypes.byref(cnt), 3, s))
    return out, gstat, E.value, cnt.value


def _gn(x, N, HW, C, src):
    """(out, stats) by the statistics pass (src None) or from granule sources [(gstat, C0), gstat1, E, cnt]."""
    from ifd import _lib
    from ifd.train import P, chk, lib

    s = _lib.stream_ptr(DEV)
    g = torch.Generator().manual_seed(C)
    gamma = (1 + 0.1 * torch.randn(C, generator=g)).to(DEV)
    beta = (0.1 * torch.randn(C, generator=g)).to(DEV)
    out = torch.empty(N, HW, C, device=DEV)
    stats = torch.empty(N * 64, device=DEV)
    if src is None:
        nsl = lib().ifd_tr_gn_slices(HW, N, C)
        work = torch.empty(N * nsl * 64, device=DEV, dtype=torch.float64)
        chk(lib().ifd_tr_gn_fwd(P(x), N, HW, C, P(gamma), P(beta), None, 0, 1, P(out), P(stats), P(work), work.numel(),
                                s))
    else:
        g0, c0, g1, E, cnt = src
        chk(lib().ifd_tr_gn_fwd_gstat(P(x), N, HW, C, P(gamma), P(beta), None, 0, 1, P(g0), c0, P(g1), E, cnt, P(out),
                                      P(stats), s))
    return out, stats.view(N, 32, 2)


def _check(x, N, HW, C, src):
    o_ref, st_ref = _gn(x, N, HW, C, None)
    o, st = _gn(x, N, HW, C, src)
    torch.cuda.synchronize()
    scale = st_ref[..., 0].abs() + 1 / st_ref[..., 1]
    assert ((st[..., 0] - st_ref[..., 0]).abs() <= 1e-6 * scale).all(), "mean"
    assert ((st[..., 1] - st_ref[..., 1]).abs() <= 1e-5 * st_ref[..., 1]).all(), "rstd"
    assert (o - o_ref).abs().max().item() <= 1e-5 * o_ref.abs().max().item(), "out"


@pytest.mark.parametrize("N,H,cin,cout,res", CASES)
def test_conv_granule_stats(N, H, cin, cout, res):
    out, gstat, E, cnt = _conv(N, H, cin, cout, res, seed=H * 100 + cout)
    if E == 0:
        pytest.skip("this geometry writes no granules (multi-image tiles): the trainer runs ifd_tr_gn_fwd")
    assert E * cnt == 4 * H * H
    _check(out, N, H * H, cout, (gstat, cout, None, E, cnt))


def test_concat_granule_stats():
    N, H = 2, 32
    a, ga, Ea, ca = _conv(N, H, 128, 256, False, seed=1)
    b, gb, Eb, cb = _conv(N, H, 128, 128, True, seed=2)
    assert Ea > 0 and (Ea, ca) == (Eb, cb)
    cat = torch.cat([a, b], dim=-1).contiguous()  # 384 channels: groups of 12 straddle the two sources
    _check(cat, N, H * H, 384, (ga, 256, gb, Ea, ca))
