"""GroupNorm applied on load in the training step (UNetTrainer fuse_gn, csrc/train_ops.hip):
ifd_tr_gn_coef's coefficients, the forward conv's prologue (ifd_tr_conv_x3_gn / ifd_tr_conv_gn) and the
split weight gradient's staging (ifd_tr_conv_wgrad_x3_gn) against the same ops on the materialised
activation silu(A x + B) (ifd_tr_act_apply), and the whole 3xf16 step fused vs unfused.

The fused and materialised paths compute the same activation per value (fma, then SiLU through exp2 and
rcp); the kernels may round exp / rcp at different points, so the gates are stated as tolerances:
  * stats: bit-identical to ifd_tr_gn_fwd's (same reduction kernels);
  * act_apply vs gn_fwd's output:          |d| <= 1e-5 max|out| (A/B form vs (x - mean) rstd gamma + beta);
  * conv / wgrad fused vs materialised:    rel-L2 <= 1e-6, max |d| <= 1e-5 max|ref|;
  * full 256^2 step, B = 4, fused vs not:  loss relative 1e-6, every parameter gradient rel-L2 <= 1e-5.
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _coef(x, N, HW, C, ss=None, seed=0):
    from ifd import _lib
    from ifd.train import P, chk, lib

    s = _lib.stream_ptr(DEV)
    g = torch.Generator().manual_seed(seed)
    gamma = (1 + 0.1 * torch.randn(C, generator=g)).to(DEV)
    beta = (0.1 * torch.randn(C, generator=g)).to(DEV)
    nsl = lib().ifd_tr_gn_slices(HW, N, C)
    work = torch.empty(N * nsl * 64, device=DEV, dtype=torch.float64)
    A, B = torch.empty(N, C, device=DEV), torch.empty(N, C, device=DEV)
    st = torch.empty(N * 64, device=DEV)
    chk(lib().ifd_tr_gn_coef(P(x), N, HW, C, P(gamma), P(beta), P(ss), 2 * C if ss is not None else 0, None, 0, None,
                             0, 0.0, P(st), P(A), P(B), P(work), work.numel(), s))
    out = torch.empty(N, HW, C, device=DEV)
    st2 = torch.empty(N * 64, device=DEV)
    chk(lib().ifd_tr_gn_fwd(P(x), N, HW, C, P(gamma), P(beta), P(ss), 2 * C if ss is not None else 0, 1, P(out),
                            P(st2), P(work), work.numel(), s))
    return A, B, st, out, st2


def _apply(x, N, HW, C, A, B):
    from ifd import _lib
    from ifd.train import P, chk, lib

    out = torch.empty(N, HW, C, device=DEV)
    chk(lib().ifd_tr_act_apply(P(x), N, HW, C, P(A), P(B), 1, P(out), _lib.stream_ptr(DEV)))
    return out


def _close(a, b, rel=1e-6, mx=1e-5):
    a, b = a.double(), b.double()
    r = float((a - b).norm() / b.norm())
    m = float((a - b).abs().max() / b.abs().max())
    assert r <= rel and m <= mx, (r, m)
    return r, m


@pytest.mark.parametrize("N,H,C,with_ss", [(2, 32, 128, False), (2, 16, 256, True), (3, 8, 64, True)])
def test_gn_coef_matches_gn_fwd(N, H, C, with_ss):
    g = torch.Generator().manual_seed(N * H + C)
    x = (torch.randn(N, H, H, C, generator=g) * 1.7 + 0.4).to(DEV)
    ss = (0.2 * torch.randn(N, 2 * C, generator=g)).to(DEV) if with_ss else None
    A, B, st, out, st2 = _coef(x, N, H * H, C, ss, seed=C)
    a = _apply(x, N, H * H, C, A, B)
    torch.cuda.synchronize()
    assert torch.equal(st, st2)
    assert float((a - out).abs().max()) <= 1e-5 * float(out.abs().max())


@pytest.mark.parametrize("N,H,cin,cout", [(2, 32, 128, 128), (2, 16, 256, 128), (4, 8, 128, 256)])
def test_conv_x3_gn_matches_materialised(N, H, cin, cout, record):
    from ifd import _lib
    from ifd.train import P, chk, lib

    s = _lib.stream_ptr(DEV)
    g = torch.Generator().manual_seed(7 + H)
    x = (torch.randn(N, H, H, cin, generator=g) + 0.3).to(DEV)
    w = (torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)).to(DEV)
    b = (0.3 * torch.randn(cout, generator=g)).to(DEV)
    A, B, _, _, _ = _coef(x, N, H * H, cin, seed=3)
    a = _apply(x, N, H * H, cin, A, B)
    guard = torch.zeros(4, device=DEV, dtype=torch.int32)
    wx3 = torch.empty(cout * cin * 9, device=DEV)
    chk(lib().ifd_tr_pack_conv_x3(P(w), cout, cin, 9, cin, cout, 0, P(wx3), P(guard), s))
    pf = lib().ifd_tr_conv_x3_part_floats(N, H, cin, cout)
    part = torch.empty(max(pf, 1), device=DEV)
    ref = torch.empty(N, H, H, cout, device=DEV)
    out = torch.empty_like(ref)
    chk(lib().ifd_tr_conv_x3_taps(P(a), cin, None, 0, N, H, P(wx3), P(b), cin, cout, None, P(ref), P(part), pf,
                                  P(guard), 9, 3, s))
    E, cnt = ctypes.c_int(0), ctypes.c_float(0.0)
    rc = lib().ifd_tr_conv_x3_gn(P(x), cin, None, 0, N, H, P(wx3), P(b), cin, cout, P(A), P(B), None, P(out), P(part),
                                 pf, P(guard), None, 0, ctypes.byref(E), ctypes.byref(cnt), 3, s)
    chk(rc)
    torch.cuda.synchronize()
    assert int(guard.max()) == 0
    r, m = _close(out, ref)
    record(f"train_fuse/conv_x3_gn/{N}x{H}x{cin}->{cout}", rel_l2=r, max_rel=m)


@pytest.mark.parametrize("N,H,cin,cout", [(2, 32, 128, 128), (2, 64, 64, 128), (8, 8, 256, 256), (2, 16, 128, 8)])
def test_wgrad_x3_gn_matches_materialised(N, H, cin, cout, record):
    from ifd import _lib
    from ifd.train import P, chk, lib

    s = _lib.stream_ptr(DEV)
    g = torch.Generator().manual_seed(11 + H + cout)
    x = (torch.randn(N, H, H, cin, generator=g) + 0.3).to(DEV)
    dy = torch.randn(N, H, H, cout, generator=g).to(DEV)
    A, B, _, _, _ = _coef(x, N, H * H, cin, seed=5)
    a = _apply(x, N, H * H, cin, A, B)
    P_ = N * H * H
    S = ctypes.c_int()
    need = lib().ifd_tr_wgrad_part_floats(cout, cin, 9, P_, ctypes.byref(S))
    part = torch.empty(need, device=DEV)
    colpart = torch.empty(((P_ + 1023) // 1024) * cout, device=DEV)
    guard = torch.zeros(4, device=DEV, dtype=torch.int32)
    dw0, db0 = torch.zeros(cout * cin * 9, device=DEV), torch.zeros(cout, device=DEV)
    dw1, db1 = torch.zeros_like(dw0), torch.zeros_like(db0)
    chk(lib().ifd_tr_conv_wgrad_x3(P(dy), cout, P(a), cin, None, 0, N, H, 9, P(dw0), P(db0), P(part), need,
                                   P(colpart), colpart.numel(), P(guard), 3, s))
    chk(lib().ifd_tr_conv_wgrad_x3_gn(P(dy), cout, P(x), cin, None, 0, N, H, P(A), P(B), P(dw1), P(db1), P(part),
                                      need, P(colpart), colpart.numel(), P(guard), 3, s))
    torch.cuda.synchronize()
    assert int(guard.max()) == 0
    assert torch.equal(db0, db1)
    r, m = _close(dw1, dw0)
    record(f"train_fuse/wgrad_x3_gn/{N}x{H}x{cin}->{cout}", rel_l2=r, max_rel=m)


def test_train_fuse_gn_step_matches_unfused(record):
    """Full config, B = 4: the 3xf16 step with the GroupNorm applied on load vs materialised."""
    from test_gpu_train import _full_step
    res = {}
    for fuse in (False, True):
        tr, loss = _full_step("3xf16", fuse_gn=fuse)
        assert tr.guard_trips == 0
        res[fuse] = (loss, tr.grad.clone(), tr.offsets)
        del tr
    (l0, g0, offs), (l1, g1, _) = res[False], res[True]
    worst, wname = 0.0, None
    for k, (o, shape) in offs.items():
        n = int(np.prod(shape))
        b = g0[o:o + n].double()
        if float(b.norm()) > 0:
            r = float((g1[o:o + n].double() - b).norm() / b.norm())
            if r > worst:
                worst, wname = r, k
    record("train_fuse/step_fused_vs_unfused", rel_loss=abs(l1 - l0) / abs(l0), max_tensor_grad_rel=worst,
           worst_tensor=wname)
    assert abs(l1 - l0) <= 1e-6 * abs(l0)
    assert worst <= 1e-5, (worst, wname)


def test_train_fuse_gnb_step_matches_unfused(record):
    """Full config, B = 4: the 3xf16 step with the GroupNorm backward's pass 1 in the dgrad conv's epilogue
    (fuse_gnb, ifd_tr_conv_x3_gnb + ifd_tr_gn_bwd_from_part) vs the separate partial pass. The partial sums run
    over other pixel blocks (64-pixel wave blocks vs 256-pixel slices), so the gate is a tolerance: loss equal
    (the forward is the same), every parameter gradient rel-L2 <= 1e-5."""
    from test_gpu_train import _full_step
    res = {}
    for fuse in (False, True):
        tr, loss = _full_step("3xf16", fuse_gnb=fuse)
        assert tr.guard_trips == 0
        res[fuse] = (loss, tr.grad.clone(), tr.offsets)
        del tr
    (l0, g0, offs), (l1, g1, _) = res[False], res[True]
    worst, wname = 0.0, None
    for k, (o, shape) in offs.items():
        n = int(np.prod(shape))
        b = g0[o:o + n].double()
        if float(b.norm()) > 0:
            r = float((g1[o:o + n].double() - b).norm() / b.norm())
            if r > worst:
                worst, wname = r, k
    record("train_fuse/step_gnb_vs_separate", rel_loss=abs(l1 - l0) / abs(l0), max_tensor_grad_rel=worst,
           worst_tensor=wname)
    assert l1 == l0
    assert worst <= 1e-5, (worst, wname)


def test_conv_x3_gnb_partials_match_separate_pass(record):
    """ifd_tr_conv_x3_gnb's partial sums, reduced, against ifd_tr_gn_bwd_cat's (same dgrad output, same x): the
    whole GroupNorm backward from the fused partials equals the separate pass's to rel-L2 1e-6 (dx, dgamma,
    dbeta, dscale/shift), for a single source with scale/shift and for a two-source concat input."""
    from ifd import _lib
    from ifd.train import P, chk, lib

    s = _lib.stream_ptr(DEV)
    # (shapes with >= 256 units, so the geometry takes no split-K: the fused path)
    for (N, H, cdy, C, C0, use_ss) in ((8, 64, 128, 128, 128, True), (16, 32, 128, 256, 128, False)):
        g = torch.Generator().manual_seed(N * H + C)
        dy = torch.randn(N, H, H, cdy, generator=g).to(DEV)
        w = (torch.randn(cdy, C, 3, 3, generator=g) / (3 * C ** 0.5)).to(DEV)  # forward conv C -> cdy; dgrad cdy -> C
        x = (torch.randn(N, H, H, C, generator=g) + 0.2).to(DEV)
        x0, x1 = x[..., :C0].contiguous(), (x[..., C0:].contiguous() if C0 < C else None)
        gam = (1 + 0.1 * torch.randn(C, generator=g)).to(DEV)
        bet = (0.1 * torch.randn(C, generator=g)).to(DEV)
        ss = (0.1 * torch.randn(N, 2 * C, generator=g)).to(DEV) if use_ss else None
        st = torch.empty(N * 64, device=DEV)
        nsl0 = lib().ifd_tr_gn_slices(H * H, N, C)
        work = torch.empty(N * nsl0 * 64, device=DEV, dtype=torch.float64)
        out = torch.empty(N, H * H, C, device=DEV)
        chk(lib().ifd_tr_gn_fwd(P(x), N, H * H, C, P(gam), P(bet), P(ss), 2 * C if use_ss else 0, 1, P(out), P(st),
                                P(work), work.numel(), s))
        wx3 = torch.empty(C * cdy * 9, device=DEV)
        guard = torch.zeros(4, device=DEV, dtype=torch.int32)
        chk(lib().ifd_tr_pack_conv_x3(P(w), cdy, C, 9, cdy, C, 1, P(wx3), P(guard), s))
        zb = torch.zeros(4096, device=DEV)
        pf = lib().ifd_tr_conv_x3_part_floats(N, H, cdy, C)
        part = torch.empty(max(pf, 1), device=DEV)
        da = torch.empty(N, H, H, C, device=DEV)
        gpf = lib().ifd_tr_gnb_part_floats(N, H, C)
        gpart = torch.empty(gpf, device=DEV)
        nsl = ctypes.c_int(0)
        chk(lib().ifd_tr_conv_x3_gnb(P(dy), cdy, N, H, P(wx3), P(zb), cdy, C, P(da), P(part), pf, P(guard), P(x0), C0,
                                     P(x1), P(st), P(gam), P(bet), P(ss), 2 * C if use_ss else 0, 1, P(gpart), gpf,
                                     ctypes.byref(nsl), 3, s))
        assert nsl.value == (H * H // 256) * 4, nsl.value
        outs = {}
        for fused in (False, True):
            dx = torch.empty(N, H, H, C, device=DEV)
            dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
            dss = torch.zeros(N, 2 * C, device=DEV) if use_ss else None
            if fused:
                wk = torch.empty(N * C * 3 + N * 64, device=DEV)
                chk(lib().ifd_tr_gn_bwd_from_part(P(da), P(x0), C0, P(x1), N, H * H, C, P(gam), P(bet), P(ss),
                                                  2 * C if use_ss else 0, 1, P(st), P(gpart), nsl.value, P(dx), 0, P(dg),
                                                  P(db), P(dss), P(wk), wk.numel(), None, 0, None, s))
            else:
                wk = torch.empty(N * nsl0 * C * 3 + N * C * 3 + N * 64, device=DEV)
                chk(lib().ifd_tr_gn_bwd_cat(P(da), P(x0), C0, P(x1), N, H * H, C, P(gam), P(bet), P(ss),
                                            2 * C if use_ss else 0, 1, P(st), P(dx), 0, P(dg), P(db), P(dss), P(wk),
                                            wk.numel(), None, 0, None, s))
            torch.cuda.synchronize()
            outs[fused] = (dx, dg, db, dss)
        assert int(guard.max()) == 0
        for name, a, b in zip(("dx", "dgamma", "dbeta", "dss"), outs[True], outs[False]):
            if b is None:
                continue
            r = float((a.double() - b.double()).norm() / b.double().norm())
            record(f"train_fuse/gnb/{N}x{H}x{cdy}->{C}(C0={C0})/{name}", rel_l2=r)
            assert r <= 1e-6, (name, r)


@pytest.mark.parametrize("N,H,cin", [(2, 32, 128), (3, 16, 64)])
def test_head_x3_matches_fp32(N, H, cin, record):
    """ifd_tr_conv_head_x3 (the split head kernel, NHWC 8 channels) vs the fp32 conv kernel with the same
    GroupNorm + SiLU prologue (ifd_tr_conv_gn): rel-L2 <= 1e-6, padded channels exactly zero."""
    from ifd import _lib
    from ifd.train import P, chk, lib

    s = _lib.stream_ptr(DEV)
    g = torch.Generator().manual_seed(N + H + cin)
    x = (torch.randn(N, H, H, cin, generator=g) + 0.3).to(DEV)
    w = (torch.randn(6, cin, 3, 3, generator=g) / (3 * cin ** 0.5)).to(DEV)
    b = (0.1 * torch.randn(6, generator=g)).to(DEV)
    A, B, _, _, _ = _coef(x, N, H * H, cin, seed=9)
    b8 = torch.zeros(8, device=DEV)
    b8[:6] = b
    guard = torch.zeros(4, device=DEV, dtype=torch.int32)
    wp = torch.empty(lib().ifd_tr_head_x3_pack_floats(cin), device=DEV)
    out = torch.full((N, H, H, 8), float("nan"), device=DEV)
    chk(lib().ifd_tr_conv_head_x3(P(x), cin, N, H, P(w), 6, P(wp), P(b8), P(A), P(B), P(out), P(guard), s))
    # the fp32 reference: weights packed for the fp32 kernel (cout padded to 8, bn 32)
    wpk = torch.empty(32 * cin * 9, device=DEV)
    chk(lib().ifd_tr_pack_conv(P(w), 6, cin, 9, 32, cin, 32, 0, P(wpk), s))
    ref = torch.empty(N, H, H, 8, device=DEV)
    pf = lib().ifd_tr_conv_part_floats(N, H, cin, 8, 32, 32, 9)
    part = torch.empty(max(pf, 1), device=DEV)
    chk(lib().ifd_tr_conv_gn(P(x), cin, None, 0, N, H, P(wpk), P(b8), cin, 8, 32, 32, 9, P(A), P(B), None, P(ref),
                             P(part), pf, s))
    torch.cuda.synchronize()
    assert int(guard.max()) == 0
    assert float(out[..., 6:].abs().max()) == 0.0
    r, m = _close(out[..., :6], ref[..., :6])
    record(f"train_fuse/head_x3/{N}x{H}x{cin}", rel_l2=r, max_rel=m)


@pytest.mark.parametrize("N,H,c0,c1,cout", [(2, 32, 128, 128, 128), (2, 16, 256, 64, 256)])
def test_concat_sources_match_materialised(N, H, c0, c1, cout, record):
    """The output blocks' concat read by channel range (UNetTrainer: the skip concat is never written):
    the GroupNorm backward (ifd_tr_gn_bwd_cat), the 3x3 weight gradient with the GroupNorm prologue and the
    1x1 weight gradient on two sources vs the same ops on the materialised concat: bit-identical."""
    from ifd import _lib
    from ifd.train import P, chk, lib

    s = _lib.stream_ptr(DEV)
    C = c0 + c1
    g = torch.Generator().manual_seed(N + H + c0 + c1)
    xa = (torch.randn(N, H, H, c0, generator=g) + 0.2).to(DEV)
    xb = (torch.randn(N, H, H, c1, generator=g) - 0.1).to(DEV)
    cat = torch.cat([xa, xb], dim=-1).contiguous()
    dy = torch.randn(N, H, H, cout, generator=g).to(DEV)
    A, B, st, _, _ = _coef(cat, N, H * H, C, seed=2)
    guard = torch.zeros(4, device=DEV, dtype=torch.int32)
    P_ = N * H * H
    res = {}
    for taps in (9, 1):
        S = ctypes.c_int()
        need = lib().ifd_tr_wgrad_part_floats(cout, C, taps, P_, ctypes.byref(S))
        part = torch.empty(need, device=DEV)
        colpart = torch.empty(((P_ + 1023) // 1024) * cout, device=DEV)
        outs = []
        for two in (False, True):
            dw, db = torch.zeros(cout * C * taps, device=DEV), torch.zeros(cout, device=DEV)
            x0, cc0, x1, cc1 = (xa, c0, xb, c1) if two else (cat, C, None, 0)
            if taps == 9:
                chk(lib().ifd_tr_conv_wgrad_x3_gn(P(dy), cout, P(x0), cc0, P(x1), cc1, N, H, P(A), P(B), P(dw), P(db),
                                                  P(part), need, P(colpart), colpart.numel(), P(guard), 3, s))
            else:
                chk(lib().ifd_tr_conv_wgrad_x3(P(dy), cout, P(x0), cc0, P(x1), cc1, N, H, 1, P(dw), P(db), P(part),
                                               need, P(colpart), colpart.numel(), P(guard), 3, s))
            outs.append((dw, db))
        res[taps] = outs
    gamma = (1 + 0.1 * torch.randn(C, generator=g)).to(DEV)
    beta = (0.1 * torch.randn(C, generator=g)).to(DEV)
    da = torch.randn(N, H, H, C, generator=g).to(DEV)
    nsl = lib().ifd_tr_gn_slices(H * H, N, C)
    gx = []
    for two in (False, True):
        dx = torch.empty(N, H, H, C, device=DEV)
        dgam, dbet = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        work = torch.empty(N * nsl * C * 3 + N * C * 3 + N * 64, device=DEV)
        x0, cc0, x1 = (xa, c0, xb) if two else (cat, C, None)
        chk(lib().ifd_tr_gn_bwd_cat(P(da), P(x0), cc0, P(x1), N, H * H, C, P(gamma), P(beta), None, 0, 1, P(st), P(dx),
                                    0, P(dgam), P(dbet), None, P(work), work.numel(), None, 0, None, s))
        gx.append((dx, dgam, dbet))
    torch.cuda.synchronize()
    assert int(guard.max()) == 0
    for taps in (9, 1):
        assert torch.equal(res[taps][0][0], res[taps][1][0]) and torch.equal(res[taps][0][1], res[taps][1][1]), taps
    for a, b in zip(gx[0], gx[1]):
        assert torch.equal(a, b)
    record(f"train_fuse/concat_sources/{N}x{H}x{c0}+{c1}->{cout}", bit_identical=True)


@pytest.mark.parametrize("N,H,C,stride,off", [(2, 16, 128, 256, 128), (3, 8, 64, 192, 64)])
def test_gn_bwd_addend(N, H, C, stride, off):
    """ifd_tr_gn_bwd_cat's dx addend (the output blocks' skip gradient joining the encoder chain's): dx with the
    addend equals dx without it plus that channel range of the wider tensor, to the rounding of one add (the
    kernel may fuse the last product and the add into one fma)."""
    from ifd import _lib
    from ifd.train import P, chk, lib

    s = _lib.stream_ptr(DEV)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(N, H * H, C, generator=g).to(DEV)
    dout = torch.randn(N, H * H, C, generator=g).to(DEV)
    wide = torch.randn(N, H * H, stride, generator=g).to(DEV)
    gam = (1 + 0.1 * torch.randn(C, generator=g)).to(DEV)
    bet = (0.1 * torch.randn(C, generator=g)).to(DEV)
    st = torch.empty(N * 64, device=DEV)
    nsl = lib().ifd_tr_gn_slices(H * H, N, C)
    wk = torch.empty(N * nsl * 64, device=DEV, dtype=torch.float64)
    chk(lib().ifd_tr_gn_fwd(P(x), N, H * H, C, P(gam), P(bet), None, 0, 1, P(torch.empty_like(x)), P(st), P(wk),
                            wk.numel(), s))
    outs = []
    for add in (False, True):
        dx = torch.empty(N, H * H, C, device=DEV)
        dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        work = torch.empty(N * nsl * C * 3 + N * C * 3 + N * 64, device=DEV)
        ap = ctypes.c_void_p(wide.data_ptr() + 4 * off) if add else None
        chk(lib().ifd_tr_gn_bwd_cat(P(dout), P(x), C, None, N, H * H, C, P(gam), P(bet), None, 0, 1, P(st), P(dx), 0,
                                    P(dg), P(db), None, P(work), work.numel(), ap, stride if add else 0, None, s))
        outs.append((dx, dg, db))
    torch.cuda.synchronize()
    ref = outs[0][0] + wide[..., off:off + C]
    err = (outs[1][0] - ref).abs()
    assert float(err.max()) <= 2.0 ** -22 * float(ref.abs().max()), float(err.max())
    assert torch.equal(outs[1][1], outs[0][1]) and torch.equal(outs[1][2], outs[0][2])


@pytest.mark.parametrize("N,H,C0,C1", [(2, 16, 128, 128), (3, 8, 192, 64)])
def test_gn_bwd_split_output(N, H, C0, C1):
    """ifd_tr_gn_bwd_cat's split output (the output blocks' concat gradient per source, no channel copy out of the
    C-wide gradient): with the skip conv's gradient as the addend, dx [.., C0] and dx1 [.., C1] equal the two channel
    ranges of the C-wide dx bit for bit (same arithmetic, other addresses), and the parameter gradients are equal."""
    from ifd import _lib
    from ifd.train import P, chk, lib

    s = _lib.stream_ptr(DEV)
    C = C0 + C1
    g = torch.Generator().manual_seed(9)
    xa = torch.randn(N, H * H, C0, generator=g).to(DEV)
    xb = torch.randn(N, H * H, C1, generator=g).to(DEV)
    dout = torch.randn(N, H * H, C, generator=g).to(DEV)
    wide = torch.randn(N, H * H, C, generator=g).to(DEV)
    gam = (1 + 0.1 * torch.randn(C, generator=g)).to(DEV)
    bet = (0.1 * torch.randn(C, generator=g)).to(DEV)
    st = torch.empty(N * 64, device=DEV)
    nsl = lib().ifd_tr_gn_slices(H * H, N, C)
    wk = torch.empty(N * nsl * 64, device=DEV, dtype=torch.float64)
    cat = torch.cat([xa, xb], -1).contiguous()
    chk(lib().ifd_tr_gn_fwd(P(cat), N, H * H, C, P(gam), P(bet), None, 0, 1, P(torch.empty_like(cat)), P(st), P(wk),
                            wk.numel(), s))
    outs = []
    for split in (False, True):
        dx = torch.empty(N, H * H, C0 if split else C, device=DEV)
        dx1 = torch.empty(N, H * H, C1, device=DEV) if split else None
        dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        work = torch.empty(N * nsl * C * 3 + N * C * 3 + N * 64, device=DEV)
        chk(lib().ifd_tr_gn_bwd_cat(P(dout), P(xa), C0, P(xb), N, H * H, C, P(gam), P(bet), None, 0, 1, P(st), P(dx),
                                    0, P(dg), P(db), None, P(work), work.numel(), P(wide), C, P(dx1), s))
        outs.append((dx, dx1, dg, db))
    torch.cuda.synchronize()
    (w, _, dg0, db0), (d0, d1, dg1, db1) = outs
    assert torch.equal(d0, w[..., :C0]) and torch.equal(d1, w[..., C0:])
    assert torch.equal(dg0, dg1) and torch.equal(db0, db1)
    # a split output is refused with accumulate or a single-source input
    from ifd import _lib as L
    with pytest.raises(RuntimeError):
        L.check(lib().ifd_tr_gn_bwd_cat(P(dout), P(xa), C0, P(xb), N, H * H, C, P(gam), P(bet), None, 0, 1, P(st),
                                        P(d0), 1, P(dg), P(db), None, P(work), work.numel(), None, 0, P(d1), s))


@pytest.mark.parametrize("N,H,c0,c1,cout,transpose", [(2, 64, 128, 128, 128, 0), (2, 64, 128, 0, 256, 1),
                                                      (1, 64, 256, 128, 128, 0), (3, 32, 64, 0, 128, 0)])
def test_conv1x1_x3_vs_fp64(N, H, c0, c1, cout, transpose, record):
    """ifd_tr_conv1x1_x3: the training step's 1x1 convs (skip_connection forward over the output blocks' concat,
    and its dgrad through W^T) on the dedicated split 1x1 kernel with the device-side weight packing, against a
    float64 reference (transpose: the input has cout channels, the output cin = c0)."""
    from ifd import _lib
    from ifd.train import P, chk, lib

    s = _lib.stream_ptr(DEV)
    g = torch.Generator().manual_seed(N + H + c0 + cout + transpose)
    # the weight W[wcout][wcin]; transpose: the dgrad maps the conv's wcout-channel gradient (here x) to wcin = cout
    wcout, wcin = (c0 + c1, cout) if transpose else (cout, c0 + c1)
    w = (torch.randn(wcout, wcin, generator=g) / 16).to(DEV)
    x0 = torch.randn(N, H, H, c0, generator=g).to(DEV)
    x1 = torch.randn(N, H, H, c1, generator=g).to(DEV) if c1 else None
    co = wcin if transpose else wcout
    b = (0.1 * torch.randn(co, generator=g)).to(DEV)
    guard = torch.zeros(4, device=DEV, dtype=torch.int32)
    wp = torch.empty(lib().ifd_tr_conv1x1_pack_floats(wcout, wcin, transpose), device=DEV)
    out = torch.empty(N, H, H, co, device=DEV)
    chk(lib().ifd_tr_conv1x1_x3(P(x0), c0, P(x1), c1, N, H, P(w), wcout, wcin, transpose, P(b), P(out), P(wp),
                                wp.numel(), P(guard), 3, s))
    torch.cuda.synchronize()
    assert int(guard.max()) == 0
    x = torch.cat([x0, x1], -1) if c1 else x0
    wm = w.double().t() if transpose else w.double()  # [co][k]
    ref = x.double() @ wm.t() + b.double()
    err = float((out.double() - ref).abs().max())
    record(f"train_fuse/conv1x1_x3/{N}x{H}x{c0}+{c1}->{co}/t{transpose}", maxabs=err)
    assert err <= 2e-6 * float(ref.abs().max()), err


@pytest.mark.parametrize("N,H,cdy,C,C0,use_ss", [(8, 64, 128, 128, 128, True), (16, 32, 128, 256, 128, False)])
def test_conv_x3_gnb_act_output(N, H, cdy, C, C0, use_ss, record):
    """ifd_tr_conv_x3_gnb_act (round 6): the GNB dgrad's epilogue also writes the GroupNorm's forward output
    act = silu(GN(x) (1 + s) + shift) over every pixel and channel, against a float64 restatement from the same
    statistics (the epilogue's arithmetic rounds per step: max |d| <= 1e-5 max|ref|); the dgrad output and the
    partial sums equal the plain entry's bit for bit."""
    from ifd import _lib
    from ifd.train import P, chk, lib

    s = _lib.stream_ptr(DEV)
    g = torch.Generator().manual_seed(N * H + C + 1)
    dy = torch.randn(N, H, H, cdy, generator=g).to(DEV)
    w = (torch.randn(cdy, C, 3, 3, generator=g) / (3 * C ** 0.5)).to(DEV)
    x = (torch.randn(N, H, H, C, generator=g) + 0.2).to(DEV)
    x0, x1 = x[..., :C0].contiguous(), (x[..., C0:].contiguous() if C0 < C else None)
    gam = (1 + 0.1 * torch.randn(C, generator=g)).to(DEV)
    bet = (0.1 * torch.randn(C, generator=g)).to(DEV)
    ss = (0.1 * torch.randn(N, 2 * C, generator=g)).to(DEV) if use_ss else None
    st = torch.empty(N * 64, device=DEV)
    nsl0 = lib().ifd_tr_gn_slices(H * H, N, C)
    work = torch.empty(N * nsl0 * 64, device=DEV, dtype=torch.float64)
    gout = torch.empty(N, H * H, C, device=DEV)
    chk(lib().ifd_tr_gn_fwd(P(x), N, H * H, C, P(gam), P(bet), P(ss), 2 * C if use_ss else 0, 1, P(gout), P(st),
                            P(work), work.numel(), s))
    wx3 = torch.empty(C * cdy * 9, device=DEV)
    guard = torch.zeros(4, device=DEV, dtype=torch.int32)
    chk(lib().ifd_tr_pack_conv_x3(P(w), cdy, C, 9, cdy, C, 1, P(wx3), P(guard), s))
    zb = torch.zeros(4096, device=DEV)
    pf = lib().ifd_tr_conv_x3_part_floats(N, H, cdy, C)
    part = torch.empty(max(pf, 1), device=DEV)
    gpf = lib().ifd_tr_gnb_part_floats(N, H, C)
    outs = []
    for with_act in (False, True):
        da = torch.empty(N, H, H, C, device=DEV)
        gpart = torch.empty(gpf, device=DEV)
        act = torch.full((N, H, H, C), float("nan"), device=DEV) if with_act else None
        nsl = ctypes.c_int(0)
        chk(lib().ifd_tr_conv_x3_gnb_act(P(dy), cdy, N, H, P(wx3), P(zb), cdy, C, P(da), P(part), pf, P(guard), P(x0),
                                         C0, P(x1), P(st), P(gam), P(bet), P(ss), 2 * C if use_ss else 0, 1, P(gpart),
                                         gpf, ctypes.byref(nsl), P(act), 3, s))
        assert nsl.value > 0
        outs.append((da, gpart, act))
    torch.cuda.synchronize()
    (da0, gp0, _), (da1, gp1, act) = outs
    assert torch.equal(da0, da1) and torch.equal(gp0, gp1)
    stc = st.view(N, 32, 2).double().cpu()
    xd = x.double().cpu().view(N, H * H, 32, C // 32)
    xhat = (xd - stc[:, None, :, 0:1]) * stc[:, None, :, 1:2]
    z = xhat.view(N, H * H, C) * gam.double().cpu() + bet.double().cpu()
    if use_ss:
        sd = ss.double().cpu()
        z = z * (1 + sd[:, None, :C]) + sd[:, None, C:]
    ref = (z * torch.sigmoid(z)).view(N, H, H, C)
    err = float((act.double().cpu() - ref).abs().max())
    record(f"train_fuse/gnb_act/{N}x{H}x{C}", maxabs=err, ref_max=float(ref.abs().max()))
    assert torch.isfinite(act).all()
    assert err <= 1e-5 * float(ref.abs().max()), err
