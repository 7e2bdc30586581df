"""Partial four-image 8 x 8 tiles on the split kernel (conv_x3.hip unit_of) in the training ops, round 6.

A four-image tile of a batch whose size is not a multiple of 4 recomputes the batch's last image in its spare
slots by moving those slots' tile origin n0 below image 0. Round 5's status-700 fault of the training step came
from the coefficient loads of an ACT_NONE conv (every dgrad), which still read from that moved origin, i.e. 1-3
images below the tensor (the loads issue for a fixed vmcnt count whether or not the values are used). They now
read from the slot's own image. These tests run the entry points that take that path — the forward conv without a
prologue, the transposed (dgrad) conv, the GroupNorm-prologue conv, the 1x1 over two sources — at N = 1, 2, 3 on
separately allocated tensors placed at the START of their own allocation (so a read below the tensor leaves the
allocation), against float64 references, and three asynchronous reduced-config training steps at B = 2 (the
round-5 repro, profiles/r05r/repro4.sh) against the fp32 trainer.

Tolerances (written here): split conv vs float64, max-abs <= 2e-6 max|ref| (the split arithmetic's per-product
error ~2^-21 relative over K = 9 Cin terms); training step 3xf16 vs fp32: loss relative 1e-5, every parameter
gradient rel-L2 <= 1e-4 (the bounds of test_gpu_train.py::test_train_x3_full_matches_fp32).
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _fresh(shape, gen, scale=1.0, shift=0.0):
    """A tensor at offset 0 of its own 64 MiB+ allocation (the caching allocator gives such a request its own
    segment), so an address below it is outside every byte this test owns."""
    n = int(np.prod(shape))
    big = torch.empty(max(n, 16 << 20), device=DEV)
    t = big[:n].view(*shape)
    t.copy_((torch.randn(*shape, generator=gen) * scale + shift).to(DEV))
    return t


def _conv_ref(x_nhwc, w, b, transpose):
    """float64 conv3x3 (padding 1) of an NHWC tensor; transpose: the dgrad of the conv with weight w (cout, cin),
    i.e. the conv with the 180-degree rotated, in/out-transposed kernel."""
    xx = x_nhwc.double().cpu().permute(0, 3, 1, 2)
    ww = w.double().cpu()
    if transpose:
        ww = ww.flip(2, 3).transpose(0, 1)
    y = torch.nn.functional.conv2d(xx, ww, b.double().cpu(), padding=1)
    return y.permute(0, 2, 3, 1)


@pytest.mark.parametrize("N", [1, 2, 3])
@pytest.mark.parametrize("kind", ["plain", "dgrad", "gn"])
def test_conv_x3_partial_tiles_8x8(N, kind, record):
    from ifd import _lib
    from ifd.train import P, chk, lib

    s = _lib.stream_ptr(DEV)
    H, cin, cout = 8, 128, 256
    g = torch.Generator().manual_seed(100 * N + len(kind))
    transpose = kind == "dgrad"
    # forward: w (cout, cin); dgrad: the forward conv maps cout -> cin, its dgrad maps cin -> cout, so the packed
    # weight is w (cin, cout) transposed
    w = (torch.randn(*((cin, cout) if transpose else (cout, cin)), 3, 3, generator=g) / (3 * cin ** 0.5)).to(DEV)
    x = _fresh((N, H, H, cin), g, shift=0.2)
    b = (0.1 * torch.randn(cout, generator=g)).to(DEV)
    guard = torch.zeros(4, device=DEV, dtype=torch.int32)
    wx3 = torch.empty(cout * cin * 9, device=DEV)
    if transpose:
        chk(lib().ifd_tr_pack_conv_x3(P(w), cin, cout, 9, cin, cout, 1, P(wx3), P(guard), s))
    else:
        chk(lib().ifd_tr_pack_conv_x3(P(w), cout, cin, 9, cin, cout, 0, P(wx3), P(guard), s))
    pf = lib().ifd_tr_conv_x3_part_floats(N, H, cin, cout)
    part = torch.empty(max(pf, 1), device=DEV)
    out = _fresh((N, H, H, cout), g)
    if kind == "gn":
        A = (1 + 0.1 * torch.randn(N, cin, generator=g)).to(DEV)
        B = (0.1 * torch.randn(N, cin, generator=g)).to(DEV)
        E, cnt = ctypes.c_int(0), ctypes.c_float(0.0)
        chk(lib().ifd_tr_conv_x3_gn(P(x), cin, None, 0, N, H, P(wx3), P(b), cin, cout, P(A), P(B), None, P(out),
                                    P(part), pf, P(guard), None, 0, ctypes.byref(E), ctypes.byref(cnt), 3, s))
        z = A.double().cpu()[:, None, None, :] * x.double().cpu() + B.double().cpu()[:, None, None, :]
        xin = z * torch.sigmoid(z)
    else:
        chk(lib().ifd_tr_conv_x3_taps(P(x), cin, None, 0, N, H, P(wx3), P(b), cin, cout, None, P(out), P(part), pf,
                                      P(guard), 9, 3, s))
        xin = x
    torch.cuda.synchronize()
    assert int(guard.max()) == 0
    ref = _conv_ref(xin, w, b, transpose)
    err = float((out.double().cpu() - ref).abs().max())
    record(f"partial_tiles/conv_x3/{kind}/N{N}", maxabs=err, ref_max=float(ref.abs().max()))
    assert err <= 2e-6 * float(ref.abs().max()), err


@pytest.mark.parametrize("N", [1, 2, 3])
def test_conv1x1_x3_two_sources_partial_tiles_8x8(N, record):
    """The split kernel's 1x1-only launch (SKIP instantiation, operand in registers) over two sources at 8 x 8."""
    from ifd import _lib
    from ifd.train import P, chk, lib

    s = _lib.stream_ptr(DEV)
    H, c0, c1, cout = 8, 128, 64, 128
    g = torch.Generator().manual_seed(7 + N)
    w = (torch.randn(cout, c0 + c1, generator=g) / 16).to(DEV)
    x0 = _fresh((N, H, H, c0), g)
    x1 = _fresh((N, H, H, c1), g)
    b = (0.1 * torch.randn(cout, generator=g)).to(DEV)
    guard = torch.zeros(4, device=DEV, dtype=torch.int32)
    wx3 = torch.empty(cout * (c0 + c1), device=DEV)
    chk(lib().ifd_tr_pack_conv_x3(P(w), cout, c0 + c1, 1, c0 + c1, cout, 0, P(wx3), P(guard), s))
    pf = lib().ifd_tr_conv_x3_part_floats(N, H, c0 + c1, cout)
    part = torch.empty(max(pf, 1), device=DEV)
    out = _fresh((N, H, H, cout), g)
    chk(lib().ifd_tr_conv_x3_taps(P(x0), c0, P(x1), c1, N, H, P(wx3), P(b), c0 + c1, cout, None, P(out), P(part), pf,
                                  P(guard), 1, 3, s))
    torch.cuda.synchronize()
    assert int(guard.max()) == 0
    x = torch.cat([x0, x1], -1).double().cpu()
    ref = x @ w.double().cpu().t() + b.double().cpu()
    err = float((out.double().cpu() - ref).abs().max())
    record(f"partial_tiles/conv1x1_x3/N{N}", maxabs=err)
    assert err <= 2e-6 * float(ref.abs().max()), err


def _reduced_steps(precision, B, steps):
    from ifd.manifest import make_state_dict
    from ifd.schedules import create_gaussian_diffusion
    from ifd.topology import REDUCED
    from ifd.train import UNetTrainer
    tr = UNetTrainer(REDUCED, device=DEV, precision=precision)
    tr.load_state_dict(make_state_dict(REDUCED, seed=1))
    diff = create_gaussian_diffusion(steps=1000, learn_sigma=True, noise_schedule="linear")
    g = torch.Generator().manual_seed(0)
    img = torch.rand(B, 3, 64, 64, generator=g) * 2 - 1
    mask = (torch.rand(B, 1, 64, 64, generator=g) > 0.5).float()
    t = torch.randint(0, 1000, (B,), generator=g)
    torch.manual_seed(5)  # the steps' noise draws (noise_device="cpu": the global CPU generator)
    losses = []
    for _ in range(steps):  # asynchronous: no synchronisation between the steps (the round-5 repro)
        losses.append(tr.train_step(diff, img.to(DEV), (img * (1 - mask)).to(DEV), mask.to(DEV), t.to(DEV),
                                    noise_device="cpu"))
    torch.cuda.synchronize()
    return tr, [float(x) for x in losses]


def test_train_reduced_b2_three_async_steps(record):
    """profiles/r05r/repro4.sh as a test: three 3xf16 steps at B = 2 on the reduced config (its 8 x 8 dgrad convs
    on partial four-image tiles), launched without a synchronisation between them, against the fp32 trainer."""
    tr3, l3 = _reduced_steps("3xf16", 2, 3)
    assert tr3.guard_trips == 0
    tr32, l32 = _reduced_steps("fp32", 2, 3)
    rel = [abs(a - b) / abs(b) for a, b in zip(l3, l32)]
    worst, wname = 0.0, None
    for k, (o, shape) in tr32.offsets.items():
        n = int(np.prod(shape))
        a, b = tr3.grad[o:o + n].double(), tr32.grad[o:o + n].double()
        if float(b.norm()) > 0:
            r = float((a - b).norm() / b.norm())
            if r > worst:
                worst, wname = r, k
    record("partial_tiles/train_reduced_b2_3steps", losses=l3, losses_fp32=l32, rel_loss=rel,
           max_tensor_grad_rel=worst, worst_tensor=wname)
    assert max(rel) <= 1e-5, rel
    assert worst <= 1e-4, (worst, wname)


def test_launch_failure_names_its_entry():
    """Error contract: a launch that fails (an empty grid the host check lets through: ifd_tr_add with n = 0)
    reports a message naming that entry point, not a message an earlier call left behind."""
    from ifd import _lib
    from ifd.train import P, lib

    L = lib()
    s = _lib.stream_ptr(DEV)
    assert L.ifd_tr_scale(None, 4, 1.0, s) != 0  # leaves "ifd_tr_scale: bad arguments" (not checked)
    a = torch.zeros(4, device=DEV)
    rc = L.ifd_tr_add(P(a), P(a), P(a), 0, s)
    if rc == 0:
        pytest.skip("this HIP runtime accepts an empty grid")
    msg = L.ifd_last_error().decode()
    assert msg.startswith("ifd_tr_add: "), msg
    with pytest.raises(RuntimeError, match="ifd_tr_add"):
        _lib.check(rc)
    assert L.ifd_last_error() == b""
    torch.cuda.synchronize()
