"""GroupNorm(32) training kernels (ifd_tr_gn_fwd / ifd_tr_gn_bwd, csrc/train_ops.hip) vs float64 torch
autograd of the reference's formula: GroupNorm32 (code/nn.py:46-48), the ResBlock's scale/shift
(code/unet.py, use_scale_shift_norm: norm(h) * (1 + scale) + shift) and SiLU.

The kernels run 256 threads as (pixel row x channel quad) over 256-pixel slices, so the cases pick
channel counts whose layout leaves idle threads (96, 192, 384), the widest one (1024), and pixel
counts that are not multiples of the slice or of the row count (17, 300, 1100). The backward also runs
in accumulate mode (dx += ...), as the trainer uses it for residual gradients.
Tolerance: fp32 kernels vs the fp64 reference, max-abs within 2e-5 x max|ref| per output.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")

CASES = [  # N, HW, C, scale/shift, SiLU, accumulate
    (2, 64, 384, True, True, False),
    (3, 300, 96, False, True, False),
    (2, 256, 1024, True, False, False),
    (1, 17, 32, False, False, False),
    (2, 1100, 192, True, True, True),
]


def _ref(x, gamma, beta, ss, silu):
    N, HW, C = x.shape
    z = F.group_norm(x.permute(0, 2, 1), 32, gamma, beta, eps=1e-5).permute(0, 2, 1)
    if ss is not None:
        z = z * (1 + ss[:, None, :C]) + ss[:, None, C:]
    return z * torch.sigmoid(z) if silu else z


def _close(got, ref, name):
    ref = ref.detach().cpu()
    err = (got.detach().cpu().double() - ref).abs().max().item()
    tol = 2e-5 * max(ref.abs().max().item(), 1e-30)
    assert err <= tol, f"{name}: max-abs {err:.3e} > {tol:.3e}"


@pytest.mark.parametrize("N,HW,C,use_ss,silu,acc", CASES)
def test_gn_fwd_bwd(N, HW, C, use_ss, silu, acc):
    from ifd import _lib
    from ifd.train import P, chk, lib

    g = torch.Generator().manual_seed(N * 7919 + HW * 31 + C)
    x = torch.randn(N, HW, C, generator=g, dtype=torch.float64) * 1.7 + 0.3
    gamma = 1 + 0.2 * torch.randn(C, generator=g, dtype=torch.float64)
    beta = 0.1 * torch.randn(C, generator=g, dtype=torch.float64)
    ss = 0.3 * torch.randn(N, 2 * C, generator=g, dtype=torch.float64) if use_ss else None
    dout = torch.randn(N, HW, C, generator=g, dtype=torch.float64)
    prev = torch.randn(N, HW, C, generator=g, dtype=torch.float64) if acc else None

    leaves = [t.requires_grad_() for t in (x, gamma, beta) + ((ss,) if use_ss else ())]
    y = _ref(x, gamma, beta, ss, silu)
    grads = torch.autograd.grad(y, leaves, dout)

    f = lambda t: None if t is None else t.detach().float().contiguous().to(DEV)  # noqa: E731
    xd, gd, bd, sd, dd = f(x), f(gamma), f(beta), f(ss), f(dout)
    s = _lib.stream_ptr(DEV)
    nsl = lib().ifd_tr_gn_slices(HW, N, C)
    out = torch.empty(N, HW, C, device=DEV)
    stats = torch.empty(N * 64, device=DEV)
    work = torch.empty(N * nsl * 64, device=DEV, dtype=torch.float64)
    chk(lib().ifd_tr_gn_fwd(P(xd), N, HW, C, P(gd), P(bd), P(sd), 2 * C, int(silu), P(out), P(stats), P(work),
                            work.numel(), s))
    dx = f(prev) if acc else torch.empty(N, HW, C, device=DEV)
    dgam = torch.zeros(C, device=DEV)
    dbet = torch.zeros(C, device=DEV)
    dss = torch.zeros(N, 2 * C, device=DEV) if use_ss else None
    wb = torch.empty(N * nsl * C * 3 + N * C * 3 + N * 64, device=DEV)
    chk(lib().ifd_tr_gn_bwd(P(dd), P(xd), N, HW, C, P(gd), P(bd), P(sd), 2 * C, int(silu), P(stats), P(dx), int(acc),
                            P(dgam), P(dbet), P(dss), P(wb), wb.numel(), s))
    torch.cuda.synchronize()

    _close(out, y, "out")
    _close(dx, grads[0] + (prev if acc else 0), "dx")
    _close(dgam, grads[1], "dgamma")
    _close(dbet, grads[2], "dbeta")
    if use_ss:
        _close(dss, grads[3], "dss")
    # the statistics the backward consumed: (mean, rstd) per (image, group)
    xs = x.detach().view(N, HW, 32, C // 32)
    mean = xs.mean(dim=(1, 3))
    var = xs.var(dim=(1, 3), unbiased=False)
    st = stats.view(N, 32, 2).cpu().double()
    np.testing.assert_allclose(st[..., 0].numpy(), mean.numpy(), rtol=0, atol=1e-6)
    np.testing.assert_allclose(st[..., 1].numpy(), (1 / torch.sqrt(var + 1e-5)).numpy(), rtol=1e-6)
