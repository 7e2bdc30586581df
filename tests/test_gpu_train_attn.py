"""QKVAttention training kernels (ifd_tr_attention / ifd_tr_attention_bwd, csrc/train_ops.hip) vs float64
torch autograd of the reference's chunk-first attention (code/nn.py:222-235): per head, q, k, v are
64-channel slices at offsets (0, C, 2C) + 64 h of the qkv row, weight = softmax((q s)(k s)^T) with
s = 64^-1/4, out = weight v.

The backward's row and column kernels take 32 query / key rows per block and clamp the key index of
a partial block, so the cases include T not a multiple of 32 (40, 100) next to T = 32 and 256.
Tolerance: fp32 kernels vs the fp64 reference, max-abs within 2e-5 x max|ref|.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")

CASES = [(2, 32, 64), (1, 40, 128), (2, 100, 64), (1, 256, 256)]  # N, T, C


def _ref(qkv, C):
    N, T, _ = qkv.shape
    s = 1 / math.sqrt(math.sqrt(64))
    out = []
    for h in range(C // 64):
        q = qkv[:, :, h * 64:(h + 1) * 64]
        k = qkv[:, :, C + h * 64:C + (h + 1) * 64]
        v = qkv[:, :, 2 * C + h * 64:2 * C + (h + 1) * 64]
        w = torch.softmax(torch.einsum("ntd,nsd->nts", q * s, k * s), dim=-1)
        out.append(torch.einsum("nts,nsd->ntd", w, v))
    return torch.cat(out, dim=-1)


def _close(got, ref, name):
    ref = ref.detach().cpu()
    err = (got.detach().cpu().double() - ref).abs().max().item()
    tol = 2e-5 * ref.abs().max().item()
    assert err <= tol, f"{name}: max-abs {err:.3e} > {tol:.3e}"


@pytest.mark.parametrize("N,T,C", CASES)
def test_attention_fwd_bwd(N, T, C):
    from ifd import _lib
    from ifd.train import P, chk, lib

    g = torch.Generator().manual_seed(N * 131 + T * 7 + C)
    qkv = (1.5 * torch.randn(N, T, 3 * C, generator=g, dtype=torch.float64)).requires_grad_()
    dout = torch.randn(N, T, C, generator=g, dtype=torch.float64)
    y = _ref(qkv, C)
    (dqkv_ref,) = torch.autograd.grad(y, [qkv], dout)

    s = _lib.stream_ptr(DEV)
    scale = 1 / math.sqrt(math.sqrt(64))
    qd = qkv.detach().float().contiguous().to(DEV)
    dd = dout.float().contiguous().to(DEV)
    out = torch.empty(N, T, C, device=DEV)
    chk(lib().ifd_tr_attention(P(qd), N, T, C, scale, P(out), s))
    sf = lib().ifd_tr_attention_bwd_scratch_floats(N, T, C)
    scratch = torch.empty(sf, device=DEV)
    dqkv = torch.empty(N, T, 3 * C, device=DEV)
    chk(lib().ifd_tr_attention_bwd(P(qd), P(dd), N, T, C, scale, P(dqkv), P(scratch), sf, s))
    torch.cuda.synchronize()
    _close(out, y, "out")
    for i, nm in enumerate(("dq", "dk", "dv")):
        _close(dqkv[:, :, i * C:(i + 1) * C], dqkv_ref[:, :, i * C:(i + 1) * C], nm)
