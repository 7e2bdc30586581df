"""Bisect helper (round 5 session r): ifd_tr_conv_x3_gn at 8x8, cin = cout = C, with a residual, against the fp32
conv of the materialised activation. usage: repro2.py N C"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "face-inpainting-diffusion-models_amd"))
import ctypes
import torch
from ifd import _lib
from ifd.train import P, chk, lib

N, C = int(sys.argv[1]), int(sys.argv[2])
H = 8
DEV = torch.device("cuda:0")
s = _lib.stream_ptr(DEV)
g = torch.Generator().manual_seed(3)
x = (torch.randn(N, H, H, C, generator=g) + 0.3).to(DEV)
res = torch.randn(N, H, H, C, generator=g).to(DEV)
w = (torch.randn(C, C, 3, 3, generator=g) / (3 * C ** 0.5)).to(DEV)
b = (0.3 * torch.randn(C, generator=g)).to(DEV)
A = (1 + 0.1 * torch.randn(N, C, generator=g)).to(DEV)
B = (0.1 * torch.randn(N, C, generator=g)).to(DEV)
guard = torch.zeros(4, device=DEV, dtype=torch.int32)
wx3 = torch.empty(C * C * 9, device=DEV)
chk(lib().ifd_tr_pack_conv_x3(P(w), C, C, 9, C, C, 0, P(wx3), P(guard), s))
pf = lib().ifd_tr_conv_x3_part_floats(N, H, C, C)
part = torch.empty(max(pf, 1), device=DEV)
gf = lib().ifd_tr_gstat_floats(N, H, C)
gstat = torch.empty(max(gf, 1), device=DEV)
out = torch.empty(N, H, H, C, device=DEV)
E, cnt = ctypes.c_int(0), ctypes.c_float(0.0)
print(f"N={N} C={C} part_floats={pf} gstat_floats={gf}", flush=True)
chk(lib().ifd_tr_conv_x3_gn(P(x), C, None, 0, N, H, P(wx3), P(b), C, C, P(A), P(B), P(res), P(out), P(part), pf,
                            P(guard), P(gstat), gf, ctypes.byref(E), ctypes.byref(cnt), 3, s))
torch.cuda.synchronize()
a = torch.nn.functional.silu(x * A[:, None, None, :] + B[:, None, None, :])
ref = torch.nn.functional.conv2d(a.permute(0, 3, 1, 2).double(), w.double(), b.double(), padding=1).permute(0, 2, 3, 1)
ref = ref + res.double()
print("maxabs", float((out.double() - ref).abs().max()), "E", E.value, flush=True)
