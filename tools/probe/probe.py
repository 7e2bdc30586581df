"""Toolchain probe: hipcc-7.2 gfx950 code object loaded next to torch's bundled HIP runtime.

Checks (1) ctypes load after torch, (2) launch on torch's current stream, (3) the
v_mfma_f32_32x32x2_f32 A/B/C lane maps with asymmetric data.
"""
import ctypes, os, sys, subprocess
import torch
here = os.path.dirname(os.path.abspath(__file__))
so = os.path.join(here, "libprobe.so")
lib = ctypes.CDLL(so, mode=ctypes.RTLD_GLOBAL)
maps = open("/proc/self/maps").read()
print("hip libs loaded:", sorted({l.split()[-1] for l in maps.splitlines() if "amdhip64" in l}))
dev = torch.device("cuda:0")
a = torch.arange(1000, dtype=torch.float32, device=dev)
b = torch.empty_like(a)
s = torch.cuda.current_stream().cuda_stream
rc = lib.run_add(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()), 1000, ctypes.c_void_p(s))
torch.cuda.synchronize()
print("add rc", rc, "ok", torch.equal(b, a * 2 + 1))
# MFMA 32x32x2: A[i][k] from lane i + 32k ; B[k][j] from lane j + 32k
A = torch.randn(32, 2, dtype=torch.float64)
B = torch.randn(2, 32, dtype=torch.float64)
al = torch.empty(64); bl = torch.empty(64)
for l in range(64):
    al[l] = A[l & 31, l >> 5]; bl[l] = B[l >> 5, l & 31]
c = torch.empty(64 * 16, device=dev)
ad = al.to(dev); bd = bl.to(dev)
rc = lib.run_mfma(ctypes.c_void_p(ad.data_ptr()), ctypes.c_void_p(bd.data_ptr()),
                  ctypes.c_void_p(c.data_ptr()), ctypes.c_void_p(s))
torch.cuda.synchronize()
c = c.cpu().view(64, 16)
C = (A.float() @ B.float())
err = 0.0
for l in range(64):
    for r in range(16):
        row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5); col = l & 31
        err = max(err, abs(float(c[l, r]) - float(C[row, col])))
print("mfma rc", rc, "maxerr", err)
import numpy as np, os
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/mfma.npz", c=c.numpy(), A=A.numpy(), B=B.numpy())
print(torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0).multi_processor_count)
