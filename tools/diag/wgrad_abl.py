"""Development: time the 3x3 split weight gradient (wgrad_ws_kernel) at the training step's dominant shape
(256^2, B = 32, 128 -> 128), with the GroupNorm prologue (GNA, ifd_tr_conv_wgrad_x3_gn) and without
(ifd_tr_conv_wgrad_x3), on the loaded library (IFD_LIB_PATH selects a WS_ABL ablation build). Prints one JSON line."""
import ctypes, json, os, sys, time
_R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(_R, "face-inpainting-diffusion-models_amd"))
import torch
from ifd import train as T
N, H, C = 32, 256, 128
dev = torch.device("cuda:0")
dy = torch.randn(N, H, H, C, device=dev)
x = torch.randn(N, H, H, C, device=dev)
A = 1 + 0.1 * torch.randn(N, C, device=dev)
B = 0.1 * torch.randn(N, C, device=dev)
dw = torch.zeros(C * C * 9, device=dev)
db = torch.zeros(C, device=dev)
S = ctypes.c_int()
need = T.lib().ifd_tr_wgrad_part_floats(C, C, 9, N * H * H, ctypes.byref(S))
part = torch.empty(need, device=dev)
colpart = torch.empty(((N * H * H + 1023) // 1024) * C, device=dev)
guard = torch.zeros(4, device=dev, dtype=torch.int32)
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
P = T.P
flops = 2.0 * N * H * H * C * C * 9


def run(gn):
    if gn:
        return T.lib().ifd_tr_conv_wgrad_x3_gn(P(dy), C, P(x), C, None, 0, N, H, P(A), P(B), P(dw), P(db), P(part), need,
                                               P(colpart), colpart.numel(), P(guard), 3, s)
    return T.lib().ifd_tr_conv_wgrad_x3(P(dy), C, P(x), C, None, 0, N, H, 9, P(dw), P(db), P(part), need, P(colpart),
                                        colpart.numel(), P(guard), 3, s)


out = {"lib": os.environ.get("IFD_LIB_PATH", "in-tree"), "splits": S.value}
for gn in (1, 0):
    for _ in range(3):
        T.chk(run(gn))
    torch.cuda.synchronize()
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        T.chk(run(gn))
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    out["gna" if gn else "plain"] = {"ms": round(ms, 4), "tflops": round(flops / ms / 1e9, 1)}
print(json.dumps(out), flush=True)
