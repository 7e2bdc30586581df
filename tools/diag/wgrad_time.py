"""Development: time one 3x3 weight gradient (256^2, B = 32, 128 -> 128) on the fp32 kernel and the 3xf16
kernel of the loaded library (IFD_LIB_PATH selects a variant build)."""
import ctypes, os, sys, time
_R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(_R, "face-inpainting-diffusion-models_amd"))
import torch
from ifd import train as T
N, H, C = 32, 256, 128
dev = torch.device("cuda:0")
dy = torch.randn(N, H, H, C, device=dev)
x = torch.randn(N, H, H, C, device=dev)
dw = torch.zeros(C * C * 9, device=dev)
db = torch.zeros(C, device=dev)
S = ctypes.c_int()
need = T.lib().ifd_tr_wgrad_part_floats(C, C, 9, N * H * H, ctypes.byref(S))
part = torch.empty(need, device=dev)
colpart = torch.empty(((N * H * H + 1023) // 1024) * C, device=dev)
guard = torch.zeros(4, device=dev, dtype=torch.int32)
s = torch.cuda.current_stream().cuda_stream
P = T.P
def run(x3):
    if x3:
        return T.lib().ifd_tr_conv_wgrad_x3(P(dy), C, P(x), C, None, 0, N, H, 9, P(dw), P(db), P(part), need, P(colpart),
                                            colpart.numel(), P(guard), 3, ctypes.c_void_p(s))
    return T.lib().ifd_tr_conv_wgrad(P(dy), C, P(x), C, None, 0, N, H, 9, P(dw), P(db), P(part), need, P(colpart),
                                     colpart.numel(), ctypes.c_void_p(s))
for x3 in (0, 1):
    for _ in range(2): T.chk(run(x3))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5): T.chk(run(x3))
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 5 * 1e3
    print(f"{os.environ.get('IFD_LIB_PATH', 'main')} x3={x3}: {ms:.3f} ms  {2 * N * H * H * C * C * 9 / ms / 1e9:.1f} TFLOP/s", flush=True)
