"""Census of the training step's channel copies (UNetTrainer.copy_ch): call site, channels, pixels, bytes.
One 3xf16 step at B = 32, 256^2 on the GPU; prints one line per copy and the totals."""
import sys, os, traceback
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "face-inpainting-diffusion-models_amd"))
import torch
from bench import synth_inputs
from ifd.manifest import make_state_dict
from ifd.schedules import create_gaussian_diffusion
from ifd.topology import FULL
from ifd.train import UNetTrainer

dev = torch.device("cuda:0")
B = 32
diff = create_gaussian_diffusion(steps=1000, learn_sigma=True, noise_schedule="quadratic")
gt, mask = synth_inputs(B, FULL.image_size, seed=7, device=dev)
tr = UNetTrainer(FULL, device=dev, precision="3xf16")
tr.load_state_dict(make_state_dict(FULL, seed=1))
log = []
orig = tr.copy_ch
def spy(src, cs, soff, dst, cd, doff, nc, npix, acc):
    line = traceback.extract_stack(limit=3)[0].lineno
    log.append((line, cs, cd, nc, npix, acc, 4.0 * npix * nc * (3 if acc else 2)))
    return orig(src, cs, soff, dst, cd, doff, nc, npix, acc)
tr.copy_ch = spy
t = torch.randint(0, 1000, (B,), device=dev)
tr.train_step(diff, gt, gt * (1 - mask), mask, t)
torch.cuda.synchronize()
tot = 0
for l in log:
    print("line %4d src_c %4d dst_c %4d nc %4d npix %8d acc %d  MB %.0f" % (l[0], l[1], l[2], l[3], l[4], l[5], l[6] / 1e6))
    tot += l[6]
print("copies", len(log), "total MB", round(tot / 1e6))
