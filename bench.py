"""Headline benchmark: 256x256 DDIM-100 inpainted images/sec on MI355X (BASELINE.json `metric`).

One "step" = one full DDIM-100 inpainting pass (101 UNet evals, each with the DDIM update and the
known-region re-injection fused into the last conv, then the final blend) over a batch of
synthetic 256x256 inputs, per GPU. Workload = BASELINE.json configs[1]: batch 16 per GPU, DDIM-100
cosine T=1000, eta 0.75 (code/test_inp_ddim_100.py:820), fp32, random-init weights of the
reference architecture (seeded manifest), gt ~ U(-1,1), 25 % centre-square + random-rectangle masks.
N GPUs = N independent shards (weak scaling), one RCCL all_gather of the outputs inside the
timed region. `--gpus N` without a torch.distributed.run environment starts N ranks itself (a
torch.distributed.run child launched before this process touches the GPU) and relays rank 0's
line. `--noise parity` draws every noise tensor for the whole global batch in the reference's order
on the rank's GPU (the reference draws on the model's device, code/test_inp_ddim_100.py:481,554,567;
every rank seeds the device generator identically, so the full-batch draw is the same on every rank)
and keeps the rank's rows (results independent of the GPU count, at the cost of
generating N x the rank's noise on-device); the default `device` mode draws per rank (per-rank seeds).

`--noise parity` also builds the model with the handle option `batch_invariant` (split-K and tile choice
per image, include/ifd.h), so a rank's images come out bit-identical whatever the shard size: with it the
line is GPU-count-independent as well as seed-consistent (`config.options` records it).
`--workload dropin` times what a user of the UNCHANGED reference script gets: the same B = 16 DDIM-100 loop
driven through `model(x, t, masked_image=, mask=)` once per step with the script's own torch algebra
(code/test_inp_ddim_100.py:470-576, restated in `script_ddim_pass`), instead of one fused library call per
step; the line carries the fused rate of the same run beside it.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--noise device|parity]
    python bench.py --workload c4 --gpus 8      # configs[3]: 512 images sharded 8 ways (64 per GPU)
    python bench.py --workload dropin           # the reference script's per-step loop over model()
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "face-inpainting-diffusion-models_amd")]

import torch  # noqa: E402

PEAK_FP32_TFLOPS = 157.3   # MI355X dense fp32 (vector = MFMA f32), /opt/skills/guides/MI355X_MICROARCH.md
PEAK_F16_TFLOPS = 2500.0   # MI355X dense f16/bf16 MFMA (no sparsity), same guide
# the 3xf16 split mode spends 3 f16 MFMA products per fp32 MAC: its ceiling in algorithmic FLOP/s
PEAK_3XF16_TFLOPS = PEAK_F16_TFLOPS / 3
PEAK_HBM_GBS = 8000.0
README_S_PER_SAMPLE_DDIM100 = 3.42   # reference README.md:76 (unstated GPU, batch 4)


def synth_inputs(B, H, seed, device):
    g = torch.Generator().manual_seed(seed)
    gt = torch.rand(B, 3, H, H, generator=g) * 2 - 1
    mask = torch.zeros(B, 1, H, H)
    q = H // 4
    mask[:, :, q:H - q, q:H - q] = 1.0
    for b in range(B):
        for _ in range(2):
            y0, x0 = [int(v) for v in torch.randint(0, H // 2, (2,), generator=g)]
            hh, ww = [int(v) for v in torch.randint(H // 16, H // 3, (2,), generator=g)]
            mask[b, :, y0:y0 + hh, x0:x0 + ww] = 1.0
    return gt.to(device), mask.to(device)


class _BudgetSpent(Exception):
    pass


def cpu_baseline(budget_s, H=256):
    """The oracle (pure-torch CPU restatement of the reference, pinned bit-exact to it by tests/golden)
    timed on this host's cores: the reference's own DDIM-100 script loop (oracle script_ddim_loop =
    code/test_inp_ddim_100.py:470-576: model_fn, UNet, DDIM update, injection) at B=1 256x256, run
    step by step until `budget_s` elapses. Per-step time = the span between the first and the last
    completed step's model call (the first step is warm-up); images/s = 1 / (101 x per-step)."""
    from ifd.manifest import make_state_dict
    from ifd.topology import FULL
    from oracle import ref_diffusion, ref_unet
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(cores)
    sd = ref_unet.strip_prefix(make_state_dict(FULL, seed=1))
    tb = ref_diffusion.Tables(ref_diffusion.get_named_beta_schedule("cosine", 1000))
    torch.manual_seed(0)
    gt, mask = synth_inputs(1, H, seed=7, device="cpu")
    stamps = []

    def unet_call(x, t, masked, m):
        stamps.append(time.time())
        if len(stamps) >= 3 and (stamps[-1] - stamps[0] > budget_s or len(stamps) > 101):
            raise _BudgetSpent
        return ref_unet.inpaint_forward(sd, x, t, masked, m, FULL)
    with torch.no_grad():
        try:
            ref_diffusion.script_ddim_loop(tb, ref_diffusion.model_fn_factory(unet_call), (1, 3, H, H), gt, mask,
                                           100, clip=True, eta=0.75)
            stamps.append(time.time())
        except _BudgetSpent:
            pass
    steps = len(stamps) - 2  # complete steps between the 2nd model call and the last stamp
    t_step = (stamps[-1] - stamps[1]) / steps
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": 1.0 / (101 * t_step), "unit": "images/s", "cores": cores, "kind": "port",
            "sample": f"{steps} timed steps (after 1 warm-up) of the oracle's DDIM-100 cosine script loop "
                      f"(oracle/ref_diffusion.script_ddim_loop + ref_unet, torch CPU fp32) at B=1 256x256, "
                      f"{t_step * 1e3:.0f} ms/step, x101 steps per image",
            "s_per_step": t_step, "cpu_model": cpu_model}


def pmc_traffic(kernel):
    """HBM bytes per launch and MFMA-busy fraction of `kernel` from the newest committed PMC summary
    (profiles/<tag>/pmc_summary.json, written by tools/gpu_round.sh: separate rocprofv3 --pmc passes over
    this same bench command, FETCH_SIZE x2 / WRITE_SIZE x1 per tools/micro/pmc_cal.hip). PMC counters
    cannot be read inside a live run without the profiler, so the live line cites that file."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_summary.json")), reverse=True):
        try:
            k = json.load(open(path))["kernels"].get(kernel)
        except (OSError, ValueError, KeyError):
            continue
        if k and k.get("hbm_bytes_per_launch"):
            return {"traffic": k["hbm_bytes_per_launch"], "mfma_busy": k.get("mfma_busy_frac"),
                    "traffic_source": os.path.relpath(path, ROOT)}
    return {"traffic": None}


def device_key(hostname, pr):
    """One GPU's identity: host, device UUID AND PCI domain:bus:device. Both, because a ROCm build may report
    a non-unique UUID (all zeros) for every device, and PCI IDs alone repeat across hosts."""
    return (hostname, str(getattr(pr, "uuid", "")),
            f"{getattr(pr, 'pci_domain_id', '?')}:{getattr(pr, 'pci_bus_id', '?')}:{getattr(pr, 'pci_device_id', '?')}")


def fp32_accuracy_note():
    """The exact-fp32 mode's per-eval error against an fp64 UNet relative to the reference's own fp32 error, from the
    newest committed GPU parity record (tests/test_gpu_full.py::test_c1_eval_error_vs_fp64 writes c1_eval0/fp32)."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "parity.json")), reverse=True):
        try:
            e = json.load(open(path)).get("c1_eval0/fp32")
        except (OSError, ValueError):
            continue
        if e and "gpu_vs_fp64" in e and "reference_vs_fp64" in e:
            g, r = e["gpu_vs_fp64"], e["reference_vs_fp64"]
            ratio = {k: round(g[k] / r[k], 2) for k in ("mean", "p999", "max")}
            return {"per_eval_error_vs_reference_own": ratio, "source": os.path.relpath(path, ROOT),
                    "note": "exact fp32 products, but one fp32 accumulation chain over K = 9 Cin (up to 4608 terms) per "
                            "output: %sx the reference's (oneDNN) per-eval error vs fp64 at the mean - NOT fp32-class by "
                            "the 1.5x bar the 3xf16 default meets; the exactness / bit-comparison mode" % ratio["mean"]}
    return None


def distinct_devices(dev):
    """Number of distinct GPUs the ranks ran on: every rank contributes its device_key and the unique entries
    are counted, so multi-node jobs and launchers that give each rank one visible device are counted right
    (the local torch.cuda.device_count() sees only this process's devices)."""
    import socket
    import torch.distributed as dist
    key = device_key(socket.gethostname(), torch.cuda.get_device_properties(dev))
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return 1
    keys = [None] * dist.get_world_size()
    dist.all_gather_object(keys, key)
    return len(set(keys))


def parallelism_note(ws, ndev):
    """The parallel layout as it really ran: backend and distinct devices. Fewer GPUs than ranks (ranks
    sharing a device over gloo) is a rehearsal of the N-rank path, not an N-GPU measurement."""
    if ws == 1:
        return "dp1 (one GPU)"
    import torch.distributed as dist
    backend = dist.get_backend() if dist.is_initialized() else "none"
    note = f"dp{ws} (image shards over {ndev} device(s), {backend} all_gather of outputs)"
    if ndev < ws:
        note += " REHEARSAL: ranks share devices, not an N-GPU result"
    return note


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n):
    """Run this script as N ranks under torch.distributed.run (one process per GPU) and return its
    exit code. Called before anything here touches the GPU; the child is a separate process (no
    exec), and its stdout (rank 0's JSON line) is inherited."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def time_train(dev, B, precision, steps, warmup, rank=0):
    """`steps` timed training steps (after `warmup` untimed ones) of BASELINE configs[4] on `dev`: B synthetic 256x256
    images, t ~ randint, training_losses with injection, backward, clip_grad_norm_(1.0), AdamW
    (code/train_inpainting.py:15-79). Returns (max-over-ranks seconds, last loss, guard trips)."""
    from ifd import parallel
    from ifd.manifest import make_state_dict
    from ifd.schedules import create_gaussian_diffusion
    from ifd.topology import FULL
    from ifd.train import UNetTrainer
    H = FULL.image_size
    diff = create_gaussian_diffusion(steps=1000, learn_sigma=True, noise_schedule="quadratic")
    gt, mask = synth_inputs(B, H, seed=7 + rank, device=dev)
    masked = gt * (1 - mask)
    tr = UNetTrainer(FULL, device=dev, precision=precision, fuse_gn=os.environ.get("IFD_TRAIN_FUSE_GN", "1") != "0",
                     fuse_gnb=os.environ.get("IFD_TRAIN_FUSE_GNB", "1") != "0",
                     gnb_act=os.environ.get("IFD_TRAIN_GNB_ACT", "0") != "0")
    tr.load_state_dict(make_state_dict(FULL, seed=1))
    gen = torch.Generator(device=dev).manual_seed(1 + rank)

    def step():
        t = torch.randint(0, 1000, (B,), device=dev, generator=gen)
        return tr.train_step(diff, gt, masked, mask, t)
    for _ in range(warmup):
        step()
    parallel.barrier(dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize(dev)
    parallel.barrier(dev)
    el = parallel.max_over_ranks(time.perf_counter() - t0, dev)
    lv = float(loss)
    assert math.isfinite(lv)
    trips = tr.guard_trips
    del tr
    torch.cuda.empty_cache()
    return el, lv, trips


def train_main(args):
    """`--workload train`: BASELINE configs[4]'s training step (code/train_inpainting.py:15-79), B images per GPU
    at 256x256 (time_train). Step = one optimizer step. --precision 3xf16 (default): forward, dgrad and wgrad 3x3
    convs on the fp32-accurate split kernels (ifd/train.py UNetTrainer precision="3xf16"); fp32: every conv on fp32
    MFMA, as the reference trains (no bf16 / LoRA exists in the reference). At N=1 the other mode is timed beside it.
    Multi-GPU: per-rank steps (data parallelism would add an all-reduce of the 374 MB gradient; not part of
    the reference, which trains on one device)."""
    from ifd import parallel
    from ifd.topology import FULL, gflop_per_image
    rank, ws, local = parallel.world()
    dev = parallel.device_for(local)
    torch.cuda.set_device(dev)
    parallel.init(device=dev)
    B = args.batch
    prec = args.precision

    def run(precision, steps, warmup):
        return time_train(dev, B, precision, steps, warmup, rank)

    elapsed, lossv, trips = run(prec, args.steps, args.warmup)
    value = B * ws * args.steps / elapsed
    gf = gflop_per_image(FULL)
    res = {"metric": f"training step images/sec ({prec} fwd+bwd+clip+AdamW, 256x256 9-ch UNet)", "value": round(value, 4),
           "unit": "images/s", "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(elapsed / args.steps * 1e3, 2), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None,
           "dtype": {"fp32": "f32", "3xf16": "f32 (3xf16 split MFMA for the forward, dgrad and wgrad 3x3 convs)",
                     "f16": "f16 operands, fp32 accumulate (reduced precision, not fp32-class)"}[prec],
           "data": "synthetic (gt~U(-1,1), rectangle masks, seeded weights)",
           "config": {"workload": "train_inpainting.py train_epoch step (BASELINE configs[4]; the reference trains "
                                  "fp32 and has no bf16/LoRA)", "global_batch": B * ws, "batch_per_gpu": B,
                      "parallelism": f"{ws} independent ranks"},
           "loss": lossv, "guard_trips": trips,
           "algorithmic_tflops": round(3 * gf * B * ws * args.steps / elapsed / 1e3, 2)}
    if ws == 1 and args.fp32_exact_steps > 0 and prec != "fp32":
        el2, _, _ = run("fp32", args.fp32_exact_steps, 1)
        res["fp32_exact"] = {"value": round(B * args.fp32_exact_steps / el2, 4), "unit": "images/s",
                             "ms_per_step": round(el2 / args.fp32_exact_steps * 1e3, 2),
                             "steps": args.fp32_exact_steps}
    if ws == 1 and args.f16_steps > 0 and prec == "3xf16":
        # the reduced-precision variant (BASELINE configs[4]'s "bf16" wording; not fp32-class), timed separately
        el3, l3, t3 = run("f16", args.f16_steps, 1)
        res["f16_reduced"] = {"value": round(B * args.f16_steps / el3, 4), "unit": "images/s",
                              "ms_per_step": round(el3 / args.f16_steps * 1e3, 2), "steps": args.f16_steps,
                              "loss": l3, "guard_trips": t3,
                              "dtype": "f16 operands, fp32 accumulate (tests/test_gpu_train.py::test_train_f16_full_vs_fp32)"}
    if rank == 0:
        print(json.dumps(res), flush=True)


def ddpm_main(args):
    """`--workload ddpm`: BASELINE configs[2] (CelebA-HQ-shaped 256x256, B = 64 per GPU, DDPM-1000 linear,
    code/tes_ddpm.py:402-468): step = one full 1000-eval inpainting_p_sample_loop + final blend over B
    synthetic images; value = images/s. A full-step stress of the fused DDPM epilogue at B = 64 (the
    workspace arena at this batch is reported); not the headline line."""
    from ifd import parallel
    from ifd.manifest import make_state_dict
    from ifd.model import DiffusionInpaintingModel
    from ifd.sampler import InpaintingSampler
    from ifd.schedules import create_gaussian_diffusion
    from ifd.topology import FULL, gflop_per_image
    rank, ws, local = parallel.world()
    dev = parallel.device_for(local)
    torch.cuda.set_device(dev)
    parallel.init(device=dev)
    B, H = args.batch, FULL.image_size
    opts = model_options(args)
    model = DiffusionInpaintingModel(FULL, device=dev, precision=args.precision, options=opts)
    model.load_state_dict(make_state_dict(FULL, seed=1))
    diffusion = create_gaussian_diffusion(steps=args.ddpm_steps, learn_sigma=True, noise_schedule="linear")
    sampler = InpaintingSampler(model, diffusion, device=dev)
    gt, mask = synth_inputs(B, H, seed=7 + rank, device=dev)

    def one_pass(i):
        torch.manual_seed(42 + 1000 * rank + i)
        with torch.no_grad():
            y = sampler.inpainting_p_sample_loop(sampler.model_fn, (B, 3, H, H), gt, mask, True, dev, False)
            return parallel.gather_images(sampler.final_blend(y, gt, mask), B * ws)
    for i in range(args.warmup):
        one_pass(i)
    parallel.barrier(dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        y = one_pass(args.warmup + i)
    torch.cuda.synchronize(dev)
    parallel.barrier(dev)
    elapsed = parallel.max_over_ranks(time.perf_counter() - t0, dev)
    assert torch.isfinite(y).all()
    model.guard_check()  # the lazy range guard of the drop-in loop's forwards (raises on a trip)
    n_evals = diffusion.num_timesteps
    res = {"metric": "256x256 DDPM-1000 inpainted images/sec (BASELINE configs[2], full-step stress)",
           "value": round(B * ws * args.steps / elapsed, 4), "unit": "images/s", "n_gpus": ws, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 2),
           "unet_ms_per_eval": round(elapsed / args.steps / n_evals * 1e3, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f32" if args.precision == "fp32" else
           f"f32 ({args.precision} conv arithmetic)", "data": "synthetic",
           "config": {"workload": f"256x256 9-ch UNet inpainting, DDPM-{n_evals} linear (configs[2])",
                      "global_batch": B * ws, "batch_per_gpu": B, "unet_evals_per_image": n_evals},
           "algorithmic_tflops": round(gflop_per_image(FULL) * B * ws * n_evals * args.steps / elapsed / 1e3, 2),
           "torch_max_memory_allocated_gb": round(torch.cuda.max_memory_allocated(dev) / 1e9, 2)}
    import ctypes
    from ifd import _lib
    wb, wsb = ctypes.c_int64(), ctypes.c_int64()
    _lib.check(_lib.lib().ifd_memory(model.handle(dev).h, ctypes.byref(wb), ctypes.byref(wsb)))
    res["library_memory_gb"] = {"weights": round(wb.value / 1e9, 3), "workspace": round(wsb.value / 1e9, 3)}
    if rank == 0:
        print(json.dumps(res), flush=True)


def model_options(args):
    """Handle options the run's model is built with: parity mode fixes the conv geometry per image
    (`batch_invariant`), so a C4 shard of 64 images equals the same images run at any other batch size."""
    return {"batch_invariant": 1} if args.noise == "parity" else {}


def script_ddim_pass(model, alphas_cumprod, shape, gt_images, masks, ddim_steps, eta, device, clip_denoised=True):
    """The reference script's DDIM loop as it runs unchanged over this library's model
    (code/test_inp_ddim_100.py:470-576; model_fn :373-385): one `model(x, t, masked_image=, mask=)` per step,
    the DDIM update and the known-region injection in torch, the per-step alpha tensors built on the device
    from the float64 table exactly as the script builds them."""
    img = torch.randn(*shape, device=device)
    c = 1000 // ddim_steps
    seq = list(range(0, 1000, c))
    if seq[-1] != 999:
        seq.append(999)
    seq = seq[::-1]
    gt_keep_mask = 1 - masks
    for step_idx, timestep in enumerate(seq):
        t = torch.tensor([timestep] * shape[0], device=device)
        masked_image = gt_images * gt_keep_mask + torch.zeros_like(gt_images) * (1 - gt_keep_mask)
        model_output = model(img, t, masked_image=masked_image, mask=1 - gt_keep_mask)
        noise_pred = model_output[:, :3]
        alpha_t = torch.tensor(alphas_cumprod[timestep], device=device)
        alpha_prev = torch.tensor(alphas_cumprod[seq[step_idx + 1]] if step_idx < len(seq) - 1 else 1.0, device=device)
        pred_x0 = (img - torch.sqrt(1 - alpha_t) * noise_pred) / torch.sqrt(alpha_t)
        if clip_denoised:
            pred_x0 = torch.clamp(pred_x0, -1, 1)
        sigma = eta * torch.sqrt((1 - alpha_prev) / (1 - alpha_t)) * torch.sqrt(1 - alpha_t / alpha_prev)
        pred_dir = torch.sqrt(1 - alpha_prev - sigma ** 2) * noise_pred
        noise = torch.randn_like(img) if timestep > 0 and eta > 0 else torch.zeros_like(img)
        img = torch.sqrt(alpha_prev) * pred_x0 + pred_dir + sigma * noise
        if timestep > 0:
            known_noise = torch.randn_like(gt_images)
            noised_known_regions = torch.sqrt(alpha_prev) * gt_images + torch.sqrt(1 - alpha_prev) * known_noise
            img = img * masks + noised_known_regions * gt_keep_mask
    return img * masks + gt_images * (1 - masks)  # the script's final blend (:692-696)


def build_parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=16, help="images per GPU")
    ap.add_argument("--ddim-steps", type=int, default=100)
    ap.add_argument("--eta", type=float, default=0.75)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=20.0)
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--precision", choices=["fp32", "3xf16", "f16"], default="3xf16",
                    help="conv arithmetic: the fp32-accurate 3xf16 split MFMA (default), or exact fp32 MFMA")
    ap.add_argument("--fp32-exact-steps", type=int, default=1,
                    help="N=1 only: also time this many steps in exact-fp32 mode (0 = skip)")
    ap.add_argument("--f16-steps", type=int, default=1,
                    help="N=1 only: also time this many steps in the reduced-precision f16 mode, reported separately "
                         "(the reference's .half() experiment, code/test_quant.py:390-409; 0 = skip)")
    ap.add_argument("--train-steps", type=int, default=5,
                    help="sample workload, N=1 only: also time this many 3xf16 training steps (BASELINE configs[4], "
                         "B=--train-batch, after one warm-up step), reported as `train` beside the headline (0 = skip)")
    ap.add_argument("--train-batch", type=int, default=32, help="images per training step of the `train` leg")
    ap.add_argument("--ddpm-steps", type=int, default=1000, help="--workload ddpm: diffusion steps T (linear)")
    ap.add_argument("--workload", choices=["sample", "c4", "train", "ddpm", "dropin"], default="sample",
                    help="sample: the headline DDIM-100 sampler, --batch images per GPU (default; configs[1]); c4: the "
                         "same loop over a fixed global batch of 512 sharded over the ranks (configs[3]); train: the "
                         "training step (configs[4]); ddpm: DDPM-1000 at B=64 (configs[2]); dropin: configs[1] through "
                         "the reference script's own per-step loop over model() (the fused rate beside it)")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="sample / c4: total images over all ranks, sharded contiguously (sizes differ by at most "
                         "one; default --batch x ranks, or 512 for c4)")
    ap.add_argument("--noise", choices=["device", "parity"], default="device",
                    help="device: per-rank GPU RNG (throughput); parity: full-batch device draws in reference order, "
                         "sliced per rank, batch-invariant conv geometry (GPU-count-independent results)")
    return ap


def main():
    args = build_parser().parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    if args.workload == "train":
        return train_main(args)
    if args.workload == "ddpm":
        return ddpm_main(args)

    from ifd import parallel
    from ifd.manifest import make_state_dict
    from ifd.model import DiffusionInpaintingModel
    from ifd.sampler import InpaintingSampler
    from ifd.schedules import create_gaussian_diffusion
    from ifd.topology import FULL, gflop_per_image
    from ifd import _lib

    rank, ws, local = parallel.world()
    if ws != args.gpus and rank == 0:
        print(f"bench: WORLD_SIZE={ws} overrides --gpus {args.gpus}", file=sys.stderr)
    dev = parallel.device_for(local)
    torch.cuda.set_device(dev)
    parallel.init(device=dev)
    ndev = distinct_devices(dev)
    H = FULL.image_size
    c4 = args.workload == "c4"
    G = args.global_batch or (512 if c4 else args.batch * ws)  # the job's images (configs[3]: 512 over 8 GPUs)
    lo, hi = parallel.shard_range(G, rank, ws)
    B = hi - lo  # this rank's images
    if B < 1:
        raise SystemExit(f"bench: global batch {G} leaves rank {rank} of {ws} without images")

    opts = model_options(args)
    model = DiffusionInpaintingModel(FULL, device=dev, precision=args.precision, options=opts)
    model.load_state_dict(make_state_dict(FULL, seed=1))
    model.eval()
    diffusion = create_gaussian_diffusion(steps=1000, learn_sigma=True, noise_schedule="cosine")
    if args.noise == "parity":
        sampler = InpaintingSampler(model, diffusion, ddim_timesteps=args.ddim_steps, device=dev,
                                    noise_shard=(lo, hi, G))
        gt, mask = (v[lo:hi].contiguous() for v in synth_inputs(G, H, seed=7, device=dev))
    else:
        sampler = InpaintingSampler(model, diffusion, ddim_timesteps=args.ddim_steps, device=dev)
        gt, mask = synth_inputs(B, H, seed=7 + rank, device=dev)
    shape = (B, 3, H, H)
    n_evals = len(sampler.create_ddim_timestep_sequence(1000, args.ddim_steps))
    handle = model.handle(dev)
    L = _lib.lib()

    dropin = args.workload == "dropin"

    def fused_pass(i):
        torch.manual_seed(42 + i if args.noise == "parity" else 42 + 1000 * rank + i)
        with torch.no_grad():
            y = sampler.inpainting_ddim_sample_loop(sampler.model_fn, shape, gt, mask, True, dev, False, args.eta)
            y = sampler.final_blend(y, gt, mask)
            return parallel.gather_images(y, G)

    def dropin_pass(i):
        torch.manual_seed(42 + 1000 * rank + i)
        with torch.no_grad():
            y = script_ddim_pass(model, diffusion.alphas_cumprod, shape, gt, mask, args.ddim_steps, args.eta, dev)
            return parallel.gather_images(y, G)

    one_pass = dropin_pass if dropin else fused_pass

    prof = not args.no_profile
    import ctypes
    cbuf = ctypes.create_string_buffer(1 << 16)
    kernels = {}
    for i in range(args.warmup):
        full = prof and i == args.warmup - 1
        if full:  # per-kernel breakdown from the last warmup pass (every launch bracketed by events)
            _lib.check(L.ifd_profile_filter(handle.h, b""))
            _lib.check(L.ifd_profile_enable(handle.h, 1))
        one_pass(i)
        if full:
            torch.cuda.synchronize(dev)
            _lib.check(L.ifd_profile_report(handle.h, cbuf, len(cbuf)))
            _lib.check(L.ifd_profile_enable(handle.h, 0))
            kernels = json.loads(cbuf.value.decode())["kernels"]
    if prof:
        # timed region: events only around the dominant conv instantiation (from the breakdown;
        # every conv kernel when there was no warmup pass), not around all ~200 launches per eval
        convw = {k: v for k, v in kernels.items() if k.startswith("conv_")}
        dom_name = max(convw, key=lambda k: convw[k]["ms"]) if convw else "conv_"
        _lib.check(L.ifd_profile_filter(handle.h, dom_name.encode()))
        _lib.check(L.ifd_profile_enable(handle.h, 1))
    parallel.barrier(dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        y = one_pass(args.warmup + i)
    torch.cuda.synchronize(dev)
    parallel.barrier(dev)
    elapsed = parallel.max_over_ranks(time.perf_counter() - t0, dev)
    assert torch.isfinite(y).all()
    model.guard_check()  # the lazy range guard of the drop-in loop's forwards (raises on a trip)

    roofline = None
    if prof:
        _lib.check(L.ifd_profile_report(handle.h, cbuf, len(cbuf)))
        _lib.check(L.ifd_profile_enable(handle.h, 0))
        _lib.check(L.ifd_profile_filter(handle.h, b""))
        timed = json.loads(cbuf.value.decode())["kernels"]
        conv_t = {k: v for k, v in timed.items() if k.startswith("conv_")}
        dom = max(conv_t, key=lambda k: conv_t[k]["ms"])
        d = conv_t[dom]  # launch durations measured live in the timed region
        conv = {k: v for k, v in (kernels or timed).items() if k.startswith("conv_")}
        achieved = d["flops"] / (d["ms"] * 1e-3) / 1e12
        f16_1 = dom.startswith("conv_x3") and dom.endswith(",1>")  # the f16 mode: one product per MAC
        peak = PEAK_F16_TFLOPS if f16_1 else (PEAK_3XF16_TFLOPS if dom.startswith("conv_x3") else PEAK_FP32_TFLOPS)
        roofline = {"bound": "mfma", "achieved": round(achieved, 2), "peak": round(peak, 1), "unit": "TFLOP/s",
                    "frac": round(achieved / peak, 4), "traffic": None, "kernel": dom,
                    "peak_basis": ("dense f16 MFMA 2.5 PFLOP/s (f16 mode: one product per MAC)" if f16_1 else
                                   "dense f16 MFMA 2.5 PFLOP/s / 3 split products per fp32 MAC (algorithmic fp32 "
                                   "FLOP/s ceiling of the 3xf16 kernel)" if dom.startswith("conv_x3")
                                   else "dense fp32 MFMA (= fp32 vector rate)"),
                    "avg_launch_ms": d["ms"] / d["count"], "flops_per_launch": d["flops"] / d["count"],
                    "algorithmic_bytes_per_launch": d["bytes"] / d["count"], "launches": int(d["count"])}
        roofline.update(pmc_traffic(dom))
        if roofline["traffic"]:
            roofline["traffic_over_algorithmic"] = round(roofline["traffic"] / roofline["algorithmic_bytes_per_launch"], 3)
        tot_ms = sum(v["ms"] for v in (kernels or timed).values())
        conv_flops = sum(v["flops"] for v in conv.values())
        conv_ms = sum(v["ms"] for v in conv.values())
        roofline["all_conv_launches"] = {"achieved": round(conv_flops / (conv_ms * 1e-3) / 1e12, 2),
                                         "time_share": round(conv_ms / tot_ms, 4)}

    value = G * args.steps / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    res = {
        "metric": "256x256 DDIM-100 inpainted images/sec at 1/2/4/8 MI355X; per-step UNet ms",
        "value": round(value, 4),
        "unit": "images/s",
        "n_gpus": ndev,
        "n_ranks": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 2),
        "unet_ms_per_eval": round(ms_per_step / n_evals, 3),
        "unet_ms_per_eval_note": "per UNet eval of the largest rank's shard (the slowest rank sets the time)",
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value * README_S_PER_SAMPLE_DDIM100, 2),
        "vs_baseline_ref": "reference README.md:76: DDIM-100 3.42 s/sample (unstated GPU, batch 4)",
        "dtype": "f32" if args.precision == "fp32" else "f32 (3xf16 split MFMA, fp32 accumulate)",
        "precision": {"mode": args.precision,
                      "note": ("exact fp32 MFMA (an fp32 fma chain)" if args.precision == "fp32" else
                               "each fp32 operand = f16 hi + f16 lo; 3 exact f16 MFMA products per MAC, hi x hi into "
                               "one fp32 accumulator and the two correction products into a second, added once per "
                               "output; error vs an fp64 UNet within ~1.2x of the reference's own fp32 error "
                               "(tests/test_gpu_full.py::test_c1_eval_error_vs_fp64, tools/diag/acc_model.py)")},
        "data": "synthetic (gt~U(-1,1), centre-square + rectangle masks, seeded random-init weights)",
        "noise": args.noise,
        "config": {"workload": ("C4: CelebA-HQ-shaped 256x256, global batch sharded over the ranks, DDIM-100 cosine "
                                "T=1000 eta=0.75, all_gather of the outputs (BASELINE configs[3])" if c4 else
                                "256x256 9-ch UNet inpainting, DDIM-100 cosine T=1000 eta=0.75 (BASELINE configs[1]) "
                                "through the reference script's per-step loop over model() "
                                "(code/test_inp_ddim_100.py:470-576, sync range guard)" if dropin else
                                "256x256 9-ch UNet inpainting, DDIM-100 cosine T=1000 eta=0.75 (BASELINE configs[1])"),
                   "options": opts,
                   "global_batch": G, "batch_per_gpu": B if G % ws == 0 else f"{G // ws}-{-(-G // ws)}",
                   "unet_evals_per_image": n_evals,
                   "gflop_per_unet_eval_per_image": round(gflop_per_image(FULL), 2),
                   "parallelism": parallelism_note(ws, ndev)},
        "roofline": roofline,
        "cpu_baseline": None,
    }
    if dropin:  # the fused loop of the same run, same inputs, for the gap
        fused_pass(0)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for i in range(args.steps):
            fused_pass(1 + i)
        torch.cuda.synchronize(dev)
        elf = parallel.max_over_ranks(time.perf_counter() - t1, dev)
        res["fused"] = {"value": round(G * args.steps / elf, 4), "unit": "images/s",
                        "ms_per_step": round(elf / args.steps * 1e3, 2),
                        "dropin_over_fused": round(value / (G * args.steps / elf), 4)}
    extras = ws == 1 and not c4 and not dropin  # the other arithmetic modes beside the headline, N = 1 only
    if extras and args.precision != "fp32" and args.fp32_exact_steps > 0:
        # the same workload in exact-fp32 mode, timed separately (same inputs, same clocked region)
        model.precision = "fp32"
        one_pass(0)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for i in range(args.fp32_exact_steps):
            one_pass(1 + i)
        torch.cuda.synchronize(dev)
        el32 = time.perf_counter() - t1
        model.precision = args.precision
        res["fp32_exact"] = {"value": round(B * args.fp32_exact_steps / el32, 4), "unit": "images/s",
                             "ms_per_step": round(el32 / args.fp32_exact_steps * 1e3, 2),
                             "steps": args.fp32_exact_steps, "warmup": 1, "dtype": "f32",
                             "accuracy_vs_reference": fp32_accuracy_note()}
    if extras and args.precision == "3xf16" and args.f16_steps > 0:
        # the reduced-precision variant (not fp32-class), same workload, timed separately
        model.precision = "f16"
        one_pass(0)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for i in range(args.f16_steps):
            one_pass(1 + i)
        torch.cuda.synchronize(dev)
        el16 = time.perf_counter() - t1
        model.precision = args.precision
        res["f16_reduced"] = {"value": round(B * args.f16_steps / el16, 4), "unit": "images/s",
                              "ms_per_step": round(el16 / args.f16_steps * 1e3, 2), "steps": args.f16_steps,
                              "warmup": 1, "dtype": "f16 operands, fp32 accumulate (not fp32-class; "
                                                    "tests/test_gpu_f16.py records its error)"}
    if extras and args.train_steps > 0:
        # BASELINE configs[4] on the driver's clock: the 3xf16 training step at B = 32 (time_train), after the
        # sampler's lines; the sampler's workspace arena is released first
        model._handle = model._lz = None
        torch.cuda.synchronize(dev)
        torch.cuda.empty_cache()
        try:
            elt, lt, tt = time_train(dev, args.train_batch, "3xf16", args.train_steps, 1)
        except Exception as e:  # the headline line is still printed; the failure is reported in it
            print(f"bench: training leg failed: {e!r}", file=sys.stderr)
            elt = None
    if extras and args.train_steps > 0 and elt is None:
        res["train"] = {"error": "the training leg raised (stderr has the exception)"}
    elif extras and args.train_steps > 0:
        res["train"] = {"value": round(args.train_batch * args.train_steps / elt, 4), "unit": "images/s",
                        "ms_per_step": round(elt / args.train_steps * 1e3, 2), "steps": args.train_steps, "warmup": 1,
                        "batch": args.train_batch, "loss": lt, "guard_trips": tt,
                        "workload": "train_inpainting.py train_epoch step: training_losses + backward + "
                                    "clip_grad_norm_(1.0) + AdamW, 256x256 9-ch UNet (BASELINE configs[4])",
                        "dtype": "f32 (3xf16 split MFMA for the forward, dgrad and wgrad convs)",
                        "algorithmic_tflops": round(3 * gflop_per_image(FULL) * args.train_batch * args.train_steps
                                                    / elt / 1e3, 2)}
    if rank == 0 and kernels:
        res["kernels"] = {k: {"count": int(v["count"]), "ms": round(v["ms"], 3)} for k, v in kernels.items()}
    # the process group goes first: no rank then waits inside a collective while rank 0 times the CPU path
    if ws > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    if rank == 0:
        if args.cpu_baseline_seconds > 0:  # on this node's host cores, at any N, after the timed region
            res["cpu_baseline"] = cpu_baseline(args.cpu_baseline_seconds)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
