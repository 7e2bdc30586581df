"""BASELINE configs the other GPU tests do not run at their own sizes:

  * C4's per-rank shard (configs[3]: B=512 over 8 GPUs = 64 images per rank, DDIM-100 cosine,
    eta 0.75; code/test_inp_ddim_100.py:470-576): the first steps of the fused DDIM loop at B=64,
    256x256, in both modes, and the whole 100-step trajectory in 3xf16 (finite, no range-guard trip).
    With the batch-invariant geometry (the multi-GPU parity mode) images equal their own B=1 runs bit
    for bit, the noise drawn for the full batch and sliced.
  * C5's batch (configs[4]: the training step at B=32, code/train_inpainting.py:15-79): the full-size
    3xf16 step against the fp32 step, the gates of test_gpu_train.py::test_train_x3_full_matches_fp32.
  * The timed B=16 bench geometry (default options: persistent split-kernel units, four-image 8x8
    tiles, split-K 1x1 launches) pinned to the reference itself: the reference fixture's image sits in
    slot k of a batch of 16 random images; slot k must be within 1e-5 of the reference's UNet output.
  * The workspace arena at B=16 and B=64 (recorded next to the host-side plan).

Tolerances (written here): C4 slices bit-identical; C5 loss rel 1e-5, grad norm rel 1e-5, every
parameter gradient rel-L2 1e-4 vs fp32, no guard trip; bench geometry max-abs 1e-5 (the per-eval gate
of test_gpu_parity.py / test_gpu_x3.py at B=1).
"""
import ctypes

import numpy as np
import pytest
import torch

from ifd.manifest import make_state_dict
from ifd.topology import FULL

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
PRECISIONS = ["fp32", "3xf16"]


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


_MODELS = {}


def _model(prec, **options):
    from ifd.model import DiffusionInpaintingModel
    key = (prec, tuple(sorted(options.items())))
    if key not in _MODELS:
        _MODELS.clear()  # one full-size handle (and its arena) alive at a time
        torch.cuda.empty_cache()
        m = DiffusionInpaintingModel(FULL, device=DEV, precision=prec, options=options)
        m.load_state_dict(make_state_dict(FULL, seed=1))
        _MODELS[key] = m.eval()
    return _MODELS[key]


def _ddim_steps(model, gt, mask, steps, seed, eta=0.75, noise_shard=None):
    """The first `steps` iterations of inpainting_ddim_sample_loop (DDIM-100 cosine) through
    ifd_ddim_step, draws in the reference's order (code/test_inp_ddim_100.py:481,554,567)."""
    from ifd import _lib
    from ifd.sampler import InpaintingSampler, ddim_coeffs
    from ifd.schedules import create_gaussian_diffusion
    diff = create_gaussian_diffusion(steps=1000, learn_sigma=True, noise_schedule="cosine")
    s = InpaintingSampler(model, diff, ddim_timesteps=100, device=DEV, noise_device="cpu", noise_shard=noise_shard)
    seq = s.create_ddim_timestep_sequence(1000, 100)
    B, _, H, W = gt.shape
    h = model.handle(DEV)
    L = _lib.lib()
    torch.manual_seed(seed)
    img = s._randn((B, 3, H, W), DEV)
    with torch.no_grad():
        for k in range(steps):
            c = ddim_coeffs(diff.alphas_cumprod, seq, k, eta)
            t = torch.full((B,), int(seq[k]), device=DEV, dtype=torch.int64)
            noise = s._randn((B, 3, H, W), DEV) if c.use_noise else None
            known = s._randn((B, 3, H, W), DEV) if c.inject else None
            _lib.check(L.ifd_ddim_step(h.h, _lib.ptr(t), B, H, W, _lib.ptr(img), _lib.ptr(gt), _lib.ptr(mask),
                                       _lib.ptr(noise), _lib.ptr(known), c, _lib.stream_ptr(DEV)))
    torch.cuda.synchronize()
    return img


@pytest.mark.parametrize("prec", PRECISIONS)
def test_c4_rank_shard_ddim100_b64(record, prec):
    """C4 per rank: B=64 at 256x256, three DDIM-100 cosine steps (eta 0.75) are finite and images
    0, 37 and 63 equal their own B=1 runs bit for bit (batch-invariant geometry, full-batch noise
    sliced per image)."""
    from bench import synth_inputs
    B = 64
    gt, mask = synth_inputs(B, 256, seed=7, device=DEV)
    m = _model(prec, batch_invariant=1)
    y = _ddim_steps(m, gt, mask, 3, seed=42)
    assert torch.isfinite(y).all()
    diffs = {}
    for i in (0, 37, 63):
        y1 = _ddim_steps(m, gt[i:i + 1].contiguous(), mask[i:i + 1].contiguous(), 3, seed=42,
                         noise_shard=(i, i + 1, B))
        diffs[i] = float((y1 - y[i:i + 1]).abs().max())
        assert torch.equal(y1, y[i:i + 1]), (i, diffs[i])
    wb, wsb = m.memory()
    record(f"c4_rank_shard_b64_ddim3/{prec}", slice_vs_b1_maxabs=max(diffs.values()), workspace_bytes=wsb,
           weight_bytes=wb)


def test_c4_rank_shard_full_trajectory(record):
    """C4 per rank, the WHOLE trajectory: B=64 at 256x256, all 100 DDIM steps (cosine, eta 0.75, the
    sampler's own loop with device-side full-batch draws) + the final blend in 3xf16 (the default
    arithmetic). The output is finite, the range guard never trips (late-trajectory activations are the
    ones that could approach the f16 range), and images 0 and 63 equal their own B=1 runs bit for bit
    (batch-invariant geometry; the B=1 runs draw the full batch's noise and keep their row)."""
    from bench import synth_inputs
    from ifd.sampler import InpaintingSampler
    from ifd.schedules import create_gaussian_diffusion
    B, H = 64, 256
    gt, mask = synth_inputs(B, H, seed=7, device=DEV)
    m = _model("3xf16", batch_invariant=1)
    trips0 = m.guard_trips
    diff = create_gaussian_diffusion(steps=1000, learn_sigma=True, noise_schedule="cosine")

    def run(lo, hi, shard):
        s = InpaintingSampler(m, diff, ddim_timesteps=100, device=DEV, noise_shard=(lo, hi, B) if shard else None)
        torch.manual_seed(42)
        with torch.no_grad():
            y = s.inpainting_ddim_sample_loop(s.model_fn, (hi - lo, 3, H, H), gt[lo:hi].contiguous(),
                                              mask[lo:hi].contiguous(), True, DEV, False, 0.75)
            return s.final_blend(y, gt[lo:hi].contiguous(), mask[lo:hi].contiguous())
    y = run(0, B, False)
    torch.cuda.synchronize()
    assert torch.isfinite(y).all()
    assert m.guard_trips == trips0
    diffs = {}
    for i in (0, 63):
        y1 = run(i, i + 1, True)
        diffs[i] = float((y1 - y[i:i + 1]).abs().max())
        assert torch.equal(y1, y[i:i + 1]), (i, diffs[i])
    assert m.guard_trips == trips0
    record("c4_rank_shard_b64_ddim100_full/3xf16", slice_vs_b1_maxabs=max(diffs.values()),
           out_absmax=float(y.abs().max()), guard_trips=m.guard_trips - trips0)


def test_workspace_arena_matches_plan(record):
    """The arena a forward allocates equals the host-side plan (ifd_workspace_plan), and stays near
    the activation bound: ~4.1 GB at B=16, ~16.6 GB at B=64 (round 2 reserved 67.9 GB at B=64)."""
    from ifd import _lib
    from bench import synth_inputs
    m = _model("3xf16")
    h = m.handle(DEV)
    got = {}
    for B in (16, 64):
        plan = ctypes.c_int64()
        _lib.check(_lib.lib().ifd_workspace_plan(h.h, B, ctypes.byref(plan)))
        gt, mask = synth_inputs(B, 256, seed=1, device=DEV)
        x = torch.randn(B, 3, 256, 256, device=DEV)
        with torch.no_grad():
            y = m(x, torch.full((B,), 500, device=DEV), masked_image=gt * (1 - mask), mask=mask)
        assert torch.isfinite(y).all()
        got[B] = m.memory()[1]
        assert got[B] == plan.value, (B, got[B], plan.value)
        del y, x, gt, mask
    record("workspace_arena", bytes_b16=got[16], bytes_b64=got[64])
    assert got[64] <= 20e9


@pytest.mark.parametrize("prec", PRECISIONS)
@pytest.mark.parametrize("slot", [0, 5, 15])
def test_bench_geometry_pinned_to_reference(evals, record, prec, slot):
    """The B=16 geometry bench.py times (default handle options), pinned to the reference: the
    reference fixture's (x, gt, mask) at t=999 in slot `slot` of 15 random images; that slot's output
    is within 1e-5 of the reference's own UNet output (code/unet.py:154-200)."""
    B = 16
    g = torch.Generator(device=DEV).manual_seed(100 + slot)
    x = torch.randn(B, 3, 256, 256, device=DEV, generator=g)
    gt = torch.rand(B, 3, 256, 256, device=DEV, generator=g) * 2 - 1
    mask = (torch.rand(B, 1, 256, 256, device=DEV, generator=g) > 0.5).float()
    t = torch.randint(0, 1000, (B,), device=DEV, generator=g)
    x[slot], gt[slot], mask[slot] = (_t(evals[f"full/{k}"])[0].to(DEV) for k in ("x", "gt", "mask"))
    t[slot] = 999
    m = _model(prec)
    with torch.no_grad():
        y = m(x, t, masked_image=gt * (1 - mask), mask=mask)
    assert torch.isfinite(y).all()
    err = float((y[slot:slot + 1].double().cpu() - _t(evals["full_t999/y"]).double()).abs().max())
    record(f"bench_geometry_slot{slot}/{prec}", maxabs=err)
    assert err <= 1e-5, err


def test_c5_train_b32_x3_matches_fp32(record):
    """C5 at its batch (B=32, 256x256): one 3xf16 training step against the fp32 step from the same
    state, noise and GT-noise draw; the gates of test_train_x3_full_matches_fp32."""
    from test_gpu_train import _full_step
    _MODELS.clear()
    torch.cuda.empty_cache()
    tr32, l32 = _full_step("fp32", B=32)
    g32 = tr32.grad.clone()
    n32 = float(tr32.norm_coef[0])
    offs = tr32.offsets
    del tr32
    torch.cuda.empty_cache()
    tr3, l3 = _full_step("3xf16", B=32)
    assert tr3.guard_trips == 0
    rel_loss = abs(l3 - l32) / abs(l32)
    rel_gn = abs(float(tr3.norm_coef[0]) - n32) / n32
    worst, wname = 0.0, None
    for k, (o, shape) in offs.items():
        n = int(np.prod(shape))
        a, b = tr3.grad[o:o + n].double(), g32[o:o + n].double()
        bn = float(b.norm())
        if bn == 0.0:
            continue
        r = float((a - b).norm()) / bn
        if r > worst:
            worst, wname = r, k
    record("train_x3_b32_vs_fp32", loss=l3, loss_fp32=l32, rel_loss=rel_loss, rel_grad_norm=rel_gn,
           max_tensor_grad_rel=worst, worst_tensor=wname)
    del tr3
    torch.cuda.empty_cache()
    assert rel_loss <= 1e-5 and rel_gn <= 1e-5, (rel_loss, rel_gn)
    assert worst <= 1e-4, (worst, wname)
