"""GPU parity at full size (256x256): the headline DDIM-100 loop (C2), the DDPM-1000 loop (C3),
the B=64 DDPM workload, sharded == unsharded sampling, the fp64-referenced C1 error budget and
`sample_with_advanced_inpainting`. Fixtures: tests/golden/full/ (make_golden_full.py, made by
importing the reference). Every measured error is recorded (conftest `record`).

Tolerances (written here, fp32 class throughout):
  * C2 / C3 full loops vs the reference:           max-abs < 1e-4 (north_star), both modes
  * UNet eval error vs an fp64 UNet (C1's eval):   3xf16 (the default mode): mean and p99.9 within
                                                   1.5x of the fp32 reference's own error vs fp64,
                                                   max within 2x (measured 1.16x / 1.15x / 1.21x).
                                                   fp32 mode: 3x / 4x — its MFMA chain sums K = 9 Cin
                                                   terms sequentially in one accumulator with one
                                                   rounding per product (measured 2.6x oneDNN's mean)
  * C1 10-step loops vs the fp64 loop:             3xf16: p99.9 within 2x of the reference's own
                                                   p99.9 vs the fp64 loop, max within 2.5x (measured
                                                   1.40x / 2.08x at eta 0). The max is a tail statistic
                                                   of a chaotic loop: a rel-1e-6 perturbation of eps
                                                   alone moves it by 4.4e-3 = 4.9x the reference's
                                                   (golden/conditioning.json). fp32 mode: the rel-1e-5
                                                   perturbation envelope (max, p99.9)
  * advanced-inpainting loops vs the fp64 loop:    max-abs within max(1e-4, 4x the reference's)
  * sharded vs unsharded (batch_invariant option): bit-identical
"""
import numpy as np
import pytest
import torch

from conftest import golden_full
from ifd.manifest import make_state_dict
from ifd.topology import FULL, REDUCED

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
PRECISIONS = ["fp32", "3xf16"]


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def _stats(a, b):
    d = (a.double().cpu() - b.double().cpu()).abs().flatten()
    return {"max": float(d.max()), "p999": float(d.quantile(0.999)), "mean": float(d.mean())}


_MODELS = {}


def _model(prec, cfg=FULL, **options):
    from ifd.model import DiffusionInpaintingModel
    key = (prec, cfg.image_size, tuple(sorted(options.items())))
    if key not in _MODELS:
        m = DiffusionInpaintingModel(cfg, device=DEV, precision=prec, options=options)
        m.load_state_dict(make_state_dict(cfg, seed=1))
        _MODELS[key] = m.eval()
    return _MODELS[key]


def _script_loop(model, lm, gt, mask, **sampler_kw):
    from ifd.sampler import InpaintingSampler
    from ifd.schedules import create_gaussian_diffusion
    diff = create_gaussian_diffusion(steps=lm["T"], learn_sigma=True, noise_schedule=lm["schedule"])
    s = InpaintingSampler(model, diff, ddim_timesteps=lm["ddim_steps"] or 100, device=DEV, noise_device="cpu",
                          **sampler_kw)
    H = gt.shape[-1]
    shape = (gt.shape[0], 3, H, H)
    torch.manual_seed(lm["seed"])
    with torch.no_grad():
        if lm["method"] == "ddim":
            y = s.inpainting_ddim_sample_loop(s.model_fn, shape, gt.to(DEV), mask.to(DEV), True, DEV, False, lm["eta"])
        else:
            y = s.inpainting_p_sample_loop(s.model_fn, shape, gt.to(DEV), mask.to(DEV), True, DEV, False)
        return s.final_blend(y, gt.to(DEV), mask.to(DEV))


@pytest.mark.parametrize("prec", PRECISIONS)
def test_c2_ddim100_full(meta_full, record, prec):
    """BASELINE configs[1]'s loop at full size: code/test_inp_ddim_100.py:470-576, DDIM-100 cosine,
    eta 0.75, the real reference's output (B=1)."""
    name = "c2_cos100_eta0.75"
    g = golden_full(name)
    y = _script_loop(_model(prec), meta_full["loops"][name], _t(g["gt"]), _t(g["mask"]))
    s_ref = _stats(y, _t(g["y"]))
    s64 = _stats(y, _t(g["y64"]))
    record(f"{name}/{prec}", vs_reference=s_ref, vs_fp64=s64, reference_vs_fp64=meta_full["envelopes"][name])
    assert torch.isfinite(y).all()
    assert s_ref["max"] < 1e-4


@pytest.mark.parametrize("prec", PRECISIONS)
def test_c3_ddpm1000_full(meta_full, record, prec):
    """BASELINE configs[2]'s loop at full size: code/test_inp_ddim_50.py:402-468 (the tes_ddpm.py
    body), DDPM linear T=1000, the real reference's output (B=1), EPI_DDPM at cin 128 on 256x256."""
    name = "c3_ddpm_lin1000"
    g = golden_full(name)
    y = _script_loop(_model(prec), meta_full["loops"][name], _t(g["gt"]), _t(g["mask"]))
    s_ref = _stats(y, _t(g["y"]))
    record(f"{name}/{prec}", vs_reference=s_ref)
    assert torch.isfinite(y).all()
    assert s_ref["max"] < 1e-4


def _ddpm_steps(model, gt, mask, steps, seed, noise_shard=None):
    """The first `steps` iterations of inpainting_p_sample_loop (linear T=1000) through ifd_ddpm_step."""
    from ifd import _lib
    from ifd.sampler import InpaintingSampler, ddpm_coeffs
    from ifd.schedules import create_gaussian_diffusion
    diff = create_gaussian_diffusion(steps=1000, learn_sigma=True, noise_schedule="linear")
    s = InpaintingSampler(model, diff, device=DEV, noise_device="cpu", noise_shard=noise_shard)
    B, _, H, W = gt.shape
    h = model.handle(DEV)
    L = _lib.lib()
    torch.manual_seed(seed)
    img = s._randn((B, 3, H, W), DEV)
    with torch.no_grad():
        for i in range(999, 999 - steps, -1):
            c = ddpm_coeffs(diff, i)
            t = torch.full((B,), i, device=DEV, dtype=torch.int64)
            noise = s._randn((B, 3, H, W), DEV)
            known = s._randn((B, 3, H, W), DEV)
            _lib.check(L.ifd_ddpm_step(h.h, _lib.ptr(t), B, H, W, _lib.ptr(img), _lib.ptr(gt), _lib.ptr(mask),
                                       _lib.ptr(noise), _lib.ptr(known), c, _lib.stream_ptr(DEV)))
    torch.cuda.synchronize()
    return img


@pytest.mark.parametrize("prec", PRECISIONS)
def test_c3_batch64_ddpm_steps(record, prec):
    """The C3 workload size (B=64 at 256x256, 17.4 GB of workspace): three fused DDPM steps are
    finite, and with the batch-invariant geometry images 0, 37 and 63 equal their own B=1 runs
    (noise drawn for the full batch and sliced) bit for bit."""
    from bench import synth_inputs
    B = 64
    gt, mask = synth_inputs(B, 256, seed=7, device=DEV)
    m = _model(prec, batch_invariant=1)
    y = _ddpm_steps(m, gt, mask, 3, seed=5)
    assert torch.isfinite(y).all()
    diffs = {}
    for i in (0, 37, 63):
        y1 = _ddpm_steps(m, gt[i:i + 1].contiguous(), mask[i:i + 1].contiguous(), 3, seed=5,
                         noise_shard=(i, i + 1, B))
        diffs[i] = float((y1 - y[i:i + 1]).abs().max())
        assert torch.equal(y1, y[i:i + 1]), (i, diffs[i])
    record(f"c3_batch64_ddpm3/{prec}", slice_vs_b1_maxabs=max(diffs.values()), workspace_bytes=m.memory()[1])


@pytest.mark.parametrize("prec", PRECISIONS)
def test_sharded_equals_unsharded(record, prec):
    """Multi-GPU parity mode: B=4 sampled as two sequential 2-image shards, each with
    the full-batch noise sliced to its rows, is bit-identical to the B=4 run (DDIM-10 cosine,
    eta 0.75, 256x256, batch-invariant geometry)."""
    from bench import synth_inputs
    gt, mask = synth_inputs(4, 256, seed=7, device=DEV)
    lm = dict(T=1000, schedule="cosine", method="ddim", ddim_steps=10, eta=0.75, seed=42)
    m = _model(prec, batch_invariant=1)
    full = _script_loop(m, lm, gt, mask)
    parts = [_script_loop(m, lm, gt[lo:hi].contiguous(), mask[lo:hi].contiguous(), noise_shard=(lo, hi, 4))
             for lo, hi in ((0, 2), (2, 4))]
    sharded = torch.cat(parts, 0)
    record(f"sharded_vs_unsharded/{prec}", maxabs=float((sharded - full).abs().max()))
    assert torch.equal(sharded, full)


@pytest.mark.parametrize("prec", PRECISIONS)
def test_c1_eval_error_vs_fp64(meta_full, record, prec):
    """The per-eval error that the 10-step cosine loop (C1) amplifies: the GPU UNet against an
    fp64 UNet at t=999 on C1's own x_T, next to the fp32 reference's error against the same fp64
    output. The GPU must be an fp32-class UNet: mean and p99.9 within 2x, max within 4x."""
    g = golden_full("c1_eval0")
    ev = np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "loops.npz"))
    gt, mask = _t(ev["c1_full_cos10_eta0/gt"]).to(DEV), _t(ev["c1_full_cos10_eta0/mask"]).to(DEV)
    x = _t(g["x"]).to(DEV)
    with torch.no_grad():
        y = _model(prec)(x, torch.tensor([999], device=DEV), masked_image=gt * (1 - mask), mask=mask)
    s_gpu = _stats(y, _t(g["y64"]))
    s_ref = meta_full["envelopes"]["c1_eval0"]
    record(f"c1_eval0/{prec}", gpu_vs_fp64=s_gpu, reference_vs_fp64=s_ref, gpu_vs_reference=_stats(y, _t(g["y32"])))
    k, km = (1.5, 2) if prec == "3xf16" else (3, 4)
    assert s_gpu["mean"] <= k * s_ref["mean"] and s_gpu["p999"] <= k * s_ref["p999"]
    assert s_gpu["max"] <= km * s_ref["max"]


@pytest.mark.parametrize("prec", PRECISIONS)
@pytest.mark.parametrize("name", ["c1_full_cos10_eta0", "c1_full_cos10_eta0.9"])
def test_c1_loop_vs_fp64(meta, meta_full, loops, record, prec, name):
    """C1 (256x256, 10-step cosine): the first jump divides eps by sqrt(abar_999) = 4.9e-5, so
    pixels near the x0 clamp boundary amplify per-eval rounding ~2e4x. Measured against the
    fp64 oracle loop (exact arithmetic, same noise), next to the fp32 reference's own error.
    The loop is chaotic at the rounding level: two builds of the split kernels whose outputs along
    the same trajectory differ by 1e-7 (mean) and sit equally far from fp32 at every step
    (tools/diag/c1_states.py) ended 1e-3 and 9e-3 (max) from fp64. 3xf16 (the default): p99.9 within
    2x and max within 2.5x of the reference's own error against the same fp64 loop. fp32 mode (one
    rounding per product over K = 9 Cin, 2.6x the reference's per-eval error): the rel-1e-5
    perturbation envelope of tests/golden/conditioning.json (max, p99.9)."""
    import json
    import os
    cond = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "conditioning.json")))
    env = [v for k, v in cond.items() if k.startswith(name + "/rel1e-05")]
    lm = meta["loops"][name]
    gt, mask = _t(loops[f"{name}/gt"]), _t(loops[f"{name}/mask"])
    y = _script_loop(_model(prec), lm, gt, mask)
    y64 = _t(golden_full("c1_fp64")[f"{name}/y64"])
    s64 = _stats(y, y64)
    s_ref = _stats(y, _t(loops[f"{name}/y"]))
    record(f"{name}/{prec}", gpu_vs_fp64=s64, gpu_vs_reference=s_ref,
           reference_vs_fp64=meta_full["envelopes"][name],
           envelope={"max": max(v["max"] for v in env), "p999": max(v["p999"] for v in env)})
    r = meta_full["envelopes"][name]
    if prec == "3xf16":
        assert s64["p999"] <= 2 * r["p999"] and s64["max"] <= 2.5 * r["max"], (s64, r)
    else:
        assert s64["max"] <= max(1e-3, max(v["max"] for v in env))
        assert s64["p999"] <= max(1e-4, max(v["p999"] for v in env))


@pytest.mark.parametrize("prec", PRECISIONS)
@pytest.mark.parametrize("variant", ["adv_ddim_all", "adv_ddim_high_fresh", "adv_ddpm_low"])
def test_sample_with_advanced_inpainting(meta_full, record, variant, prec):
    """GaussianDiffusion.sample_with_advanced_inpainting (code/gaussian_diffusion.py:640-700) with the
    HIP model passed directly (its forward takes the gt/gt_keep_mask kwargs the library forwards),
    against the reference's output for DDIM eta 0.5 / DDPM and injection schedules all/high/low,
    cumulative and fresh-noise injection (reduced config, B=2, cosine T=40). The eta-0 "high"
    variant amplifies eval rounding like C1 (the reference itself is 1.2e-4 from the fp64 loop),
    so the gate is against the fp64 oracle loop: within max(1e-4, 4x the reference's error)."""
    from ifd.schedules import create_gaussian_diffusion
    lm = meta_full["loops"][variant]
    g = golden_full("adv_inpaint")
    gt, mask = _t(g[f"{variant}/gt"]).to(DEV), _t(g[f"{variant}/mask"]).to(DEV)
    diff = create_gaussian_diffusion(steps=lm["T"], learn_sigma=True, noise_schedule=lm["schedule"])
    diff.noise_device = "cpu"
    torch.manual_seed(lm["seed"])
    with torch.no_grad():
        y = diff.sample_with_advanced_inpainting(_model(prec, REDUCED), (2, 3, 64, 64), gt=gt, gt_keep_mask=1 - mask,
                                                 use_ddim=lm["use_ddim"], eta=lm["eta"], progress=False, device=DEV,
                                                 injection_schedule=lm["injection_schedule"],
                                                 use_cumulative_noise=lm["use_cumulative_noise"])
    s = _stats(y, _t(g[f"{variant}/y"]))
    s64 = _stats(y, _t(g[f"{variant}/y64"]))
    env = meta_full["envelopes"][variant]
    record(f"{variant}/{prec}", vs_reference=s, vs_fp64=s64, reference_vs_fp64=env)
    assert s64["max"] <= max(1e-4, 4 * env["max"]) and s64["p999"] <= max(1e-5, 4 * env["p999"])


def test_broadcast_mask_and_gt(record):
    """A [1,1,H,W] mask and a batch-1 gt are expanded like the reference broadcasts them: the
    fused loop equals the run with explicitly repeated tensors; a 3-channel mask is rejected."""
    from bench import synth_inputs
    gt, mask = synth_inputs(1, 64, seed=3, device=DEV)
    lm = dict(T=1000, schedule="cosine", method="ddim", ddim_steps=5, eta=0.9, seed=11)
    m = _model("fp32", REDUCED)
    a = _script_loop(m, lm, gt.expand(3, 3, 64, 64).contiguous(), mask.expand(3, 1, 64, 64).contiguous())
    from ifd.sampler import InpaintingSampler
    from ifd.schedules import create_gaussian_diffusion
    diff = create_gaussian_diffusion(steps=1000, learn_sigma=True, noise_schedule="cosine")
    s = InpaintingSampler(m, diff, ddim_timesteps=5, device=DEV, noise_device="cpu")
    torch.manual_seed(11)
    with torch.no_grad():
        b = s.inpainting_ddim_sample_loop(s.model_fn, (3, 3, 64, 64), gt, mask, True, DEV, False, 0.9)
        b = s.final_blend(b, gt, mask)
        assert torch.equal(a, b)
        with pytest.raises(ValueError):
            s.inpainting_ddim_sample_loop(s.model_fn, (3, 3, 64, 64), gt, mask.expand(1, 3, 64, 64), True, DEV,
                                          False, 0.9)
    record("broadcast_mask", equal=True)
