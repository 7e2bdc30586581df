"""GPU parity: the HIP path (through the C ABI) against the golden fixtures made by the reference.

Tolerances (fp32 throughout; the GPU convs sum in a different order than oneDNN):
  * one UNet eval:                    max-abs <= 1e-5 (outputs are O(1), std ~0.15)
  * update kernels vs oracle algebra: DDIM bit-exact; DDPM <= 2e-6 (expf ulp differences)
  * full loops:                       max-abs < 1e-4 (north_star), except the 256x256 10-step
                                      cosine C1 loops, whose first jump amplifies eval rounding
                                      ~1e4x at isolated pixels: bounded by the oracle's own
                                      perturbation envelope (test_script_ddim_full_c1).
"""
import os

import numpy as np
import pytest
import torch

from ifd.manifest import make_state_dict
from ifd.topology import FULL, REDUCED

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def maxabs(a, b):
    return float((a.double().cpu() - b.double().cpu()).abs().max())


@pytest.fixture(scope="module")
def red_model():
    from ifd.model import DiffusionInpaintingModel
    m = DiffusionInpaintingModel(REDUCED, device=DEV, precision="fp32")
    m.load_state_dict(make_state_dict(REDUCED, seed=1))
    return m.eval()


@pytest.fixture(scope="module")
def full_model():
    from ifd.model import DiffusionInpaintingModel
    m = DiffusionInpaintingModel(FULL, device=DEV, precision="fp32")
    m.load_state_dict(make_state_dict(FULL, seed=1))
    return m.eval()


def test_native_library_loaded(red_model):
    x = torch.zeros(1, 3, 64, 64, device=DEV)
    red_model(x, torch.tensor([5], device=DEV), masked_image=x, mask=x[:, :1])
    torch.cuda.synchronize()
    maps = open("/proc/self/maps").read()
    assert "libifd.so" in maps


def test_no_cpu_fallback(red_model):
    x = torch.zeros(1, 3, 64, 64)
    with pytest.raises(RuntimeError):
        red_model(x, torch.tensor([5]), masked_image=x, mask=x[:, :1])


@pytest.mark.parametrize("tv", [999, 500, 10])
def test_unet_reduced(evals, red_model, record, tv):
    x, gt, mask = (_t(evals[f"reduced/{k}"]).to(DEV) for k in ("x", "gt", "mask"))
    t = torch.tensor([tv] * x.shape[0], device=DEV)
    with torch.no_grad():
        y = red_model(x, t, masked_image=gt * (1 - mask), mask=mask)
    err = maxabs(y, _t(evals[f"reduced_t{tv}/y"]))
    record(f"unet_reduced_t{tv}/fp32", maxabs=err)
    assert err <= 1e-5


def test_unet_full(evals, full_model, record):
    x, gt, mask = (_t(evals[f"full/{k}"]).to(DEV) for k in ("x", "gt", "mask"))
    t = torch.tensor([999], device=DEV)
    with torch.no_grad():
        y = full_model(x, t, masked_image=gt * (1 - mask), mask=mask)
    err = maxabs(y, _t(evals["full_t999/y"]))
    record("unet_full_t999/fp32", maxabs=err)
    assert err <= 1e-5


def test_unet_batch_independent(evals, red_model):
    """Images are independent (GroupNorm/attention per sample): B=5 equals 5 x B=1."""
    x, gt, mask = (_t(evals[f"reduced/{k}"]).to(DEV) for k in ("x", "gt", "mask"))
    xs = torch.cat([x, x.flip(0), x[:1]], 0)
    gs = torch.cat([gt, gt.flip(0), gt[:1]], 0)
    ms = torch.cat([mask, mask.flip(0), mask[:1]], 0)
    t = torch.tensor([999, 500, 10, 1, 0], device=DEV)
    with torch.no_grad():
        yb = red_model(xs, t, masked_image=gs * (1 - ms), mask=ms)
        for i in range(5):
            y1 = red_model(xs[i:i + 1], t[i:i + 1], masked_image=(gs * (1 - ms))[i:i + 1], mask=ms[i:i + 1])
            assert torch.equal(y1, yb[i:i + 1]), i


@pytest.mark.parametrize("mode", ["1", "2"])
def test_stream_conv_bitwise(full_model, mode):
    """The persistent streaming convs (wide layers; mode 1: one workgroup per CU, mode 2: two)
    and the one-tile-per-workgroup conv sum in the same order: outputs must be bit-identical.
    B=3 256x256 also exercises tile counts that are not multiples of the grid. GroupNorm
    statistics come from the separate pass here (option gn_fused=0): the fused ones are merged per
    epilogue entry, whose shape differs between the kernels (covered by the golden tests)."""
    g = torch.Generator(device=DEV).manual_seed(3)
    x = torch.randn(3, 3, 256, 256, device=DEV, generator=g)
    gt = torch.rand(3, 3, 256, 256, device=DEV, generator=g) * 2 - 1
    mask = (torch.rand(3, 1, 256, 256, device=DEV, generator=g) > 0.5).float()
    t = torch.tensor([999, 500, 3], device=DEV)
    try:
        with torch.no_grad():
            full_model.options.update(gn_fused=0, conv_stream=int(mode))
            y1 = full_model(x, t, masked_image=gt * (1 - mask), mask=mask).clone()
            full_model.options["conv_stream"] = 0
            y0 = full_model(x, t, masked_image=gt * (1 - mask), mask=mask).clone()
    finally:
        full_model.options.update(gn_fused=1, conv_stream=2)
    assert torch.isfinite(y1).all()
    assert torch.equal(y0, y1), maxabs(y0, y1)


def _step_inputs(B=2, H=64, seed=0):
    g = torch.Generator().manual_seed(seed)
    out6 = torch.randn(B, 6, H, H, generator=g)
    img = torch.randn(B, 3, H, H, generator=g)
    gt = torch.rand(B, 3, H, H, generator=g) * 2 - 1
    mask = (torch.rand(B, 1, H, H, generator=g) > 0.5).float()
    noise = torch.randn(B, 3, H, H, generator=g)
    known = torch.randn(B, 3, H, H, generator=g)
    return out6, img, gt, mask, noise, known


@pytest.mark.parametrize("k", [0, 1, 5, 10])
def test_ddim_update_bitexact(k):
    """ifd_ddim_update == the script's torch arithmetic (float64 0-dim coefficients), bit for bit."""
    from ifd import _lib
    from ifd.sampler import InpaintingSampler, ddim_coeffs
    from ifd.schedules import create_gaussian_diffusion
    ac = create_gaussian_diffusion(steps=1000, learn_sigma=True, noise_schedule="cosine").alphas_cumprod
    seq = InpaintingSampler.create_ddim_timestep_sequence(1000, 10)
    eta = 0.9
    out6, img, gt, mask, noise, known = _step_inputs()
    tau = int(seq[k])
    # reference arithmetic (code/test_inp_ddim_50.py:523-574) on CPU
    eps = out6[:, :3]
    a_t = torch.tensor(ac[tau])
    a_p = torch.tensor(ac[seq[k + 1]]) if k < len(seq) - 1 else torch.tensor(1.0)
    x0 = torch.clamp((img - torch.sqrt(1 - a_t) * eps) / torch.sqrt(a_t), -1, 1)
    sigma = eta * torch.sqrt((1 - a_p) / (1 - a_t)) * torch.sqrt(1 - a_t / a_p)
    nz = noise if (tau > 0 and eta > 0) else torch.zeros_like(img)
    ref = torch.sqrt(a_p) * x0 + torch.sqrt(1 - a_p - sigma ** 2) * eps + sigma * nz
    if tau > 0:
        ref = ref * mask + (torch.sqrt(a_p) * gt + torch.sqrt(1 - a_p) * known) * (1 - mask)
    c = ddim_coeffs(ac, seq, k, eta)
    d = [v.to(DEV).contiguous() for v in (out6, img, gt, mask, noise, known)]
    B, _, H, W = img.shape
    _lib.check(_lib.lib().ifd_ddim_update(_lib.ptr(d[0]), B, H, W, _lib.ptr(d[1]), _lib.ptr(d[2]), _lib.ptr(d[3]),
                                          _lib.ptr(d[4]), _lib.ptr(d[5]), c, _lib.stream_ptr(DEV)))
    torch.cuda.synchronize()
    assert torch.equal(d[1].cpu(), ref), maxabs(d[1], ref)


@pytest.mark.parametrize("i", [999, 500, 1, 0])
def test_ddpm_update(i):
    """ifd_ddpm_update == p_mean_variance + the script update (oracle algebra on CPU)."""
    from ifd import _lib
    from ifd.sampler import ddpm_coeffs
    from ifd.schedules import create_gaussian_diffusion
    from oracle import ref_diffusion
    diff = create_gaussian_diffusion(steps=1000, learn_sigma=True, noise_schedule="linear")
    tb = ref_diffusion.Tables(diff.betas)
    out6, img, gt, mask, noise, known = _step_inputs(seed=3)
    B, _, H, W = img.shape
    t = torch.tensor([i] * B)
    o = ref_diffusion.p_mean_variance(tb, lambda x, tt: out6, img, t, True)
    ref = o["mean"] + (t != 0).float().view(-1, 1, 1, 1) * torch.exp(0.5 * o["log_variance"]) * noise
    if i > 0:
        a = torch.tensor(tb.ac[i - 1])
        ref = ref * mask + (torch.sqrt(a) * gt + torch.sqrt(1 - a) * known) * (1 - mask)
    c = ddpm_coeffs(diff, i)
    d = [v.to(DEV).contiguous() for v in (out6, img, gt, mask, noise, known)]
    _lib.check(_lib.lib().ifd_ddpm_update(_lib.ptr(d[0]), B, H, W, _lib.ptr(d[1]), _lib.ptr(d[2]), _lib.ptr(d[3]),
                                          _lib.ptr(d[4]), _lib.ptr(d[5]), c, _lib.stream_ptr(DEV)))
    torch.cuda.synchronize()
    assert maxabs(d[1], ref) <= 2e-6


def _run_script_loop(model, lm, gt, mask, fused=True):
    from ifd.sampler import InpaintingSampler
    from ifd.schedules import create_gaussian_diffusion
    diff = create_gaussian_diffusion(steps=lm["T"], learn_sigma=True, noise_schedule=lm["schedule"])
    s = InpaintingSampler(model, diff, ddim_timesteps=lm["ddim_steps"], device=DEV, noise_device="cpu")
    H = gt.shape[-1]
    shape = (lm["B"], 3, H, H)
    fn = s.model_fn if fused else (lambda x, t, **kw: s.model_fn(x, t, **kw))
    torch.manual_seed(lm["seed"])
    with torch.no_grad():
        if lm["method"] == "ddim":
            y = s.inpainting_ddim_sample_loop(fn, shape, gt.to(DEV), mask.to(DEV), True, DEV, False, lm["eta"])
        else:
            y = s.inpainting_p_sample_loop(fn, shape, gt.to(DEV), mask.to(DEV), True, DEV, False)
        y = s.final_blend(y, gt.to(DEV), mask.to(DEV))
    return y


@pytest.mark.parametrize("name", ["red_cos10_eta0.9", "red_lin500_ddim10_eta0.9", "red_quad_ddim30_eta0.9",
                                  "red_cos100_eta0.75"])
def test_script_ddim_reduced(loops, meta, red_model, record, name):
    lm = meta["loops"][name]
    gt, mask = _t(loops[f"{name}/gt"]), _t(loops[f"{name}/mask"])
    y = _run_script_loop(red_model, lm, gt, mask)
    err = maxabs(y, _t(loops[f"{name}/y"]))
    tol = 1e-3 if (lm["schedule"] == "cosine" and lm["ddim_steps"] <= 10) else 1e-4
    record(f"{name}/fp32", maxabs=err, tol=tol)
    assert err < tol


def test_script_ddim_unfused_matches_fused(loops, meta, red_model):
    name = "red_quad_ddim30_eta0.9"
    lm = meta["loops"][name]
    gt, mask = _t(loops[f"{name}/gt"]), _t(loops[f"{name}/mask"])
    a = _run_script_loop(red_model, lm, gt, mask, fused=True)
    b = _run_script_loop(red_model, lm, gt, mask, fused=False)
    assert torch.equal(a, b)


def test_script_ddpm_reduced(loops, meta, red_model, record):
    name = "red_ddpm_lin1000"
    lm = meta["loops"][name]
    gt, mask = _t(loops[f"{name}/gt"]), _t(loops[f"{name}/mask"])
    y = _run_script_loop(red_model, lm, gt, mask)
    err = maxabs(y, _t(loops[f"{name}/y"]))
    record(f"{name}/fp32", maxabs=err)
    assert err < 1e-4


@pytest.mark.parametrize("name", ["lib_ddim_lin50_eta0.5", "lib_ddpm_cos50"])
def test_library_loops(loops, meta, red_model, record, name):
    from ifd.diffusion import GaussianDiffusion  # noqa: F401
    from ifd.sampler import InpaintingSampler
    from ifd.schedules import create_gaussian_diffusion
    lm = meta["loops"][name]
    diff = create_gaussian_diffusion(steps=lm["T"], learn_sigma=True, noise_schedule=lm["schedule"])
    diff.noise_device = "cpu"
    s = InpaintingSampler(red_model, diff, device=DEV)
    gt, mask = _t(loops[f"{name}/gt"]).to(DEV), _t(loops[f"{name}/mask"]).to(DEV)
    kw = {"gt": gt, "gt_keep_mask": 1 - mask}
    shape = (lm["B"], 3, 64, 64)
    torch.manual_seed(lm["seed"])
    with torch.no_grad():
        if lm["method"] == "lib_ddim":
            y = diff.ddim_sample_loop(s.model_fn, shape, clip_denoised=True, model_kwargs=kw, device=DEV,
                                      eta=lm["eta"], use_inpainting_injection=True)
        else:
            y = diff.p_sample_loop(s.model_fn, shape, clip_denoised=True, model_kwargs=kw, device=DEV,
                                   use_inpainting_injection=True)
    err = maxabs(y, _t(loops[f"{name}/y"]))
    record(f"{name}/fp32", maxabs=err)
    assert err < 1e-4


@pytest.mark.parametrize("name", ["c1_full_cos10_eta0.9", "c1_full_cos10_eta0"])
def test_script_ddim_full_c1(loops, meta, full_model, record, name):
    """C1 (256x256, 10-step cosine): the first jump 999->900 divides eps by sqrt(abar_999) = 4.9e-5,
    so the few pixels near the x0 clamp boundary amplify ANY eval rounding difference ~1e4x.
    Bound = the oracle's OWN envelope when its eps is perturbed by a relative 1e-5 (our per-eval
    deviation from oneDNN is <= ~1e-5 relative; tests/golden/conditioning.py): max-abs, 99.9th
    percentile and the fraction of pixels off by > 1e-4 each within that envelope's."""
    import json
    cond = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "conditioning.json")))
    env = [v for k, v in cond.items() if k.startswith(name + "/rel1e-05")]
    env_max = max(v["max"] for v in env)
    env_frac = max(v["frac_gt_1e-4"] for v in env)
    env_p999 = max(v["p999"] for v in env)
    lm = meta["loops"][name]
    gt, mask = _t(loops[f"{name}/gt"]), _t(loops[f"{name}/mask"])
    y = _run_script_loop(full_model, lm, gt, mask)
    d = (y.double().cpu() - _t(loops[f"{name}/y"]).double()).abs().flatten()
    err, p999, frac = float(d.max()), float(d.quantile(0.999)), float((d > 1e-4).double().mean())
    tol = max(1e-3, env_max)
    record(f"{name}/fp32/vs_reference", maxabs=err, p999=p999, frac_gt_1e4=frac, envelope_rel1e5_max=env_max)
    assert err <= tol and p999 <= max(1e-4, env_p999) and frac <= max(env_frac, 1e-5)
