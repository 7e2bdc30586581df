"""GPU parity of the 3xf16 split-precision mode (precision="3xf16", include/ifd.h IFD_PREC_3XF16).

The same golden fixtures and tolerances as the fp32 mode (test_gpu_parity.py): the split path is
claimed fp32-accurate, so it gets no looser bound. Every test also checks that the split kernel
actually ran (profiler report names conv_x3_kernel), so a silent fallback to fp32 cannot pass.
"""
import ctypes
import json
import os

import numpy as np
import pytest
import torch

from ifd.manifest import make_state_dict
from ifd.topology import FULL

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def maxabs(a, b):
    return float((a.double().cpu() - b.double().cpu()).abs().max())


@pytest.fixture(scope="module")
def x3_model():
    from ifd.model import DiffusionInpaintingModel
    m = DiffusionInpaintingModel(FULL, device=DEV, precision="3xf16")
    m.load_state_dict(make_state_dict(FULL, seed=1))
    return m.eval()


def _kernels_run(model, fn):
    from ifd import _lib
    h = model.handle(DEV)
    L = _lib.lib()
    _lib.check(L.ifd_profile_enable(h.h, 1))
    try:
        out = fn()
        torch.cuda.synchronize()
        buf = ctypes.create_string_buffer(1 << 16)
        _lib.check(L.ifd_profile_report(h.h, buf, len(buf)))
    finally:
        _lib.check(L.ifd_profile_enable(h.h, 0))
    return out, json.loads(buf.value.decode())["kernels"]


def test_x3_precision_switch(x3_model):
    from ifd import _lib
    h = x3_model.handle(DEV)
    v = ctypes.c_int()
    _lib.check(_lib.lib().ifd_get_precision(h.h, ctypes.byref(v)))
    assert v.value == _lib.PRECISIONS["3xf16"]
    with pytest.raises(RuntimeError):
        _lib.check(_lib.lib().ifd_set_precision(h.h, 7))


def test_x3_unet_full(evals, x3_model, record):
    x, gt, mask = (_t(evals[f"full/{k}"]).to(DEV) for k in ("x", "gt", "mask"))
    t = torch.tensor([999], device=DEV)
    with torch.no_grad():
        y, ks = _kernels_run(x3_model, lambda: x3_model(x, t, masked_image=gt * (1 - mask), mask=mask))
    assert any(k.startswith("conv_x3_kernel") for k in ks), sorted(ks)
    err = maxabs(y, _t(evals["full_t999/y"]))
    record("unet_full_t999/3xf16", maxabs=err)
    assert err <= 1e-5


@pytest.mark.parametrize("skip_sep", [8, 0])
def test_x3_skip_launch(evals, x3_model, record, skip_sep):
    """ResBlock skip_connection (code/nn.py:184, added at :212) as its own split-MFMA launch
    (skip_x3_kernel; the default plan runs it at >= 64^2) against the reference output, and against
    the other plans of the same weights: skip_sep=8 runs every skip layer through it (all three
    output-channel tile widths), skip_sep=0 keeps the 1x1 segment fused into conv2's launch."""
    from ifd.model import DiffusionInpaintingModel
    x, gt, mask = (_t(evals[f"full/{k}"]).to(DEV) for k in ("x", "gt", "mask"))
    t = torch.tensor([999], device=DEV)
    m = DiffusionInpaintingModel(FULL, device=DEV, precision="3xf16", options={"skip_sep": skip_sep})
    m.load_state_dict(make_state_dict(FULL, seed=1))
    with torch.no_grad():
        y_def, ks = _kernels_run(x3_model, lambda: x3_model(x, t, masked_image=gt * (1 - mask), mask=mask))
        y, ks2 = _kernels_run(m, lambda: m(x, t, masked_image=gt * (1 - mask), mask=mask))
    assert any(k.startswith("skip_x3_kernel<128,3>") for k in ks), sorted(ks)
    if skip_sep == 8:
        assert {"skip_x3_kernel<128,3>", "skip_x3_kernel<64,3>", "skip_x3_kernel<32,3>"} <= set(ks2), sorted(ks2)
    else:
        assert not any(k.startswith("skip_x3") for k in ks2), sorted(ks2)
    ref = _t(evals["full_t999/y"])
    e_def, e = maxabs(y_def, ref), maxabs(y, ref)
    record(f"unet_full_t999/3xf16/skip_sep{skip_sep}", maxabs=e, maxabs_default_plan=e_def)
    assert e_def <= 1e-5 and e <= 1e-5
    assert maxabs(y, y_def) <= 2e-5


def test_x3_matches_fp32_batch(x3_model):
    """B=3 random inputs (tile counts not a multiple of the grid) at three timesteps: the split
    mode against the fp32 mode of the same weights."""
    from ifd.model import DiffusionInpaintingModel
    g = torch.Generator(device=DEV).manual_seed(11)
    x = torch.randn(3, 3, 256, 256, device=DEV, generator=g)
    gt = torch.rand(3, 3, 256, 256, device=DEV, generator=g) * 2 - 1
    mask = (torch.rand(3, 1, 256, 256, device=DEV, generator=g) > 0.5).float()
    t = torch.tensor([999, 500, 3], device=DEV)
    m32 = DiffusionInpaintingModel(FULL, device=DEV, precision="fp32")
    m32.load_state_dict(make_state_dict(FULL, seed=1))
    with torch.no_grad():
        y3 = x3_model(x, t, masked_image=gt * (1 - mask), mask=mask)
        y32 = m32(x, t, masked_image=gt * (1 - mask), mask=mask)
    assert torch.isfinite(y3).all()
    err = maxabs(y3, y32)
    print(f"3xf16 vs fp32 B=3 maxabs={err:.3g}")
    assert err <= 2e-5
    # images stay independent under the split path as well
    with torch.no_grad():
        y1 = x3_model(x[1:2], t[1:2], masked_image=(gt * (1 - mask))[1:2], mask=mask[1:2])
    assert maxabs(y1, y3[1:2]) <= 2e-5


def test_x3_matches_fp32_batch4(x3_model):
    """B=4: the batch sizes that are a multiple of 4 run the 8x8 layers as tiles of four whole
    images and the attention 1x1s as split-kernel launches; against the fp32 mode, and each image
    against its own B=1 run (the four images of a tile stay independent)."""
    from ifd.model import DiffusionInpaintingModel
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(4, 3, 256, 256, device=DEV, generator=g)
    gt = torch.rand(4, 3, 256, 256, device=DEV, generator=g) * 2 - 1
    mask = (torch.rand(4, 1, 256, 256, device=DEV, generator=g) > 0.5).float()
    t = torch.tensor([999, 640, 120, 7], device=DEV)
    m32 = DiffusionInpaintingModel(FULL, device=DEV, precision="fp32")
    m32.load_state_dict(make_state_dict(FULL, seed=1))
    with torch.no_grad():
        y3, ks = _kernels_run(x3_model, lambda: x3_model(x, t, masked_image=gt * (1 - mask), mask=mask))
        y32 = m32(x, t, masked_image=gt * (1 - mask), mask=mask)
        y1 = x3_model(x[2:3], t[2:3], masked_image=(gt * (1 - mask))[2:3], mask=mask[2:3])
    assert any(k.startswith("conv_x3_kernel") and k.endswith(",8,3>") for k in ks), sorted(ks)
    assert torch.isfinite(y3).all()
    err = maxabs(y3, y32)
    print(f"3xf16 vs fp32 B=4 maxabs={err:.3g}")
    assert err <= 2e-5
    assert maxabs(y1, y3[2:3]) <= 2e-5


def test_x3_invariant_partial_image_tiles():
    """Batch-invariant geometry at B = 5: the 8x8 layers run as four-image tiles at any batch (the last tile
    holds one image; its spare slots recompute that image, conv_x3.hip unit_of). Against the fp32 mode, and
    images 0 and 4 (a full and a partial tile) bit for bit against their own B = 1 runs, which are partial
    tiles of one image."""
    from ifd.model import DiffusionInpaintingModel
    g = torch.Generator(device=DEV).manual_seed(13)
    x = torch.randn(5, 3, 256, 256, device=DEV, generator=g)
    gt = torch.rand(5, 3, 256, 256, device=DEV, generator=g) * 2 - 1
    mask = (torch.rand(5, 1, 256, 256, device=DEV, generator=g) > 0.5).float()
    t = torch.tensor([999, 640, 120, 7, 450], device=DEV)
    mi = DiffusionInpaintingModel(FULL, device=DEV, precision="3xf16", options={"batch_invariant": 1})
    mi.load_state_dict(make_state_dict(FULL, seed=1))
    m32 = DiffusionInpaintingModel(FULL, device=DEV, precision="fp32")
    m32.load_state_dict(make_state_dict(FULL, seed=1))
    mk = gt * (1 - mask)
    with torch.no_grad():
        y, ks = _kernels_run(mi, lambda: mi(x, t, masked_image=mk, mask=mask))
        y32 = m32(x, t, masked_image=mk, mask=mask)
        ys = [mi(x[i:i + 1], t[i:i + 1], masked_image=mk[i:i + 1], mask=mask[i:i + 1]) for i in (0, 4)]
    assert any(k.startswith("conv_x3_kernel") and k.endswith(",8,3>") for k in ks), sorted(ks)
    assert torch.isfinite(y).all()
    err = maxabs(y, y32)
    print(f"3xf16 invariant vs fp32 B=5 maxabs={err:.3g}")
    assert err <= 2e-5
    assert torch.equal(ys[0], y[0:1]) and torch.equal(ys[1], y[4:5])


def test_x3_matches_fp32_bench_batch(x3_model):
    """The bench configuration itself (B=16 at 256x256, the geometry bench.py times: blk_major
    units, four-image 8x8 tiles, split-K 1x1 launches): 3xf16 against fp32 at two timesteps."""
    from ifd.model import DiffusionInpaintingModel
    g = torch.Generator(device=DEV).manual_seed(9)
    x = torch.randn(16, 3, 256, 256, device=DEV, generator=g)
    gt = torch.rand(16, 3, 256, 256, device=DEV, generator=g) * 2 - 1
    mask = (torch.rand(16, 1, 256, 256, device=DEV, generator=g) > 0.5).float()
    t = torch.tensor([999] * 8 + [250] * 8, device=DEV)
    m32 = DiffusionInpaintingModel(FULL, device=DEV, precision="fp32")
    m32.load_state_dict(make_state_dict(FULL, seed=1))
    with torch.no_grad():
        y3 = x3_model(x, t, masked_image=gt * (1 - mask), mask=mask)
        y32 = m32(x, t, masked_image=gt * (1 - mask), mask=mask)
    err = maxabs(y3, y32)
    print(f"3xf16 vs fp32 B=16 maxabs={err:.3g}")
    assert torch.isfinite(y3).all() and err <= 2e-5


@pytest.mark.parametrize("name", ["c1_full_cos10_eta0.9", "c1_full_cos10_eta0"])
def test_x3_script_ddim_full_c1(loops, meta, x3_model, record, name):
    """C1 loops under the split mode, held to the same oracle-envelope bound as the fp32 mode
    (test_gpu_parity.py::test_script_ddim_full_c1)."""
    from test_gpu_parity import _run_script_loop
    cond = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "conditioning.json")))
    env = [v for k, v in cond.items() if k.startswith(name + "/rel1e-05")]
    env_max = max(v["max"] for v in env)
    env_frac = max(v["frac_gt_1e-4"] for v in env)
    env_p999 = max(v["p999"] for v in env)
    lm = meta["loops"][name]
    gt, mask = _t(loops[f"{name}/gt"]), _t(loops[f"{name}/mask"])
    y = _run_script_loop(x3_model, lm, gt, mask)
    d = (y.double().cpu() - _t(loops[f"{name}/y"]).double()).abs().flatten()
    err, p999, frac = float(d.max()), float(d.quantile(0.999)), float((d > 1e-4).double().mean())
    record(f"{name}/3xf16/vs_reference", maxabs=err, p999=p999, frac_gt_1e4=frac)
    assert err <= max(1e-3, env_max) and p999 <= max(1e-4, env_p999) and frac <= max(env_frac, 1e-5)


def _scaled_state_dict(layer="input_blocks.1.0.in_layers.0.", factor=1e5):
    """Manifest weights with one GroupNorm affine scaled so that layer's conv operand reaches
    ~4e5 >> 65504 (the conv weights stay in the split's range)."""
    sd = make_state_dict(FULL, seed=1)
    for k in ("weight", "bias"):
        sd["base_model." + layer + k] = sd["base_model." + layer + k] * factor
    return sd


def test_x3_range_guard_forward(evals, record):
    """guard="sync": an out-of-f16-range operand trips the guard and the forward is recomputed in fp32:
    the 3xf16 model returns exactly the fp32 model's output (code/nn.py:184,212 feed the raw residual
    stream to the 1x1 skip as well; both operand paths are guarded)."""
    from ifd.model import DiffusionInpaintingModel
    sd = _scaled_state_dict()
    m3 = DiffusionInpaintingModel(FULL, device=DEV, precision="3xf16", guard="sync")
    m3.load_state_dict(sd)
    m32 = DiffusionInpaintingModel(FULL, device=DEV, precision="fp32")
    m32.load_state_dict(sd)
    x, gt, mask = (_t(evals[f"full/{k}"]).to(DEV) for k in ("x", "gt", "mask"))
    t = torch.tensor([500], device=DEV)
    with torch.no_grad(), pytest.warns(UserWarning, match="range guard"):
        y3 = m3(x, t, masked_image=gt * (1 - mask), mask=mask)
    with torch.no_grad():
        y32 = m32(x, t, masked_image=gt * (1 - mask), mask=mask)
    record("x3_range_guard/forward", trips=m3.guard_trips, maxabs_vs_fp32=maxabs(y3, y32))
    assert m3.guard_trips == 1
    assert torch.equal(y3, y32)
    assert torch.isfinite(y3).all()


def test_x3_range_guard_lazy(evals):
    """guard="lazy" (opt-in since round 6): forwards never wait on the GPU; a trip is reported by a later forward
    or by guard_check() as a RuntimeError (the flagged outputs are not recomputed), counted once, and the
    guard is re-armed afterwards: in-range forwards of the same model then pass again."""
    from ifd.model import DiffusionInpaintingModel
    x, gt, mask = (_t(evals[f"full/{k}"]).to(DEV) for k in ("x", "gt", "mask"))
    t = torch.tensor([500], device=DEV)
    m3 = DiffusionInpaintingModel(FULL, device=DEV, precision="3xf16", guard="lazy")
    assert m3.guard == "lazy"
    m3.load_state_dict(_scaled_state_dict())
    with torch.no_grad():
        m3(x, t, masked_image=gt * (1 - mask), mask=mask)  # trips; nothing waits here
        with pytest.raises(RuntimeError, match="range guard tripped"):
            for _ in range(3):  # raised by a later forward once the copy has landed, or by the check
                m3(x, t, masked_image=gt * (1 - mask), mask=mask)
            m3.guard_check()
    assert m3.guard_trips == 1
    m3.load_state_dict(make_state_dict(FULL, seed=1))
    with torch.no_grad():
        for _ in range(3):
            m3(x, t, masked_image=gt * (1 - mask), mask=mask)
        m3.guard_check()
    assert m3.guard_trips == 1


def test_x3_range_guard_dropin_script_loop(record):
    """The drop-in default survives a trip: the UNCHANGED reference script loop (bench.script_ddim_pass restates
    code/test_inp_ddim_100.py:470-576: model() once per step, the DDIM update and injection in torch) over a 3xf16
    model whose layer trips the guard at every forward completes, and its output equals the fp32 model's run of
    the same loop bit for bit (the default guard="sync" recomputes each flagged forward in fp32 before returning
    it)."""
    from bench import script_ddim_pass, synth_inputs
    from ifd.model import DiffusionInpaintingModel
    from ifd.schedules import create_gaussian_diffusion
    sd = _scaled_state_dict()
    diff = create_gaussian_diffusion(steps=1000, learn_sigma=True, noise_schedule="cosine")
    gt, mask = synth_inputs(2, 256, seed=7, device=DEV)
    outs = {}
    for prec in ("3xf16", "fp32"):
        m = DiffusionInpaintingModel(FULL, device=DEV, precision=prec)
        m.load_state_dict(sd)
        torch.manual_seed(4)
        with torch.no_grad(), (pytest.warns(UserWarning, match="range guard") if prec == "3xf16"
                               else __import__("contextlib").nullcontext()):
            outs[prec] = script_ddim_pass(m, diff.alphas_cumprod, (2, 3, 256, 256), gt, mask, 5, 0.75, DEV)
        if prec == "3xf16":
            assert m.guard == "sync" and m.guard_trips == 6  # every forward of the 6-step loop (999 .. 0)
    record("x3_range_guard/dropin_script_loop", maxabs_vs_fp32=maxabs(outs["3xf16"], outs["fp32"]))
    assert torch.isfinite(outs["3xf16"]).all()
    assert torch.equal(outs["3xf16"], outs["fp32"])


def test_x3_range_guard_quiet_on_manifest(evals, x3_model):
    """In-range inputs never trip the guard (the bench workload stays on the split kernels)."""
    x, gt, mask = (_t(evals[f"full/{k}"]).to(DEV) for k in ("x", "gt", "mask"))
    before = x3_model.guard_trips
    with torch.no_grad():
        x3_model(x, torch.tensor([999], device=DEV), masked_image=gt * (1 - mask), mask=mask)
    assert x3_model.guard_trips == before


def test_x3_range_guard_loop(record):
    """The fused DDIM loop in 3xf16 with an out-of-range layer: one guard check at the end, the
    RNG rewound and the loop re-run in fp32 -> identical to the fp32 loop for the same seed."""
    from bench import synth_inputs
    from ifd.model import DiffusionInpaintingModel
    from ifd.sampler import InpaintingSampler
    from ifd.schedules import create_gaussian_diffusion
    sd = _scaled_state_dict()
    diff = create_gaussian_diffusion(steps=1000, learn_sigma=True, noise_schedule="cosine")
    gt, mask = synth_inputs(2, 256, seed=7, device=DEV)
    outs = {}
    for prec in ("3xf16", "fp32"):
        m = DiffusionInpaintingModel(FULL, device=DEV, precision=prec)
        m.load_state_dict(sd)
        s = InpaintingSampler(m, diff, ddim_timesteps=4, device=DEV)
        torch.manual_seed(3)
        with torch.no_grad(), (pytest.warns(UserWarning, match="range guard") if prec == "3xf16"
                               else __import__("contextlib").nullcontext()):
            outs[prec] = s.inpainting_ddim_sample_loop(s.model_fn, (2, 3, 256, 256), gt, mask, True, DEV, False, 0.75)
        if prec == "3xf16":
            assert m.guard_trips == 1 and m.precision == "3xf16"
    record("x3_range_guard/loop", maxabs_vs_fp32=maxabs(outs["3xf16"], outs["fp32"]))
    assert torch.equal(outs["3xf16"], outs["fp32"])


def test_x3_deferred_guard_scope(evals, x3_model):
    """deferred_guard(): a caller-driven loop of 3xf16 forwards reads the guard once at the scope's
    exit (no per-forward sync); in-range inputs pass, an out-of-range layer raises at exit."""
    from ifd.model import DiffusionInpaintingModel
    x, gt, mask = (_t(evals[f"full/{k}"]).to(DEV) for k in ("x", "gt", "mask"))
    t = torch.tensor([999], device=DEV)
    with torch.no_grad():
        ref = x3_model(x, t, masked_image=gt * (1 - mask), mask=mask)
        with x3_model.deferred_guard():
            ys = [x3_model(x, t, masked_image=gt * (1 - mask), mask=mask) for _ in range(3)]
    assert all(torch.equal(y, ref) for y in ys)
    m3 = DiffusionInpaintingModel(FULL, device=DEV, precision="3xf16")
    m3.load_state_dict(_scaled_state_dict())
    with torch.no_grad(), pytest.raises(RuntimeError, match="deferred_guard"):
        with m3.deferred_guard():
            m3(x, t, masked_image=gt * (1 - mask), mask=mask)
    assert m3.guard_trips == 1
    # the scope's forwards on a second stream: the entry reset is ordered before them, so the trip is
    # still seen at the exit
    side = torch.cuda.Stream(DEV)
    with torch.no_grad(), pytest.raises(RuntimeError, match="deferred_guard"):
        with m3.deferred_guard():
            with torch.cuda.stream(side):
                m3(x, t, masked_image=gt * (1 - mask), mask=mask)
    assert m3.guard_trips == 2
