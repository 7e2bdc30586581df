"""Training step of the 9-channel inpainting UNet on the HIP library (BASELINE C5).

One iteration of the reference's `train_epoch` (code/train_inpainting.py:15-79):

    losses = diffusion.training_losses(model, images, t, {'masked_image', 'mask'})  (gaussian_diffusion.py:540-614)
    losses['loss'].backward()
    clip_grad_norm_(model.parameters(), 1.0)
    AdamW(lr, weight_decay, betas=(0.9, 0.999)).step()

runs here as `UNetTrainer.train_step`, every tensor operation a libifd kernel (include/ifd_train.h):
q_sample + the known-region injection with the t[0]-keyed, never-cleared GT-noise cache, the UNet
forward in fp32 keeping what the backward needs, the masked eps-MSE and its gradient, the
backward of every module (conv dgrad / wgrad on fp32 MFMA, GroupNorm + scale/shift + SiLU,
up/down-sampling, QKV attention, the embedding MLPs), the global grad-norm clip and a fused AdamW.
PyTorch provides device memory and the stream only; nothing here computes through ATen.

Parameters, gradients and both AdamW moments are four flat fp32 device buffers in the reference's
state_dict order and torch layouts (`state_dict()` returns views with the reference's key names,
`base_model.` prefixed like DiffusionInpaintingModel's). Activations are NHWC.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch

from . import _lib
from .topology import FULL, UNetConfig, layer_plan, state_dict_spec

_c = ctypes
vp, i32, i64, f32 = _c.c_void_p, _c.c_int, _c.c_int64, _c.c_float
TRAIN_EXPORTS = {
    "ifd_tr_pack_conv": (i32, [vp, i32, i32, i32, i32, i32, i32, i32, vp, vp]),
    "ifd_tr_conv_part_floats": (i64, [i32, i32, i32, i32, i32, i32, i32]),
    "ifd_tr_pack_conv_x3": (i32, [vp, i32, i32, i32, i32, i32, i32, vp, vp, vp]),
    "ifd_tr_pack_desc_bytes": (i64, []),
    "ifd_tr_pack_x3_batch": (i32, [vp, i32, i64, vp, vp]),
    "ifd_tr_conv_x3_part_floats": (i64, [i32, i32, i32, i32]),
    "ifd_tr_conv_x3": (i32, [vp, i32, vp, i32, i32, i32, vp, vp, i32, i32, vp, vp, vp, i64, vp, vp]),
    "ifd_tr_conv_x3_taps": (i32, [vp, i32, vp, i32, i32, i32, vp, vp, i32, i32, vp, vp, vp, i64, vp, i32, i32, vp]),
    "ifd_tr_conv1x1_pack_floats": (i64, [i32, i32, i32]),
    "ifd_tr_conv1x1_x3": (i32, [vp, i32, vp, i32, i32, i32, vp, i32, i32, i32, vp, vp, vp, i64, vp, i32, vp]),
    "ifd_tr_gstat_floats": (i64, [i32, i32, i32]),
    "ifd_tr_conv_x3_gstat": (i32, [vp, i32, vp, i32, i32, i32, vp, vp, i32, i32, vp, vp, vp, i64, vp, i32, vp, i64,
                                   vp, vp, i32, vp]),
    "ifd_tr_gn_fwd_gstat": (i32, [vp, i32, i32, i32, vp, vp, vp, i32, i32, vp, i32, vp, i32, f32, vp, vp, vp]),
    "ifd_tr_conv_x3_gn": (i32, [vp, i32, vp, i32, i32, i32, vp, vp, i32, i32, vp, vp, vp, vp, vp, i64, vp, vp, i64,
                                vp, vp, i32, vp]),
    "ifd_tr_conv_gn": (i32, [vp, i32, vp, i32, i32, i32, vp, vp, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, i64,
                             vp]),
    "ifd_tr_conv_wgrad_x3_gn": (i32, [vp, i32, vp, i32, vp, i32, i32, i32, vp, vp, vp, vp, vp, i64, vp, i64, vp, i32,
                                      vp]),
    "ifd_tr_gn_bwd_cat": (i32, [vp, vp, i32, vp, i32, i32, i32, vp, vp, vp, i32, i32, vp, vp, i32, vp, vp, vp, vp, i64,
                                vp, i32, vp, vp]),
    "ifd_tr_gn_slices": (i64, [i32, i32, i32]),
    "ifd_tr_gnb_part_floats": (i64, [i32, i32, i32]),
    "ifd_tr_conv_x3_gnb": (i32, [vp, i32, i32, i32, vp, vp, i32, i32, vp, vp, i64, vp, vp, i32, vp, vp, vp, vp, vp, i32,
                                 i32, vp, i64, _c.POINTER(i32), i32, vp]),
    "ifd_tr_conv_x3_gnb_act": (i32, [vp, i32, i32, i32, vp, vp, i32, i32, vp, vp, i64, vp, vp, i32, vp, vp, vp, vp, vp,
                                     i32, i32, vp, i64, _c.POINTER(i32), vp, i32, vp]),
    "ifd_tr_gn_bwd_from_part": (i32, [vp, vp, i32, vp, i32, i32, i32, vp, vp, vp, i32, i32, vp, vp, i32, vp, i32, vp, vp,
                                      vp, vp, i64, vp, i32, vp, vp]),
    "ifd_tr_gn_coef": (i32, [vp, i32, i32, i32, vp, vp, vp, i32, vp, i32, vp, i32, f32, vp, vp, vp, vp, i64, vp]),
    "ifd_tr_act_apply": (i32, [vp, i32, i32, i32, vp, vp, i32, vp, vp]),
    "ifd_tr_act_resample": (i32, [vp, i32, i32, i32, vp, vp, i32, vp, vp, vp]),
    "ifd_tr_gn_bwd_resampled": (i32, [vp, vp, i32, i32, i32, vp, vp, i32, vp, i32, vp, vp, vp, vp, vp, i32, vp, i64,
                                      vp]),
    "ifd_tr_head_x3_pack_floats": (i64, [i32]),
    "ifd_tr_conv_head_x3": (i32, [vp, i32, i32, i32, vp, i32, vp, vp, vp, vp, vp, vp, vp]),
    "ifd_tr_scale": (i32, [vp, i64, f32, vp]),
    "ifd_tr_conv": (i32, [vp, i32, vp, i32, i32, i32, vp, vp, i32, i32, i32, i32, i32, vp, vp, vp, i64, vp]),
    "ifd_tr_wgrad_part_floats": (i64, [i32, i32, i32, i64, _c.POINTER(i32)]),
    "ifd_tr_conv_wgrad": (i32, [vp, i32, vp, i32, vp, i32, i32, i32, i32, vp, vp, vp, i64, vp, i64, vp]),
    "ifd_tr_conv_wgrad_x3": (i32, [vp, i32, vp, i32, vp, i32, i32, i32, i32, vp, vp, vp, i64, vp, i64, vp, i32, vp]),
    "ifd_tr_gn_fwd": (i32, [vp, i32, i32, i32, vp, vp, vp, i32, i32, vp, vp, vp, i64, vp]),
    "ifd_tr_gn_bwd": (i32, [vp, vp, i32, i32, i32, vp, vp, vp, i32, i32, vp, vp, i32, vp, vp, vp, vp, i64, vp]),
    "ifd_tr_resample": (i32, [vp, i32, i32, i32, i32, vp, vp]),
    "ifd_tr_resample_bwd": (i32, [vp, i32, i32, i32, i32, vp, i32, vp]),
    "ifd_tr_add": (i32, [vp, vp, vp, i64, vp]),
    "ifd_tr_copy_channels": (i32, [vp, i32, i32, vp, i32, i32, i32, i64, i32, vp]),
    "ifd_tr_attention": (i32, [vp, i32, i32, i32, f32, vp, vp]),
    "ifd_tr_attention_bwd_scratch_floats": (i64, [i32, i32, i32]),
    "ifd_tr_attention_bwd": (i32, [vp, vp, i32, i32, i32, f32, vp, vp, i64, vp]),
    "ifd_tr_linear": (i32, [vp, i32, i32, vp, vp, i32, i32, i32, vp, vp]),
    "ifd_tr_linear_bwd": (i32, [vp, vp, i32, i32, vp, i32, i32, vp, i32, vp, vp, vp]),
    "ifd_tr_silu_bwd": (i32, [vp, vp, vp, i64, vp]),
    "ifd_tr_temb": (i32, [vp, vp, i32, i32, vp, vp]),
    "ifd_tr_pack_input": (i32, [vp, vp, vp, i32, i32, vp, vp]),
    "ifd_tr_q_sample_inject": (i32, [vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, vp, vp]),
    "ifd_tr_masked_mse": (i32, [vp, i32, vp, vp, i32, i32, vp, vp, vp, vp]),
    "ifd_tr_clip_adamw": (i32, [vp, vp, vp, vp, i64, f32] + [ctypes.c_double] * 5 + [i32, vp, vp, vp]),
}

_bound = None


def lib():
    global _bound
    L = _lib.lib()
    if _bound is not L:
        for name, (res, args) in TRAIN_EXPORTS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _bound = L
    return L


def P(t):
    return None if t is None else _c.c_void_p(t.data_ptr())


def chk(rc):
    _lib.check(rc)


def _bn(cout):
    return 64 if cout % 64 == 0 else 32


def _pad(v, m):
    return (v + m - 1) // m * m


class UNetTrainer:
    """fp32 training of the 9-channel UNet (code/unet.py:14-200) with the reference's loss, clip and AdamW.

    precision="3xf16": the 3x3 convs of the forward (and, with x3_dgrad, the dgrad convs of the backward)
    run on the sampler's fp32-accurate split kernel (conv_x3.hip: each fp32 operand = f16 hi + f16 lo,
    three f16 MFMA products per MAC, fp32 accumulation); with x3_wgrad their weight gradients run on
    wgrad_x3_kernel (both operands split on the fly, same arithmetic). The backward then carries a loss scale of
    2^x3_loss_scale_log2 (the eps-MSE gradient is ~1e-7 per element: below f16's normal range unscaled);
    every backward op is linear in the upstream gradient and the scale is a power of two, so removing it
    from the parameter gradients before clip + AdamW is exact. A split operand outside f16's range sets
    the range guard; the step is then recomputed in fp32 (same noise) with a warning. GroupNorm, attention,
    embeddings and the optimizer stay fp32.

    precision="f16": the reduced-precision variant of the same path (BASELINE configs[4] names a bf16 fine-tune,
    which the reference has no code for): the split kernels with ONE product per MAC (f16 operands, fp32
    accumulation) for the forward, dgrad and weight-gradient convs, the same loss scale and range guard.
    Not fp32-class: reported separately, checked against the fp32 step at a stated tolerance
    (tests/test_gpu_train.py::test_train_f16_full_vs_fp32).

    fuse_gn (split modes): the GroupNorm + SiLU in front of a 3x3 conv (ResBlock in_layers / out_layers,
    the output head) is not materialised: ifd_tr_gn_coef gives per-(image, channel) coefficients A, B,
    the forward conv applies silu(A x + B) to the raw input on load (the sampler's prologue) and the
    weight gradient recomputes it at staging (ifd_tr_conv_wgrad_x3_gn). Shapes a kernel does not take
    materialise the activation (ifd_tr_act_apply) and run the plain path.

    fuse_gnb (split modes): the dgrad conv whose output feeds a GroupNorm backward (ResBlock out_layers.3 ->
    out_layers.0, in_layers.2 -> in_layers.0 without resampling) computes that backward's pass-1 partial sums in
    its epilogue (ifd_tr_conv_x3_gnb): the pass over (dout, x) of ifd_tr_gn_bwd is not run.

    gnb_act (with fuse_gnb, round 6, off by default): that epilogue also writes the GroupNorm's forward output
    silu(z) — the input of the conv whose weight gradient is next (ifd_tr_conv_x3_gnb_act) — so that weight
    gradient runs the plain split kernel on it instead of re-applying GroupNorm + SiLU on load (1.82 vs 1.66 ms
    at the 256^2 128 -> 128 layer alone, profiles/r06e); the dgrad then runs first. Measured in the whole step
    it is a wash (profiles/r06g): the weight gradients gain 0.85 ms per step, the GNB dgrads lose 0.95 ms to the
    extra stores (242.7 / 243.6 vs 243.4 / 242.9 images/s off / on)."""

    SPLIT_MODES = ("3xf16", "f16")

    def __init__(self, cfg: UNetConfig = FULL, device="cuda", lr=5e-5, weight_decay=0.01, betas=(0.9, 0.999),
                 eps=1e-8, max_norm=1.0, precision="fp32", x3_dgrad=True, x3_wgrad=True, x3_loss_scale_log2=20,
                 fuse_gn=True, fuse_gnb=True, gnb_act=False):
        if precision not in ("fp32", "3xf16", "f16"):
            raise ValueError(f"precision must be 'fp32', '3xf16' or 'f16', got {precision!r}")
        self.precision = precision
        self.x3_dgrad = bool(x3_dgrad)
        self.x3_wgrad = bool(x3_wgrad)
        self.x3_loss_scale_log2 = int(x3_loss_scale_log2)
        self.fuse_gn = bool(fuse_gn)
        self.fuse_gnb = bool(fuse_gnb)
        self.gnb_act = bool(gnb_act)
        self.guard_trips = 0
        self.cfg = cfg
        self.dev = torch.device(device)
        self.lr, self.wd, self.betas, self.eps, self.max_norm = lr, weight_decay, betas, eps, max_norm
        self.spec = state_dict_spec(cfg, prefix="")
        self.offsets = {}
        n = 0
        for k, shape in self.spec:
            self.offsets[k] = (n, tuple(shape))
            n += int(np.prod(shape))
        self.numel = n
        z = lambda: torch.zeros(n, device=self.dev, dtype=torch.float32)  # noqa: E731
        self.flat, self.grad, self.m, self.v = z(), z(), z(), z()
        self.step_count = 0
        self.norm_coef = torch.zeros(2, device=self.dev)
        self.loss = torch.zeros(1, device=self.dev)
        self._gt_noise_cache = {}
        # timestep_embedding frequencies exactly as the reference builds them (code/nn.py:54-56)
        half = cfg.model_channels // 2
        self.freqs = torch.exp(-math.log(10000) * torch.arange(0, half, dtype=torch.float32) / half).to(self.dev)
        self._zero_bias = torch.zeros(4096, device=self.dev)
        self.plan = layer_plan(cfg)
        self.emb_dim = 4 * cfg.model_channels
        self.s = None  # stream pointer (set per call)
        self._guard = torch.zeros(4, device=self.dev, dtype=torch.int32)
        self._grad_clean = False
        self._pack_cache = {}
        # the split kernels' packed weights, kept across steps: every step re-packs them all in one launch at
        # the start of the forward (_repack_all); a pack first needed mid-step is packed alone and joins the table
        self._pack_persist = {}
        self._pack_table = None
        # GroupNorm granule statistics of forward activations, keyed by data_ptr: (tensor, stats, E, cnt,
        # channels, second-source stats). Valid only while the tensor holds what its producing conv wrote:
        # the `is` check guards against a reused address, and every in-place write to a tensor (the
        # accumulating add_ / copy_ch / gn_bwd / resample_bwd paths) drops its entry (_dirty).
        self._gstat = {}

    def _dirty(self, t):
        """`t` is about to be written in place: its recorded statistics no longer describe it."""
        if t is not None and self._gstat:
            self._gstat.pop(t.data_ptr(), None)

    # ------------------------------------------------------------------ parameters
    def p(self, name):
        o, shape = self.offsets[name]
        return self.flat[o:o + int(np.prod(shape))].view(shape)

    def g(self, name):
        o, shape = self.offsets[name]
        return self.grad[o:o + int(np.prod(shape))].view(shape)

    def load_state_dict(self, sd):
        sd = {(k[len("base_model."):] if k.startswith("base_model.") else k): v for k, v in sd.items()}
        missing = [k for k, _ in self.spec if k not in sd]
        if missing:
            raise KeyError(f"missing parameters: {missing[:4]}...")
        with torch.no_grad():
            for k, _ in self.spec:
                self.p(k).copy_(sd[k].to(self.dev, torch.float32))

    def state_dict(self, prefix="base_model."):
        return {prefix + k: self.p(k) for k, _ in self.spec}

    def grads(self, prefix="base_model."):
        return {prefix + k: self.g(k) for k, _ in self.spec}

    # ------------------------------------------------------------------ op wrappers
    def _empty(self, *shape):
        return torch.empty(*shape, device=self.dev, dtype=torch.float32)

    def _zeros(self, *shape):
        return torch.zeros(*shape, device=self.dev, dtype=torch.float32)

    def _packed(self, name, transpose):
        """Device packing of conv weight `name` for the forward (transpose 0) or dgrad (1) conv."""
        w = self.p(name)
        cout, cin = w.shape[0], w.shape[1]
        taps = int(np.prod(w.shape[2:])) if w.dim() > 2 else 1
        pout, pin = (cout, cin) if not transpose else (cin, cout)
        bn = _bn(pout)
        cin_pad, cout_pad = _pad(pin, 8), _pad(pout, bn)
        key = (name, transpose)
        buf = self._pack_cache.get(key)
        if buf is None:
            buf = self._empty(cout_pad * cin_pad * taps)
            chk(lib().ifd_tr_pack_conv(P(w), cout, cin, taps, bn, cin_pad, cout_pad, transpose, P(buf), self.s))
            self._pack_cache[key] = buf
        return buf, pout, pin, taps, bn, cin_pad, cout_pad

    def _x3_pack(self, name, cout, cin, taps, pad, cout_pad, transpose):
        """The split kernel's packing of conv weight `name` (ifd_tr_pack_conv_x3) in a buffer kept across steps."""
        key = (name, int(transpose), taps, pad, cout_pad)
        buf = self._pack_persist.get(key)
        if buf is None:
            buf = self._empty(cout_pad * pad * taps)
            self._pack_persist[key] = buf
            self._pack_table = None
        chk(lib().ifd_tr_pack_conv_x3(P(self.p(name)), cout, cin, taps, pad, cout_pad, int(transpose), P(buf),
                                      P(self._guard), self.s))
        return buf

    _PACK_DESC = np.dtype([("w", "<u8"), ("dst", "<u8"), ("cout", "<i4"), ("cin", "<i4"), ("pad", "<i4"),
                           ("cout_pad", "<i4"), ("transpose", "<i4"), ("taps", "<i4"), ("block0", "<i8")])

    def _repack_all(self):
        """Start of a forward: this step's weights into every kept split-kernel packing, one launch
        (ifd_tr_pack_x3_batch; was ~170 launches a step). The forward's lookups then find them packed."""
        self._pack_cache = {}
        if not (self._pack_persist and self._split()):
            return
        if self._pack_table is None:
            if lib().ifd_tr_pack_desc_bytes() != self._PACK_DESC.itemsize:  # (not an assert: kept under python -O)
                raise RuntimeError("ifd_tr_pack_x3_batch descriptor layout differs from train.py's _PACK_DESC")
            recs = np.zeros(len(self._pack_persist), dtype=self._PACK_DESC)
            nb = 0
            for i, ((name, tr, taps, pad, cout_pad), buf) in enumerate(self._pack_persist.items()):
                w = self.p(name)
                cout, cin = w.shape[0], w.shape[1]
                n = (cout_pad // 64) * (pad // 16) * 9 * 2 * 64 * 8 if taps == 9 else \
                    (cout_pad // 64) * (pad // 32) * 2 * 2 * 64 * 8
                recs[i] = (w.data_ptr(), buf.data_ptr(), cout, cin, pad, cout_pad, tr, taps, nb)
                nb += (n + 8191) // 8192  # 256 threads x 32 elements per block (ifd_train.h)
            self._pack_table = (torch.from_numpy(recs.view(np.uint8)).to(self.dev), len(recs), nb)
        t, n, nb = self._pack_table
        chk(lib().ifd_tr_pack_x3_batch(P(t), n, nb, P(self._guard), self.s))
        for (name, tr, taps, pad, cout_pad), buf in self._pack_persist.items():
            self._pack_cache[(name, tr, "x3")] = buf

    def _split(self):
        return self.precision in self.SPLIT_MODES

    def _nprod(self):
        return 1 if self.precision == "f16" else 3

    def _x3_active(self, transpose):
        return self._split() and (not transpose or self.x3_dgrad)

    def _conv_x3(self, x, cin_x, N, H, name, bias_name, res, x1, c1, transpose, gn=None):
        """The conv on the 3xf16 split kernel, or None when its shape is not eligible (fp32 kernel then).
        gn = (A, B): x is the raw GroupNorm input, silu(A x + B) applied on load (3x3 only)."""
        w = self.p(name)
        taps = int(np.prod(w.shape[2:])) if w.dim() > 2 else 1
        if taps not in (1, 9) or (gn is not None and taps != 9):
            return None
        cout, cin = w.shape[0], w.shape[1]
        pout, pin = (cout, cin) if not transpose else (cin, cout)
        nct = pout // 64
        # a 3x3 conv whose 64-channel tile count is not a power of two (the dgrad of the output blocks'
        # concat convs: 384 = 6 x 64, 768 = 12 x 64 output channels) runs padded to the next power of two
        # (zero weight rows) into a scratch tensor and is copied out: the split kernel decodes its
        # channel tiles by shifts
        ppad = pout
        if taps == 9 and pout % 64 == 0 and nct & (nct - 1) and res is None and not bias_name:
            ppad = 64 * (1 << (nct - 1).bit_length())
        if taps == 9 and (pout % 64 or cin_x + c1 != _pad(pin, 16) or cin_x % 16 or c1 % 16):
            return None
        if taps == 9 and (ppad // 64) & (ppad // 64 - 1):
            return None
        if taps == 1 and (pout % 64 or cin_x + c1 != pin or cin_x % 32 or c1 % 32):
            return None
        cin_pad = cin_x + c1
        key = (name, int(transpose), "x3")
        wx3 = self._pack_cache.get(key)
        if wx3 is None:
            wx3 = self._x3_pack(name, cout, cin, taps, cin_pad, ppad, transpose)
            self._pack_cache[key] = wx3
        b = self.p(bias_name) if bias_name else self._zero_bias
        out = self._empty(N, H, H, ppad)
        pf = lib().ifd_tr_conv_x3_part_floats(N, H, cin_pad, ppad)
        part = self._empty(max(pf, 1))
        want_stats = not transpose and ppad == pout and pout % 128 == 0
        if gn is not None:
            if ppad != pout:
                return None
            # forward convs also hand the following GroupNorm its statistics (granules from the epilogue)
            gf = lib().ifd_tr_gstat_floats(N, H, pout) if want_stats else 0
            gstat = self._empty(max(gf, 1))
            E, cnt = _c.c_int(0), _c.c_float(0.0)
            rc = lib().ifd_tr_conv_x3_gn(P(x), cin_x, P(x1), c1, N, H, P(wx3), P(b), cin_pad, ppad, P(gn[0]),
                                         P(gn[1]), P(res), P(out), P(part), pf, P(self._guard),
                                         P(gstat) if want_stats else None, gf, _c.byref(E), _c.byref(cnt),
                                         self._nprod(), self.s)
            if rc == 0 and E.value > 0:
                self._gstat[out.data_ptr()] = (out, gstat, E.value, cnt.value, pout, None)
        elif want_stats:
            gf = lib().ifd_tr_gstat_floats(N, H, pout)
            gstat = self._empty(gf)
            E, cnt = _c.c_int(0), _c.c_float(0.0)
            rc = lib().ifd_tr_conv_x3_gstat(P(x), cin_x, P(x1), c1, N, H, P(wx3), P(b), cin_pad, ppad, P(res), P(out),
                                            P(part), pf, P(self._guard), taps, P(gstat), gf, _c.byref(E),
                                            _c.byref(cnt), self._nprod(), self.s)
            if rc == 0 and E.value > 0:
                self._gstat[out.data_ptr()] = (out, gstat, E.value, cnt.value, pout, None)
        else:
            rc = lib().ifd_tr_conv_x3_taps(P(x), cin_x, P(x1), c1, N, H, P(wx3), P(b), cin_pad, ppad, P(res), P(out),
                                           P(part), pf, P(self._guard), taps, self._nprod(), self.s)
        if rc == 3:
            return None
        chk(rc)
        if ppad != pout:
            real = self._empty(N, H, H, pout)
            self.copy_ch(out, ppad, 0, real, pout, 0, pout, N * H * H, False)
            out = real
        return out

    def _head_x3(self, x, cin, N, H, gn):
        """The output head's conv (GroupNorm + SiLU on load) on the split head kernel, NHWC [N,H,H,8];
        shapes it does not take run conv() (the fp32 kernel with the same prologue)."""
        w = self.p("out.2.weight")
        if self.precision == "3xf16" and w.shape[0] <= 8:
            wp = self._empty(max(lib().ifd_tr_head_x3_pack_floats(cin), 1))
            b8 = self._zeros(8)
            b8[:w.shape[0]].copy_(self.p("out.2.bias"))
            out = self._empty(N, H, H, 8)
            rc = lib().ifd_tr_conv_head_x3(P(x), cin, N, H, P(w), w.shape[0], P(wp), P(b8), P(gn[0]), P(gn[1]), P(out),
                                           P(self._guard), self.s)
            if rc != 3:
                chk(rc)
                return out
        return self.conv(x, cin, N, H, "out.2.weight", "out.2.bias", gn=gn)

    # the dedicated split 1x1 kernel from this resolution up (the sampler's skip_sep threshold: below it the split
    # conv kernel's 1x1 chunks keep more of the chip busy)
    CONV1X1_MIN_H = 64

    def _conv1x1_x3(self, x, cin_x, N, H, name, bias_name, res, x1, c1, transpose, gn):
        """A 1x1 conv (skip_connection forward / dgrad) without residual or prologue on ifd_tr_conv1x1_x3
        (skip_x3.hip, weights packed on the device each call); None when it does not take the shape."""
        w = self.p(name)
        if w.dim() != 4 or tuple(w.shape[2:]) != (1, 1) or res is not None or gn is not None or H < self.CONV1X1_MIN_H:
            return None
        cout, cin = w.shape[0], w.shape[1]
        co = cin if transpose else cout
        if cin_x + c1 != (cout if transpose else cin) or co % 4:
            return None
        wp = self._empty(max(lib().ifd_tr_conv1x1_pack_floats(cout, cin, int(transpose)), 1))
        b = self.p(bias_name) if bias_name else self._zero_bias
        out = self._empty(N, H, H, co)
        rc = lib().ifd_tr_conv1x1_x3(P(x), cin_x, P(x1), c1, N, H, P(w), cout, cin, int(transpose), P(b), P(out), P(wp),
                                     wp.numel(), P(self._guard), self._nprod(), self.s)
        if rc == 3:
            return None
        chk(rc)
        return out

    def conv(self, x, cin_x, N, H, name, bias_name=None, res=None, x1=None, c1=0, transpose=False, gn=None):
        """NHWC conv of concat(x[cin_x], x1[c1]) with weight `name` (forward or, transposed, dgrad).
        Output channels are padded to a multiple of 4 (zero weight rows): the 6-channel head writes 8.
        gn = (A, B): the conv's input is silu(A x + B) of the raw x (fuse_gn), applied on load."""
        if self._x3_active(transpose):
            out = self._conv1x1_x3(x, cin_x, N, H, name, bias_name, res, x1, c1, transpose, gn)
            if out is None:
                out = self._conv_x3(x, cin_x, N, H, name, bias_name, res, x1, c1, transpose, gn=gn)
            if out is not None:
                return out
        buf, pout, pin, taps, bn, cin_pad, cout_pad = self._packed(name, int(transpose))
        if cin_x + c1 != cin_pad:
            raise ValueError(f"{name}: input channels {cin_x}+{c1} != packed {cin_pad}")
        real = pout
        pout = _pad(pout, 4)
        out = self._empty(N, H, H, pout)
        b = self.p(bias_name) if bias_name else self._zero_bias
        if bias_name and real != pout:
            b = self._zeros(pout)
            b[:real].copy_(self.p(bias_name))
        pf = lib().ifd_tr_conv_part_floats(N, H, cin_pad, pout, cout_pad, bn, taps)
        part = self._empty(max(pf, 1))
        if gn is not None:
            chk(lib().ifd_tr_conv_gn(P(x), cin_x, P(x1), c1, N, H, P(buf), P(b), cin_pad, pout, cout_pad, bn, taps,
                                     P(gn[0]), P(gn[1]), P(res), P(out), P(part), pf, self.s))
            return out
        chk(lib().ifd_tr_conv(P(x), cin_x, P(x1), c1, N, H, P(buf), P(b), cin_pad, pout, cout_pad, bn, taps, P(res),
                              P(out), P(part), pf, self.s))
        return out

    def wgrad(self, dy, cout, x, cin_x, N, H, name, bias_name=None, real_cin=None, gn=None, x1=None, c1=0):
        """grad[name] += conv weight gradient; grad[bias] += column sums of dy. The input is concat(x[cin_x],
        x1[c1]) (the output blocks' skip concat, never materialised).
        gn = (A, B): the forward conv's input was silu(A x + B) of the raw x (recomputed at staging, or
        materialised here when the split kernel does not take the shape)."""
        w = self.p(name)
        taps = int(np.prod(w.shape[2:])) if w.dim() > 2 else 1
        P_ = N * H * H
        cin = cin_x + c1
        S = _c.c_int()
        need = lib().ifd_tr_wgrad_part_floats(cout, cin, taps, P_, _c.byref(S))
        part = self._empty(need)
        # one row per split too, so the split kernels always fuse the bias column sums (a separate column-sum
        # pass over dy at 8^2 ran 16 blocks for 61 us)
        colpart = self._empty(max((P_ + 1023) // 1024, S.value) * cout)
        real_cin = real_cin or w.shape[1]
        real_cout = w.shape[0]
        direct = real_cin == cin and real_cout == cout
        dw = self.g(name) if direct else self._zeros(cout * cin * taps)
        db = self.g(bias_name) if (bias_name and real_cout == cout) else (self._zeros(cout) if bias_name else None)
        rc = 3
        if gn is not None and self._split() and self.x3_wgrad and taps == 9:
            rc = lib().ifd_tr_conv_wgrad_x3_gn(P(dy), cout, P(x), cin_x, P(x1), c1, N, H, P(gn[0]), P(gn[1]), P(dw),
                                               P(db), P(part), need, P(colpart), colpart.numel(), P(self._guard),
                                               self._nprod(), self.s)
        if rc != 3:
            chk(rc)
        else:
            if gn is not None:  # the split kernel does not take this shape: materialise the activation
                if x1 is not None:
                    x, cin_x, x1, c1 = self._cat(x, cin_x, x1, c1, N * H * H), cin, None, 0
                x = self.act_apply(x, N, H * H, cin_x, gn)
            self._wgrad_plain(dy, cout, x, cin_x, x1, c1, N, H, taps, dw, db, part, need, colpart)
        if not direct:  # padded input (the first conv reads 16 channels, 9 real) or output (head: 8, 6 real)
            chk(lib().ifd_tr_copy_channels(P(dw), cin * taps, 0, P(self.g(name)), real_cin * taps, 0, real_cin * taps,
                                           real_cout, 1, self.s))
        if bias_name and real_cout != cout:
            chk(lib().ifd_tr_copy_channels(P(db), cout, 0, P(self.g(bias_name)), real_cout, 0, real_cout, 1, 1, self.s))

    def _wgrad_plain(self, dy, cout, x, cin_x, x1, c1, N, H, taps, dw, db, part, need, colpart):
        if self._split() and self.x3_wgrad:
            chk(lib().ifd_tr_conv_wgrad_x3(P(dy), cout, P(x), cin_x, P(x1), c1, N, H, taps, P(dw), P(db), P(part), need,
                                           P(colpart), colpart.numel(), P(self._guard), self._nprod(), self.s))
        else:
            chk(lib().ifd_tr_conv_wgrad(P(dy), cout, P(x), cin_x, P(x1), c1, N, H, taps, P(dw), P(db), P(part), need,
                                        P(colpart), colpart.numel(), self.s))

    def _cat(self, x, cx, x1, c1, npix):
        """concat(x[cx], x1[c1]) materialised (the paths that cannot read the two sources)."""
        cat = self._empty(npix * (cx + c1))
        self.copy_ch(x, cx, 0, cat, cx + c1, 0, cx, npix, False)
        self.copy_ch(x1, c1, 0, cat, cx + c1, cx, c1, npix, False)
        return cat

    def gn_fwd(self, x, N, HW, C, prefix, ss=None, ss_stride=0, silu=True):
        out = self._empty(N * HW * C)
        stats = self._empty(N * 64)
        g = self._gstat.get(x.data_ptr())
        if g is not None and g[0] is x and C % 128 == 0:  # statistics from the producing conv(s)' granules
            chk(lib().ifd_tr_gn_fwd_gstat(P(x), N, HW, C, P(self.p(prefix + "weight")), P(self.p(prefix + "bias")),
                                          P(ss), ss_stride, int(silu), P(g[1]), g[4], P(g[5]), g[2], g[3], P(out),
                                          P(stats), self.s))
            return out, stats
        nsl = lib().ifd_tr_gn_slices(HW, N, C)
        work = torch.empty(N * nsl * 64, device=self.dev, dtype=torch.float64)
        chk(lib().ifd_tr_gn_fwd(P(x), N, HW, C, P(self.p(prefix + "weight")), P(self.p(prefix + "bias")), P(ss),
                                ss_stride, int(silu), P(out), P(stats), P(work), work.numel(), self.s))
        return out, stats

    def _gn_fused(self):
        return self.fuse_gn and self._split()

    def _granules2(self, x, x1):
        """The producing convs' granule statistics of concat(x, x1) as one record, or None."""
        ga, gb = self._gstat.get(x.data_ptr()), self._gstat.get(x1.data_ptr())
        if (ga is not None and gb is not None and ga[0] is x and gb[0] is x1 and ga[5] is None and gb[5] is None
                and ga[2:4] == gb[2:4]):
            return (None, ga[1], ga[2], ga[3], ga[4], gb[1])
        return None

    def gn_coef(self, x, N, HW, C, prefix, ss=None, ss_stride=0, x1=None):
        """(A, B), stats of GroupNorm + scale/shift for a consumer that applies silu(A x + B) on load.
        x1: the concat's second source (granule statistics of both are required)."""
        A, B = self._empty(N, C), self._empty(N, C)
        stats = self._empty(N * 64)
        g = self._granules2(x, x1) if x1 is not None else self._gstat.get(x.data_ptr())
        if x1 is not None:
            if g is None or C % 128 != 0:  # explicit (not an assert: `python -O` must not reach the wrong memory)
                raise RuntimeError("ifd.train: a concat GroupNorm on load needs both sources' granule statistics "
                                   "and C % 128 == 0")
            g = (x,) + g[1:]
        gam, bet = self.p(prefix + "weight"), self.p(prefix + "bias")
        if g is not None and g[0] is x and C % 128 == 0:
            chk(lib().ifd_tr_gn_coef(None, N, HW, C, P(gam), P(bet), P(ss), ss_stride, P(g[1]), g[4], P(g[5]), g[2],
                                     g[3], P(stats), P(A), P(B), None, 0, self.s))
        else:
            nsl = lib().ifd_tr_gn_slices(HW, N, C)
            work = torch.empty(N * nsl * 64, device=self.dev, dtype=torch.float64)
            chk(lib().ifd_tr_gn_coef(P(x), N, HW, C, P(gam), P(bet), P(ss), ss_stride, None, 0, None, 0, 0.0,
                                     P(stats), P(A), P(B), P(work), work.numel(), self.s))
        return (A, B), stats

    def act_apply(self, x, N, HW, C, gn, silu=True):
        out = self._empty(N * HW * C)
        chk(lib().ifd_tr_act_apply(P(x), N, HW, C, P(gn[0]), P(gn[1]), int(silu), P(out), self.s))
        return out

    @staticmethod
    def _addend(add):
        """add = (tensor, stride, channel offset) -> (pointer, stride) for the GroupNorm backward's dx addend."""
        if add is None:
            return None, 0
        t, stride, off = add
        return _c.c_void_p(t.data_ptr() + 4 * off), stride

    def gn_bwd(self, dout, x, N, HW, C, prefix, stats, dx=None, ss=None, ss_stride=0, dss=None, silu=True, x1=None,
               C0=None, add=None, split=None):
        """x1, C0: the GroupNorm input is concat(x[C0], x1[C - C0]) (read by channel range). add = (t, stride,
        offset): dx also gets that channel range of t (ifd_tr_gn_bwd_cat). split = (d0, d1): the gradient is
        written per concat source, d0 [.., C0] and d1 [.., C - C0] (returned as that pair; dx must be None)."""
        dx, dx1, acc = self._gn_bwd_out(dx, split, N * HW * C)
        nsl = lib().ifd_tr_gn_slices(HW, N, C)
        work = self._empty(N * nsl * C * 3 + N * C * 3 + N * 64)
        chk(lib().ifd_tr_gn_bwd_cat(P(dout), P(x), C0 if x1 is not None else C, P(x1), N, HW, C,
                                    P(self.p(prefix + "weight")), P(self.p(prefix + "bias")), P(ss), ss_stride,
                                    int(silu), P(stats), P(dx), int(acc), P(self.g(prefix + "weight")),
                                    P(self.g(prefix + "bias")), P(dss), P(work), work.numel(), *self._addend(add),
                                    P(dx1), self.s))
        return (dx, dx1) if split is not None else dx

    def _gn_bwd_out(self, dx, split, numel):
        """The GroupNorm backward's output: (dx, dx1, accumulate) for dx = given (+=), a split pair, or fresh."""
        if split is not None:
            if dx is not None:
                raise ValueError("gn_bwd: a split output does not accumulate")
            for t in split:
                self._dirty(t)
            return split[0], split[1], False
        if dx is None:
            return self._empty(numel), None, False
        self._dirty(dx)
        return dx, None, True

    def dgrad_gn_bwd(self, dy, cdy, N, H, wname, x, C, prefix, stats, dx=None, ss=None, ss_stride=0, dss=None,
                     silu=True, x1=None, C0=None, add=None, split=None, act_sink=None):
        """gn_bwd(conv^T(dy)) - the dgrad of conv `wname` fed into the GroupNorm backward of its input x (C
        channels; x1 / C0 as gn_bwd). On the split kernel the GroupNorm's pass 1 runs in the dgrad's epilogue
        (ifd_tr_conv_x3_gnb); shapes it does not take run conv() then gn_bwd(). act_sink (a list): on the fused
        path the epilogue also writes the GroupNorm's forward output silu(GN(x)(1 + s) + shift), [N, H, H, C], and
        appends it (round 6: the next weight gradient then reads it instead of re-applying GN + SiLU on load)."""
        out = self._dgrad_gnb(dy, cdy, N, H, wname, x, C, prefix, stats, dx, ss, ss_stride, dss, silu, x1, C0, add,
                              split, act_sink)
        if out is not None:
            return out
        da = self.conv(dy, cdy, N, H, wname, transpose=True)
        return self.gn_bwd(da, x, N, H * H, C, prefix, stats, dx=dx, ss=ss, ss_stride=ss_stride, dss=dss, silu=silu,
                           x1=x1, C0=C0, add=add, split=split)

    def _dgrad_gnb(self, dy, cdy, N, H, wname, x, C, prefix, stats, dx, ss, ss_stride, dss, silu, x1, C0, add=None,
                   split=None, act_sink=None):
        if not (self.fuse_gnb and self._x3_active(True)):
            return None
        w = self.p(wname)
        if w.dim() != 4 or tuple(w.shape[2:]) != (3, 3):
            return None
        cout, cin = w.shape[0], w.shape[1]  # the dgrad maps cout -> cin channels
        if cin != C or cin % 64 or ((cin // 64) & (cin // 64 - 1)) or cdy != _pad(cout, 16) or cdy % 16:
            return None
        key = (wname, 1, "x3")
        wx3 = self._pack_cache.get(key)
        if wx3 is None:
            wx3 = self._x3_pack(wname, cout, cin, 9, cdy, cin, 1)
            self._pack_cache[key] = wx3
        da = self._empty(N, H, H, cin)
        pf = lib().ifd_tr_conv_x3_part_floats(N, H, cdy, cin)
        part = self._empty(max(pf, 1))
        gpf = lib().ifd_tr_gnb_part_floats(N, H, cin)
        gpart = self._empty(gpf)
        nsl = _c.c_int(0)
        c0 = C0 if x1 is not None else C
        gam, bet = self.p(prefix + "weight"), self.p(prefix + "bias")
        act = self._empty(N, H, H, cin) if act_sink is not None and self.gnb_act else None
        rc = lib().ifd_tr_conv_x3_gnb_act(P(dy), cdy, N, H, P(wx3), P(self._zero_bias), cdy, cin, P(da), P(part), pf,
                                          P(self._guard), P(x), c0, P(x1), P(stats), P(gam), P(bet), P(ss), ss_stride,
                                          int(silu), P(gpart), gpf, _c.byref(nsl), P(act), self._nprod(), self.s)
        if rc == 3:
            return None
        chk(rc)
        if act is not None and nsl.value > 0:
            act_sink.append(act)
        if nsl.value == 0:  # (the conv ran; its geometry could not carry the partial sums)
            return self.gn_bwd(da, x, N, H * H, C, prefix, stats, dx=dx, ss=ss, ss_stride=ss_stride, dss=dss,
                               silu=silu, x1=x1, C0=C0, add=add, split=split)
        dx, dx1, acc = self._gn_bwd_out(dx, split, N * H * H * C)
        work = self._empty(N * C * 3 + N * 64)
        chk(lib().ifd_tr_gn_bwd_from_part(P(da), P(x), c0, P(x1), N, H * H, C, P(gam), P(bet), P(ss), ss_stride,
                                          int(silu), P(stats), P(gpart), nsl.value, P(dx), int(acc),
                                          P(self.g(prefix + "weight")), P(self.g(prefix + "bias")), P(dss), P(work),
                                          work.numel(), *self._addend(add), P(dx1), self.s))
        return (dx, dx1) if split is not None else dx

    def resample(self, x, N, Hin, C, mode):
        Ho = 2 * Hin if mode == 1 else Hin // 2
        out = self._empty(N, Ho, Ho, C)
        chk(lib().ifd_tr_resample(P(x), N, Hin, C, mode, P(out), self.s))
        return out

    def resample_bwd(self, dy, N, Hin, C, mode, dx=None):
        acc = dx is not None
        if dx is None:
            dx = self._empty(N, Hin, Hin, C)
        else:
            self._dirty(dx)
        chk(lib().ifd_tr_resample_bwd(P(dy), N, Hin, C, mode, P(dx), int(acc), self.s))
        return dx

    def add_(self, dst, src):
        self._dirty(dst)
        chk(lib().ifd_tr_add(P(dst), P(src), P(dst), dst.numel(), self.s))
        return dst

    def copy_ch(self, src, cs, soff, dst, cd, doff, nc, npix, acc):
        self._dirty(dst)
        chk(lib().ifd_tr_copy_channels(P(src), cs, soff, P(dst), cd, doff, nc, npix, int(acc), self.s))

    def linear(self, x, M, name_w, name_b, pre_silu=False):
        w = self.p(name_w)
        y = self._empty(M, w.shape[0])
        chk(lib().ifd_tr_linear(P(x), M, w.shape[1], P(w), P(self.p(name_b)), w.shape[0], int(pre_silu), 0, P(y), self.s))
        return y

    def linear_bwd(self, dy, x, M, name_w, name_b, pre_silu=False, dx=None, want_dx=True):
        w = self.p(name_w)
        acc = dx is not None
        if want_dx and dx is None:
            dx = self._empty(M, w.shape[1])
        chk(lib().ifd_tr_linear_bwd(P(dy), P(x), M, w.shape[1], P(w), w.shape[0], int(pre_silu),
                                    P(dx) if want_dx else None, int(acc), P(self.g(name_w)), P(self.g(name_b)), self.s))
        return dx

    # ------------------------------------------------------------------ forward / backward
    def forward(self, x, t, masked_image, mask):
        """UNet forward (code/unet.py:154-173, 197-200) keeping the activations the backward needs.
        x, masked_image [N,3,H,W], mask [N,1,H,W] NCHW fp32; t int64 [N]. Returns out6 NHWC [N,H,W,6]."""
        cfg = self.cfg
        N, _, H, _ = x.shape
        self._gstat = {}
        self.s = _lib.stream_ptr(self.dev)
        self._repack_all()
        tape = {"N": N, "H": H}
        # time embedding: temb -> Linear -> SiLU -> Linear (unet.py:44-48); all emb_layers (nn.py:167-170)
        temb = self._empty(N, cfg.model_channels)
        chk(lib().ifd_tr_temb(P(t), P(self.freqs), N, cfg.model_channels, P(temb), self.s))
        z0 = self.linear(temb, N, "time_embed.0.weight", "time_embed.0.bias")
        emb = self.linear(z0, N, "time_embed.2.weight", "time_embed.2.bias", pre_silu=True)
        tape.update(temb=temb, z0=z0, emb=emb, E={})
        x16 = self._empty(N, H, H, 16)
        chk(lib().ifd_tr_pack_input(P(x), P(masked_image), P(mask), N, H * H, P(x16), self.s))
        tape["x16"] = x16
        hs, saved = [], {}
        h, hc, hr = None, 0, H
        for section, bi, layers in self.plan:
            pend = None  # the output block's skip, read by the block's first ResBlock as concat(h, skip)
            if section == "output":
                skip = hs.pop()
                sc = skip.shape[-1]
                L0 = layers[0]
                if (self._gn_fused() and L0["kind"] == "res" and L0["cout"] != hc + sc and hc % 64 == 0
                        and sc % 32 == 0 and (hc + sc) % 128 == 0 and self._granules2(h, skip) is not None):
                    pend = (skip, sc)
                else:  # the concat materialised (code/unet.py:170)
                    cat = self._empty(N, hr, hr, hc + sc)
                    self.copy_ch(h, hc, 0, cat, hc + sc, 0, hc, N * hr * hr, False)
                    self.copy_ch(skip, sc, 0, cat, hc + sc, hc, sc, N * hr * hr, False)
                    # the concat's GroupNorm statistics from both sources' granules (same map: same E, cnt)
                    g2 = self._granules2(h, skip)
                    if g2 is not None:
                        self._gstat[cat.data_ptr()] = (cat,) + g2[1:]
                    h, hc = cat, hc + sc
            for L in layers:
                k, p = L["kind"], L["prefix"]
                if k == "conv_in":
                    h = self.conv(x16, 16, N, hr, p + "weight", p + "bias")
                    hc = L["cout"]
                elif k in ("res", "res_down", "res_up"):
                    if pend is not None:
                        h, hr = self._res_fwd(L, h, N, hr, emb, saved, x1=pend[0], c1=pend[1])
                        pend = None
                    else:
                        h, hr = self._res_fwd(L, h, N, hr, emb, saved)
                    hc = L["cout"]
                elif k == "attn":
                    h = self._attn_fwd(L, h, N, hr, saved)
                elif k == "out":
                    if self._gn_fused():
                        gn, st = self.gn_coef(h, N, hr * hr, hc, "out.0.")
                        saved["out"] = dict(x=h, a=None, gn=gn, stats=st)
                        h = self._head_x3(h, hc, N, hr, gn)
                    else:
                        a, st = self.gn_fwd(h, N, hr * hr, hc, "out.0.", silu=True)
                        saved["out"] = dict(x=h, a=a, gn=None, stats=st)
                        h = self.conv(a, hc, N, hr, "out.2.weight", "out.2.bias")
                    hc = L["cout"]
            if section == "input":
                hs.append(h)
        tape["saved"] = saved
        self._tape = tape
        return h  # [N, H, W, 8]: the 6 output channels, then 2 zero channels

    def _res_fwd(self, L, x, N, r, emb, saved, x1=None, c1=0):
        """ResBlock._forward (code/nn.py:189-212), scale-shift norm, resblock_updown. x1: the output blocks'
        skip tensor; the block's input is then concat(x, x1) (code/unet.py:170), read by channel range by every
        consumer (GroupNorm statistics from both sources' granules, conv1's prologue, the 1x1 skip conv)."""
        p, cin, cout, k = L["prefix"], L["cin"], L["cout"], L["kind"]
        mode = 1 if k == "res_up" else (2 if k == "res_down" else 0)
        ro = 2 * r if mode == 1 else (r // 2 if mode == 2 else r)
        fused = self._gn_fused()
        g1 = g2 = a1r = a2 = None
        c0 = cin - c1
        if x1 is not None:  # (the caller checked: fused mode, mode 0, cin != cout, both granules)
            g1, st1 = self.gn_coef(x, N, r * r, cin, p + "in_layers.0.", x1=x1)
            h1 = self.conv(x, c0, N, ro, p + "in_layers.2.weight", p + "in_layers.2.bias", x1=x1, c1=c1, gn=g1)
        elif fused and not mode:  # in_layers: GroupNorm + SiLU applied by conv1's prologue (and wgrad's staging)
            g1, st1 = self.gn_coef(x, N, r * r, cin, p + "in_layers.0.")
            h1 = self.conv(x, cin, N, ro, p + "in_layers.2.weight", p + "in_layers.2.bias", gn=g1)
        elif fused:  # a resampling block: act + resample of x and resample of x in one pass
            (A, B), st1 = self.gn_coef(x, N, r * r, cin, p + "in_layers.0.")
            a1r, xr = self._empty(N, ro, ro, cin), self._empty(N, ro, ro, cin)
            chk(lib().ifd_tr_act_resample(P(x), N, r, cin, P(A), P(B), mode, P(a1r), P(xr), self.s))
            h1 = self.conv(a1r, cin, N, ro, p + "in_layers.2.weight", p + "in_layers.2.bias")
        else:
            a1, st1 = self.gn_fwd(x, N, r * r, cin, p + "in_layers.0.", silu=True)
            a1r = self.resample(a1, N, r, cin, mode) if mode else a1
            h1 = self.conv(a1r, cin, N, ro, p + "in_layers.2.weight", p + "in_layers.2.bias")
        if not (fused and mode and x1 is None):
            xr = self.resample(x, N, r, cin, mode) if mode else x
        E = self.linear(emb, N, p + "emb_layers.1.weight", p + "emb_layers.1.bias", pre_silu=True)  # [N, 2 cout]
        if cin != cout:
            skip = self.conv(xr, c0, N, ro, p + "skip_connection.weight", p + "skip_connection.bias", x1=x1, c1=c1)
        else:
            skip = xr
        if fused:  # out_layers: GroupNorm + scale/shift + SiLU in conv2's prologue
            g2, st2 = self.gn_coef(h1, N, ro * ro, cout, p + "out_layers.0.", ss=E, ss_stride=2 * cout)
            out = self.conv(h1, cout, N, ro, p + "out_layers.3.weight", p + "out_layers.3.bias", res=skip, gn=g2)
        else:
            a2, st2 = self.gn_fwd(h1, N, ro * ro, cout, p + "out_layers.0.", ss=E, ss_stride=2 * cout, silu=True)
            out = self.conv(a2, cout, N, ro, p + "out_layers.3.weight", p + "out_layers.3.bias", res=skip)
        saved[p] = dict(x=x, x1=x1, c1=c1, a1r=a1r, g1=g1, xr=xr, h1=h1, a2=a2, g2=g2, E=E, st1=st1, st2=st2,
                        mode=mode, r=r, ro=ro)
        return out, ro

    def _attn_fwd(self, L, x, N, r, saved):
        """AttentionBlock._forward (code/nn.py:259-265) with QKVAttention (:222-235)."""
        p, C = L["prefix"], L["cin"]
        T = r * r
        n, st = self.gn_fwd(x, N, T, C, p + "norm.", silu=False)
        qkv = self.conv(n, C, N, r, p + "qkv.weight", p + "qkv.bias")
        a = self._empty(N, T, C)
        scale = 1.0 / math.sqrt(math.sqrt(self.cfg.num_head_channels))
        chk(lib().ifd_tr_attention(P(qkv), N, T, C, scale, P(a), self.s))
        out = self.conv(a, C, N, r, p + "proj_out.weight", p + "proj_out.bias", res=x)
        saved[p] = dict(x=x, n=n, st=st, qkv=qkv, a=a, scale=scale)
        return out

    def backward(self, dout6, grad_scale=None):
        """Gradients of every parameter (+= into the flat grad buffer) from d loss / d out6 (NHWC).
        grad_scale: the factor dout6 carries (default: the 3xf16 loss scale when dout6 is the loss's own
        gradient); the accumulated gradients are brought to it first and divided by it after (exact)."""
        if grad_scale is None:
            grad_scale = getattr(self, "_gscale", 1.0) if dout6 is getattr(self, "_dout6", None) else 1.0
        if grad_scale != 1.0 and not self._grad_clean:
            chk(lib().ifd_tr_scale(P(self.grad), self.numel, grad_scale, _lib.stream_ptr(self.dev)))
        self._backward(dout6)
        if grad_scale != 1.0:
            chk(lib().ifd_tr_scale(P(self.grad), self.numel, 1.0 / grad_scale, self.s))
        self._grad_clean = False

    def _backward(self, dout6):
        tape = self._tape
        N, H = tape["N"], tape["H"]
        saved = tape["saved"]
        emb = tape["emb"]
        demb = self._zeros(N, self.emb_dim)
        # output head: conv 128 -> 6 (its dgrad input padded to 8 channels)
        so = saved["out"]
        hc = so["x"].shape[-1]
        co = dout6.shape[-1]  # the head's channel count padded to 4 (zero gradient in the pad)
        if so["gn"] is not None:
            self.wgrad(dout6, co, so["x"], hc, N, H, "out.2.weight", "out.2.bias", gn=so["gn"])
        else:
            self.wgrad(dout6, co, so["a"], hc, N, H, "out.2.weight", "out.2.bias")
        da = dh = None
        if self._x3_active(True) and co % 16:
            # the split kernel's dgrad reads 16-channel chunks: the head gradient padded with zero channels
            # (else the 8-channel dgrad runs on the fp32 kernel, ~4x the split kernel's time at 256^2).
            # Only the split kernel takes the padded operand: when the shape is not eligible (e.g.
            # model_channels not a multiple of 64) the fp32 kernel runs on the unpadded gradient.
            d16 = self._zeros(N, H, H, 16)
            self.copy_ch(dout6, co, 0, d16, 16, 0, co, N * H * H, False)
            dh = self._dgrad_gnb(d16, 16, N, H, "out.2.weight", so["x"], hc, "out.0.", so["stats"], None, None, 0,
                                 None, True, None, None)
            if dh is None:
                da = self._conv_x3(d16, 16, N, H, "out.2.weight", None, None, None, 0, True)
        if dh is None:
            if da is None:
                da = self.conv(dout6, co, N, H, "out.2.weight", transpose=True)
            dh = self.gn_bwd(da, so["x"], N, H * H, hc, "out.0.", so["stats"], silu=True)
        # hs gradients from the output blocks' skip inputs
        in_blocks = [b for b in self.plan if b[0] == "input"]
        dhs = [None] * len(in_blocks)
        hs_idx = 0  # the last output block (first here) consumed hs[0]
        r = H
        for section, bi, layers in reversed(self.plan):
            if section in ("out",):
                continue
            if section == "input":
                break
            for i, L in enumerate(reversed(layers)):
                # the middle block's input is the last input block's output: its first layer's dx also takes that
                # block's skip gradient (filled by the output blocks above)
                last = section == "middle" and i == len(layers) - 1
                first_out = section == "output" and i == len(layers) - 1
                dh, r = self._layer_bwd(L, dh, N, saved, demb, add=self._skip_addend(dhs[-1]) if last else None,
                                        split=first_out)
                if last:
                    dhs[-1] = None
            if section == "output":
                # split d cat(h, skip) (code/unet.py:170)
                cin = layers[0]["cin"]
                sc = layers[0]["skip_ch"]
                hcur = cin - sc
                if isinstance(dh, tuple):  # already per source (the concat was never materialised)
                    dh, dskip = dh
                    dhs[hs_idx] = (dskip, sc, 0, sc, N * r * r)
                else:
                    dprev = self._empty(N, r, r, hcur)
                    self.copy_ch(dh, cin, 0, dprev, hcur, 0, hcur, N * r * r, False)
                    # the skip part stays in d cat until the input chain accumulates it (no copy of its own)
                    dhs[hs_idx] = (dh, cin, hcur, sc, N * r * r)
                    dh = dprev
                hs_idx += 1
        # middle block's input = the last input block's output: dh continues down the input chain. Input block
        # b's output gradient = the chain's + its skip part in d cat (dhs[b]): added where block b + 1's first
        # layer writes its dx (the GroupNorm backward's addend), else by a channel copy
        for bidx in range(len(in_blocks) - 1, -1, -1):
            section, bi, layers = in_blocks[bidx]
            if dhs[bidx] is not None:
                dcat, cin, off, sc, npix = dhs[bidx]
                self.copy_ch(dcat, cin, off, dh, sc, 0, sc, npix, True)
                dhs[bidx] = None
            for i, L in enumerate(reversed(layers)):
                first = i == len(layers) - 1
                if L["kind"] == "conv_in":
                    self.wgrad(dh, L["cout"], tape["x16"], 16, N, r, L["prefix"] + "weight", L["prefix"] + "bias",
                               real_cin=L["cin"])
                    dh = None
                else:
                    add = self._skip_addend(dhs[bidx - 1]) if first and bidx >= 1 else None
                    dh, r = self._layer_bwd(L, dh, N, saved, demb, add=add)
                    if add is not None:
                        dhs[bidx - 1] = None
        # embedding MLP backward (unet.py:44-48)
        dz0 = self.linear_bwd(demb, tape["z0"], N, "time_embed.2.weight", "time_embed.2.bias", pre_silu=True)
        self.linear_bwd(dz0, tape["temb"], N, "time_embed.0.weight", "time_embed.0.bias", want_dx=False)

    @staticmethod
    def _skip_addend(rec):
        """dhs entry (d cat, its channels, skip offset, skip channels, pixels) -> gn_bwd's add = (t, stride, offset)."""
        if rec is None:
            return None
        dcat, cin, off, sc, npix = rec
        return (dcat, cin, off)

    def _layer_bwd(self, L, dout, N, saved, demb, add=None, split=False):
        """add: (t, stride, offset) added into the layer's input gradient (a ResBlock's GroupNorm dx pass).
        split: an output block's first ResBlock over concat(h, skip) (never materialised) returns its input
        gradient per source, (d h, d skip), instead of one C-wide tensor."""
        k, p = L["kind"], L["prefix"]
        if k == "attn":
            if add is not None:
                raise ValueError("the skip addend goes to a block's first (ResBlock) layer")
            sv = saved[p]
            C = L["cin"]
            r = int(round(math.sqrt(sv["a"].shape[1])))
            T = r * r
            self.wgrad(dout, C, sv["a"], C, N, r, p + "proj_out.weight", p + "proj_out.bias")
            da = self.conv(dout, C, N, r, p + "proj_out.weight", transpose=True)
            dqkv = self._empty(N, T, 3 * C)
            sf = lib().ifd_tr_attention_bwd_scratch_floats(N, T, C)
            scratch = self._empty(sf)
            chk(lib().ifd_tr_attention_bwd(P(sv["qkv"]), P(da), N, T, C, sv["scale"], P(dqkv), P(scratch), sf, self.s))
            self.wgrad(dqkv, 3 * C, sv["n"], C, N, r, p + "qkv.weight", p + "qkv.bias")
            dn = self.conv(dqkv, 3 * C, N, r, p + "qkv.weight", transpose=True)
            # the residual's gradient: accumulated into dout in place (dout is not read after this)
            dx = self.gn_bwd(dn, sv["x"], N, T, C, p + "norm.", sv["st"], dx=dout, silu=False)
            return dx, r
        sv = saved[p]
        cin, cout, mode, r, ro = L["cin"], L["cout"], sv["mode"], sv["r"], sv["ro"]
        # h2 = conv2(a2) + b2; out = skip + h2. The dgrad first: its GNB epilogue can write a2 itself (act2), which
        # the weight gradient then reads instead of re-applying GroupNorm + scale/shift + SiLU to h1 on load
        dE = self._zeros(N, 2 * cout)
        act2 = []
        dh1 = self.dgrad_gn_bwd(dout, cout, N, ro, p + "out_layers.3.weight", sv["h1"], cout, p + "out_layers.0.",
                                sv["st2"], ss=sv["E"], ss_stride=2 * cout, dss=dE, silu=True,
                                act_sink=act2 if sv["g2"] is not None else None)
        if act2:
            self.wgrad(dout, cout, act2[0], cout, N, ro, p + "out_layers.3.weight", p + "out_layers.3.bias")
        elif sv["g2"] is not None:
            self.wgrad(dout, cout, sv["h1"], cout, N, ro, p + "out_layers.3.weight", p + "out_layers.3.bias",
                       gn=sv["g2"])
        else:
            self.wgrad(dout, cout, sv["a2"], cout, N, ro, p + "out_layers.3.weight", p + "out_layers.3.bias")
        del act2
        self.linear_bwd(dE, self._tape["emb"], N, p + "emb_layers.1.weight", p + "emb_layers.1.bias", pre_silu=True,
                        dx=demb)
        x1, c1 = sv.get("x1"), sv.get("c1", 0)
        c0 = cin - c1  # (x1: the block input is concat(x[c0], x1[c1]), never materialised)
        # without resampling, conv1's weight gradient waits for the dgrad below: its GNB epilogue can write
        # a1 = silu(GN1(x)) for it (act1), instead of the weight gradient re-applying GN + SiLU to x on load
        defer1 = sv["g1"] is not None and not mode
        if sv["g1"] is not None and not defer1:
            self.wgrad(dh1, cout, sv["x"], c0, N, ro, p + "in_layers.2.weight", p + "in_layers.2.bias", gn=sv["g1"],
                       x1=x1, c1=c1)
        elif sv["g1"] is None:
            self.wgrad(dh1, cout, sv["a1r"], cin, N, ro, p + "in_layers.2.weight", p + "in_layers.2.bias")
        if mode:
            da1r = self.conv(dh1, cout, N, ro, p + "in_layers.2.weight", transpose=True)
        if cin != cout:
            self.wgrad(dout, cout, sv["xr"], c0, N, ro, p + "skip_connection.weight", p + "skip_connection.bias",
                       x1=x1, c1=c1)
            dxr = self.conv(dout, cout, N, ro, p + "skip_connection.weight", transpose=True)
        else:
            dxr = dout
        if mode:
            # GroupNorm backward through the resample adjoint: dx = gn_bwd(adj(da1r)) + adj(dxr) (+ add) in one pass
            dx = self._empty(N * r * r * cin)
            nsl = lib().ifd_tr_gn_slices(r * r, N, cin)
            work = self._empty(N * nsl * cin * 3 + N * cin * 3 + N * 64)
            ap, ast = self._addend(add)
            pre = p + "in_layers.0."
            chk(lib().ifd_tr_gn_bwd_resampled(P(da1r), P(sv["x"]), N, r, cin, P(self.p(pre + "weight")),
                                              P(self.p(pre + "bias")), 1, P(sv["st1"]), mode, P(dxr), P(dx),
                                              P(self.g(pre + "weight")), P(self.g(pre + "bias")), ap, ast, P(work),
                                              work.numel(), self.s))
        else:
            # the skip path's gradient (dout itself, or the 1x1 conv's fresh dgrad) is the accumulation
            # target of the GroupNorm input gradient: no separate add pass; the dgrad of in_layers.2 carries
            # the GroupNorm backward's pass 1 (dgrad_gn_bwd)
            act1 = [] if defer1 else None
            if split and x1 is not None:
                # the skip path's gradient joins as the addend and dx comes out per concat source
                if add is not None:
                    raise ValueError("a split input gradient takes no other addend")
                pair = (self._empty(N, r, r, c0), self._empty(N, r, r, c1))
                dx = self.dgrad_gn_bwd(dh1, cout, N, ro, p + "in_layers.2.weight", sv["x"], cin, p + "in_layers.0.",
                                       sv["st1"], silu=True, x1=x1, C0=c0, add=(dxr, cin, 0), split=pair,
                                       act_sink=act1)
            else:
                dx = self.dgrad_gn_bwd(dh1, cout, N, ro, p + "in_layers.2.weight", sv["x"], cin, p + "in_layers.0.",
                                       sv["st1"], dx=dxr, silu=True, x1=x1, C0=c0, add=add, act_sink=act1)
            if act1:
                self.wgrad(dh1, cout, act1[0], cin, N, ro, p + "in_layers.2.weight", p + "in_layers.2.bias")
            elif defer1:
                self.wgrad(dh1, cout, sv["x"], c0, N, ro, p + "in_layers.2.weight", p + "in_layers.2.bias",
                           gn=sv["g1"], x1=x1, c1=c1)
        return dx, r

    # ------------------------------------------------------------------ loss / step
    def tables(self, diffusion):
        key = id(diffusion)
        if getattr(self, "_tables_key", None) != key:
            self._sa = torch.from_numpy(diffusion.sqrt_alphas_cumprod).float().to(self.dev)
            self._s1m = torch.from_numpy(diffusion.sqrt_one_minus_alphas_cumprod).float().to(self.dev)
            self._tables_key = key
        return self._sa, self._s1m

    def training_loss(self, diffusion, x_start, t, model_kwargs, noise=None, use_injection=True, noise_device=None):
        """GaussianDiffusion.training_losses (code/gaussian_diffusion.py:540-614) for the MSE loss with
        LEARNED_RANGE output, injection schedule "all" and cumulative GT noise: returns the loss (device
        scalar) and keeps d loss / d out6 for `backward`. RNG draws in the reference's order: noise (if not
        given), then the GT-noise cache entry for (shape, t[0]) on first use; the cache is never cleared."""
        self.s = _lib.stream_ptr(self.dev)
        N, _, H, W = x_start.shape
        mask = model_kwargs.get("mask")
        masked = model_kwargs.get("masked_image")
        if mask is None:
            mask = torch.ones(N, 1, H, W, device=self.dev)
        if noise is None:
            noise = (torch.randn(x_start.shape, device=noise_device) if noise_device else
                     torch.randn_like(x_start)).to(self.dev)
        inject = bool(use_injection and masked is not None)
        cached = noise
        if inject:
            t0 = int(t[0].item())  # the reference's int(t[0].item()) (gaussian_diffusion.py:131)
            key = (tuple(x_start.shape), t0)
            cached = self._gt_noise_cache.get(key)
            if cached is None:
                cached = (torch.randn(x_start.shape, device=noise_device) if noise_device else
                          torch.randn_like(x_start)).to(self.dev)
                self._gt_noise_cache[key] = cached
        sa, s1m = self.tables(diffusion)
        xt = self._empty(N, 3, H, W)
        x0c, nc_, mc = (v.to(self.dev, torch.float32).contiguous() for v in (x_start, noise, mask))
        tt = t.to(self.dev, torch.int64).contiguous()
        chk(lib().ifd_tr_q_sample_inject(P(x0c), P(nc_), P(cached.contiguous()), P(mc), P(tt), P(sa), P(s1m), N,
                                         H * W, int(inject), P(xt), self.s))
        mi = masked.to(self.dev, torch.float32).contiguous() if masked is not None else self._zeros(N, 3, H, W)
        self._keep = (xt, mi, mc, nc_, x0c, tt)
        return self._forward_loss(xt, tt, mi, mc, nc_)

    def _forward_loss(self, xt, tt, mi, mc, nc_):
        """UNet forward + masked eps-MSE; keeps d loss / d out6 (times the 3xf16 loss scale) for backward."""
        N, _, H, W = xt.shape
        out6 = self.forward(xt, tt, mi, mc)  # [N, H, W, 8]: channels 0-5 the model output
        cs = out6.shape[-1]
        self._dout6 = self._empty(N, H, W, cs)
        work = self._empty(N * 6)
        chk(lib().ifd_tr_masked_mse(P(out6), cs, P(nc_), P(mc), N, H * W, P(self.loss), P(self._dout6), P(work),
                                    self.s))
        self._gscale = 1.0
        if self._split() and (self.x3_dgrad or self.x3_wgrad):
            self._gscale = float(2.0 ** self.x3_loss_scale_log2)
            chk(lib().ifd_tr_scale(P(self._dout6), self._dout6.numel(), self._gscale, self.s))
        return self.loss

    def zero_grad(self):
        self.grad.zero_()
        self._grad_clean = True

    def optimizer_step(self):
        """clip_grad_norm_(max_norm) + AdamW (code/train_inpainting.py:64-66); norm on device, no sync."""
        self.step_count += 1
        work = torch.empty(1024, device=self.dev, dtype=torch.float64)
        b1, b2 = self.betas
        chk(lib().ifd_tr_clip_adamw(P(self.flat), P(self.grad), P(self.m), P(self.v), self.numel, self.max_norm,
                                    self.lr, b1, b2, self.eps, self.wd, self.step_count, P(work), P(self.norm_coef),
                                    _lib.stream_ptr(self.dev)))

    def train_step(self, diffusion, images, masked_images, masks, t, noise=None, noise_device=None):
        """One iteration of train_epoch (code/train_inpainting.py:27-66): zero_grad, training_losses,
        backward, clip_grad_norm_(1.0), AdamW.step(). Returns the loss as a device scalar.
        3xf16 / f16: one host read of the range guard per step; a trip recomputes the step in fp32."""
        self.zero_grad()
        if self._split():
            self._guard.zero_()
        loss = self.training_loss(diffusion, images, t, {"masked_image": masked_images, "mask": masks}, noise=noise,
                                  noise_device=noise_device)
        self.backward(self._dout6)
        if self._split() and int(self._guard[0].item()):
            import warnings
            warnings.warn(f"{self.precision} range guard tripped (an operand or weight outside the f16 split's "
                          "range): step recomputed in fp32")
            self.guard_trips += 1
            prec, self.precision = self.precision, "fp32"
            try:
                self.zero_grad()
                xt, mi, mc, nc_, _x0, tt = self._keep
                loss = self._forward_loss(xt, tt, mi, mc, nc_)
                self.backward(self._dout6)
            finally:
                self.precision = prec
        self.optimizer_step()
        return loss


class BlockTrainer(UNetTrainer):
    """Forward + backward of ONE block of the UNet on the same training ops (a per-block entry point:
    ResBlock, code/nn.py:136-212 — plain, with 1x1 skip, down, up — or AttentionBlock, :238-265).
    Parameter names are the reference module's own state_dict keys (no prefix). Tensors NCHW at the
    boundary, NHWC inside."""

    def __init__(self, kind, cin, cout, emb_dim=None, device="cuda", num_head_channels=64):
        from types import SimpleNamespace
        from .topology import _attn_params, _res_params
        self.dev = torch.device(device)
        self.kind, self.cin, self.cout = kind, cin, cout
        self.emb_dim = emb_dim
        self.cfg = SimpleNamespace(num_head_channels=num_head_channels, model_channels=0, out_channels=cout)
        spec = _res_params("", cin, cout, emb_dim) if kind.startswith("res") else _attn_params("", cin)
        self.spec = [(k, tuple(s)) for k, s in spec]
        self.offsets, n = {}, 0
        for k, shape in self.spec:
            self.offsets[k] = (n, shape)
            n += int(np.prod(shape))
        self.numel = n
        self.flat = torch.zeros(n, device=self.dev)
        self.grad = torch.zeros(n, device=self.dev)
        self._zero_bias = torch.zeros(4096, device=self.dev)
        self._pack_cache = {}
        self._gstat = {}
        self.precision, self.x3_dgrad, self.x3_loss_scale_log2, self.guard_trips = "fp32", False, 0, 0
        self.x3_wgrad = False
        self.fuse_gn = True  # (no effect in fp32: GroupNorm on load is a split-mode path)
        self.fuse_gnb = True
        self._guard = torch.zeros(4, device=self.dev, dtype=torch.int32)
        self._grad_clean = False
        self._pack_cache = {}
        self._pack_persist = {}
        self._pack_table = None
        self._gstat = {}
        self.s = None

    def load_state_dict(self, sd):
        with torch.no_grad():
            for k, _ in self.spec:
                self.p(k).copy_(torch.as_tensor(sd[k]).to(self.dev, torch.float32).reshape(self.p(k).shape))

    def forward_block(self, x, emb=None):
        self.s = _lib.stream_ptr(self.dev)
        self._pack_cache = {}
        self._gstat = {}
        N, C, H, _ = x.shape
        xh = x.to(self.dev, torch.float32).permute(0, 2, 3, 1).contiguous()
        self._saved = {}
        L = dict(kind=self.kind, prefix="", cin=self.cin, cout=self.cout)
        if self.kind.startswith("res"):
            e = emb.to(self.dev, torch.float32).contiguous()
            self._tape = {"emb": e}
            y, r = self._res_fwd(L, xh, N, H, e, self._saved)
        else:
            y, r = self._attn_fwd(L, xh, N, H, self._saved), H
        self._N, self._r, self._rin = N, r, H
        return y.view(N, r, r, -1).permute(0, 3, 1, 2).contiguous()

    def backward_block(self, dy):
        N = self._N
        dyh = dy.to(self.dev, torch.float32).permute(0, 2, 3, 1).contiguous()
        L = dict(kind=self.kind, prefix="", cin=self.cin, cout=self.cout)
        demb = self._zeros(N, self.emb_dim) if self.kind.startswith("res") else None
        dx, _ = self._layer_bwd(L, dyh, N, self._saved, demb)
        dx = dx.view(N, self._rin, self._rin, self.cin)
        return dx.permute(0, 3, 1, 2).contiguous(), demb
