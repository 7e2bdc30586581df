"""`DiffusionInpaintingModel` drop-in whose forward runs on the HIP library.

Mirrors the Python surface the reference's sampling scripts use (code/unet.py:176-200,
code/test_inp_ddim_50.py:325-385): parameters under the reference's `base_model.` state-dict keys,
`load_state_dict(sd, strict=False) -> (missing, unexpected)`, `eval()`, `parameters()` (the
scripts read `next(model.parameters()).device`), and `forward(x, t, masked_image=, mask=)`
returning the [B, 6, H, W] fp32 output (eps + learned-range variance values).

The parameters live as ordinary device tensors; on the first forward after a (re)load they are
handed to the library (`ifd_load_weights`), which packs its own NHWC/KRSC-style copies.
There is no CPU/PyTorch fallback: a CPU tensor or a missing library raises.

precision="3xf16" is guarded: the split kernels flag any operand that reaches the f16 range
(include/ifd.h ifd_guard_*). Two ways to act on the flag (`guard=`, env IFD_GUARD):
* "sync" (the default since round 6): each forward checks the guard after its launch (one stream
  synchronisation) and recomputes a flagged forward in exact fp32 (counted in `guard_trips`) before
  returning it: fp32-class for any input, so an unchanged reference script's own loop (model() once per
  step, code/test_inp_ddim_100.py:512-574) survives a trip with the fp32 run's result. Measured cost on
  that loop: none (8.733 vs 8.716 images/s with "lazy", the same box, profiles/r06a/bench_dropin_*.json):
  the GPU work of one forward (~18 ms at B = 16) dwarfs the host's enqueue of the next.
* "lazy": a forward never waits on the GPU. Each 3xf16 forward enqueues an asynchronous copy of the
  (sticky) guard word into page-locked memory; the next forwards look at the copies whose work has
  finished. A trip raises RuntimeError from a LATER forward (or from `guard_check()`), at most a few
  forwards after the one that tripped; the outputs of the forwards in between are not recomputed.
The fused sampler loops (ifd.sampler) check once per loop and re-run the whole loop in fp32, in both.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib
from .topology import FULL, UNetConfig, state_dict_spec


class _Node(torch.nn.Module):
    pass


def _config_struct(cfg: UNetConfig):
    c = _lib.IfdConfig()
    c.image_size = cfg.image_size
    c.in_channels = cfg.in_channels
    c.model_channels = cfg.model_channels
    c.out_channels = cfg.out_channels
    c.num_res_blocks = cfg.num_res_blocks
    c.num_levels = len(cfg.channel_mult)
    for i, m in enumerate(cfg.channel_mult):
        c.channel_mult[i] = m
    c.num_attention = len(cfg.attention_resolutions)
    for i, d in enumerate(cfg.attention_resolutions):
        c.attention_ds[i] = d
    c.num_head_channels = cfg.num_head_channels
    return c


class Handle:
    """Owns one `ifd_handle` (one per device)."""

    def __init__(self, cfg: UNetConfig):
        L = _lib.lib()
        h = ctypes.c_void_p()
        _lib.check(L.ifd_create(ctypes.byref(_config_struct(cfg)), ctypes.byref(h)))
        self.h = h
        self.cfg = cfg

    def __del__(self):
        try:
            if getattr(self, "h", None) is not None and _lib._lib is not None:
                _lib._lib.ifd_destroy(self.h)
        except Exception:
            pass

    def param_names(self):
        L = _lib.lib()
        n = ctypes.c_int()
        _lib.check(L.ifd_num_params(self.h, ctypes.byref(n)))
        out = []
        for i in range(n.value):
            name = ctypes.c_char_p()
            shape = (ctypes.c_int64 * 4)()
            nd = ctypes.c_int()
            _lib.check(L.ifd_param_info(self.h, i, ctypes.byref(name), shape, ctypes.byref(nd)))
            out.append((name.value.decode(), tuple(shape[k] for k in range(nd.value))))
        return out


class DiffusionInpaintingModel(torch.nn.Module):
    """9-channel inpainting UNet (code/unet.py:176-200) executed by libifd."""

    def __init__(self, cfg: UNetConfig = FULL, device=None, precision: str = "3xf16", options=None, guard=None):
        super().__init__()
        self.cfg = cfg
        self.guard = guard or os.environ.get("IFD_GUARD", "sync")  # module docstring
        if self.guard not in ("lazy", "sync"):
            raise ValueError("guard must be 'lazy' or 'sync'")
        # handle options (include/ifd.h ifd_set_option), e.g. {"batch_invariant": 1}
        self.options = dict(options or {})
        if precision not in _lib.PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(_lib.PRECISIONS)}")
        # "fp32": exact fp32 MFMA; "3xf16": split f16 MFMA with fp32-level error (include/ifd.h)
        self.precision = precision
        self.base_model = _Node()
        for key, shape in state_dict_spec(cfg, prefix=""):
            node = self.base_model
            parts = key.split(".")
            for p in parts[:-1]:
                if not hasattr(node, p) or not isinstance(getattr(node, p), torch.nn.Module):
                    node.add_module(p, _Node())
                node = getattr(node, p)
            node.register_parameter(parts[-1], torch.nn.Parameter(torch.zeros(shape, device=device),
                                                                  requires_grad=False))
        self._handle = None
        self._handle_device = None
        self._dirty = True
        self.dtype = torch.float32
        self.guard_trips = 0  # 3xf16 evals / loops recomputed in fp32 by the range guard
        self._applied = None  # (handle, precision, options) last pushed to the library
        self._deferred = None  # deferred_guard(): per-forward guard reads suspended
        self._lz = None  # lazy guard: [handle, pinned slots, pending [(event, slot)], next slot, armed]

    # -- weights -------------------------------------------------------------------------------
    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        res = super().load_state_dict(state_dict, strict=strict)
        self._dirty = True
        return res

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        self._dirty = True
        return out

    def handle(self, device):
        if self._handle is None or self._handle_device != device:
            with torch.cuda.device(device):
                self._handle = Handle(self.cfg)
            self._handle_device = device
            self._dirty = True
        if self._dirty:
            L = _lib.lib()
            torch.cuda.synchronize(device)
            with torch.cuda.device(device):
                for name, p in self.base_model.named_parameters():
                    t = p.detach().to(device=device, dtype=torch.float32).contiguous()
                    shape = (ctypes.c_int64 * max(1, t.dim()))(*t.shape)
                    _lib.check(L.ifd_load_weights(self._handle.h, name.encode(), _lib.ptr(t), shape, t.dim()))
                    del t
                _lib.check(L.ifd_finalize(self._handle.h))
            self._dirty = False
        # precision / options reach the handle only when they changed (no per-forward ctypes calls)
        state = (id(self._handle), self.precision, tuple(sorted((k, int(v)) for k, v in self.options.items())))
        if state != self._applied:
            L = _lib.lib()
            _lib.check(L.ifd_set_precision(self._handle.h, _lib.PRECISIONS[self.precision]))
            for k, v in self.options.items():
                _lib.check(L.ifd_set_option(self._handle.h, k.encode(), int(v)))
            self._applied = state
        return self._handle

    # -- forward -------------------------------------------------------------------------------
    @staticmethod
    def _dev_f32(t, device, name):
        if not isinstance(t, torch.Tensor) or t.device != device:
            raise RuntimeError(f"ifd: `{name}` must be a tensor on {device} (no CPU fallback)")
        return t.to(torch.float32).contiguous()

    def forward(self, x, t, masked_image=None, mask=None, **kwargs):
        if masked_image is None or mask is None:
            raise ValueError("DiffusionInpaintingModel.forward requires masked_image and mask")
        if not x.is_cuda:
            raise RuntimeError("ifd: the HIP UNet runs on GPU tensors only (no CPU fallback)")
        dev = x.device
        if x.dim() != 4 or x.shape[1] != 3:
            raise ValueError(f"x must be [B,3,H,W], got {tuple(x.shape)}")
        B, C, H, W = x.shape
        # the reference's torch.cat needs equal batch sizes; a batch-1 condition is broadcast here
        for name, v, c in (("masked_image", masked_image, 3), ("mask", mask, 1)):
            if not isinstance(v, torch.Tensor) or v.dim() != 4 or v.shape[1:] != (c, H, W) or v.shape[0] not in (1, B):
                raise ValueError(f"{name} must be [{B},{c},{H},{W}], got "
                                 f"{tuple(v.shape) if isinstance(v, torch.Tensor) else type(v)}")
        xx = self._dev_f32(x, dev, "x")
        mi = self._dev_f32(masked_image, dev, "masked_image").expand(B, 3, H, W).contiguous()
        mk = self._dev_f32(mask, dev, "mask").expand(B, 1, H, W).contiguous()
        tt = torch.as_tensor(t, device=dev).to(torch.int64).reshape(-1).expand(B).contiguous()
        out = torch.empty(B, self.cfg.out_channels, H, W, device=dev, dtype=torch.float32)
        h = self.handle(dev)
        L = _lib.lib()
        launch = lambda: _lib.check(L.ifd_unet_forward(  # noqa: E731
            h.h, _lib.ptr(xx), _lib.ptr(mi), _lib.ptr(mk), _lib.ptr(tt), B, H, W, _lib.ptr(out), _lib.stream_ptr(dev)))
        if self.guard == "lazy" and self.precision != "fp32" and self._deferred is None:
            self._lazy_forward(h, dev, launch)
        else:
            self.run_guarded(h, dev, launch)
        return out

    # -- the lazy range guard (module docstring) -------------------------------------------------
    _LZ_SLOTS = 8

    def _lazy_forward(self, h, dev, launch):
        L = _lib.lib()
        s = _lib.stream_ptr(dev)
        if self._lz is None or self._lz[0] is not h:
            if self._lz is not None:
                self.guard_check()  # the old handle's copies still pending are read (a trip there is reported)
            self._lz = [h, torch.zeros(self._LZ_SLOTS, dtype=torch.int32, pin_memory=True), [], 0, False]
        lz = self._lz
        self._lazy_poll(block=len(lz[2]) >= self._LZ_SLOTS)  # a full ring waits for its oldest copy
        if not lz[4]:  # armed once: the word is sticky, so one reset covers every later forward
            _lib.check(L.ifd_guard_reset(h.h, s))
            lz[4] = True
        launch()
        slot = lz[3]
        lz[3] = (slot + 1) % self._LZ_SLOTS
        _lib.check(L.ifd_guard_copy_async(h.h, ctypes.c_void_p(lz[1][slot:].data_ptr()), s))
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))
        lz[2].append((ev, slot))

    def _lazy_poll(self, block=False):
        """Look at the guard copies whose work has finished (all of them with block=True; the oldest one
        when the ring is full); raise on a trip."""
        lz = self._lz
        if lz is None:
            return
        pend = lz[2]
        while pend:
            ev, slot = pend[0]
            if block:
                ev.synchronize()
            elif not ev.query():
                break
            pend.pop(0)
            if int(lz[1][slot]):
                pend.clear()
                lz[4] = False  # re-armed (reset) by the next lazy forward
                self.guard_trips += 1
                raise RuntimeError("ifd: 3xf16 range guard tripped (a conv operand reached the f16 range) in an "
                                   "earlier forward; its output and the later ones are not fp32-accurate: re-run "
                                   "with precision='fp32' (or guard='sync', which recomputes each flagged forward)")
            block = False

    def guard_check(self):
        """Wait for every lazy guard copy and raise if any forward since the last check tripped."""
        lz = self._lz
        if lz is None:
            return
        while lz[2]:
            self._lazy_poll(block=True)

    def deferred_guard(self):
        """Context manager for a caller-driven loop of 3xf16 forwards (e.g. a reference script's own
        per-step algebra around `model(...)`): the range guard is reset once on entry and read once
        on exit instead of one stream sync per forward. A trip raises RuntimeError at exit (the
        forwards' outputs were already consumed, so the caller re-runs the loop, e.g. with
        precision="fp32"). Forwards inside the scope are not recomputed individually."""
        import contextlib

        @contextlib.contextmanager
        def scope():
            if self.precision == "fp32" or self._deferred is not None:
                yield
                return
            dev = self._handle_device or next(self.parameters()).device
            h = self.handle(dev)
            L = _lib.lib()
            s = _lib.stream_ptr(dev)
            self.guard_check()  # a lazy trip not yet seen is reported, not cleared by the reset
            _lib.check(L.ifd_guard_reset(h.h, s))
            # the scope's forwards may run on other streams: the reset (ordered on `s` only) lands first
            torch.cuda.synchronize(dev)
            if self._lz is not None:
                self._lz[4] = False
            self._deferred = dev
            try:
                yield
            finally:
                self._deferred = None
            # the scope's forwards may have been enqueued on other streams than `s`: wait for all of them
            # before the guard word is read (ifd_guard_read orders only after the work on `s`)
            torch.cuda.synchronize(dev)
            tripped = ctypes.c_int()
            _lib.check(L.ifd_guard_read(h.h, ctypes.byref(tripped), s))
            if tripped.value:
                self.guard_trips += 1
                raise RuntimeError("ifd: 3xf16 range guard tripped inside deferred_guard(); re-run in fp32")
        return scope()

    def run_guarded(self, h, dev, launch, before_retry=None):
        """Run `launch` (library calls on `h`); in 3xf16 mode check the range guard afterwards (one
        stream sync) and, if it tripped, call `before_retry` and run `launch` again in exact fp32.
        Inside deferred_guard() the check is left to the scope's exit."""
        if self.precision == "fp32" or self._deferred is not None:
            return launch()
        L = _lib.lib()
        s = _lib.stream_ptr(dev)
        self.guard_check()  # a lazy trip not yet seen is reported, not cleared by the reset
        _lib.check(L.ifd_guard_reset(h.h, s))
        if self._lz is not None:
            self._lz[4] = False
        res = launch()
        tripped = ctypes.c_int()
        _lib.check(L.ifd_guard_read(h.h, ctypes.byref(tripped), s))
        if not tripped.value:
            return res
        self.guard_trips += 1
        import warnings
        warnings.warn("ifd: 3xf16 range guard tripped (a conv operand reached the f16 range); recomputing in fp32")
        if before_retry is not None:
            before_retry()
        prec, self.precision = self.precision, "fp32"  # launch() may re-apply self.precision via handle()
        _lib.check(L.ifd_set_precision(h.h, _lib.PRECISIONS["fp32"]))
        try:
            return launch()
        finally:
            self.precision = prec
            _lib.check(L.ifd_set_precision(h.h, _lib.PRECISIONS[prec]))

    def memory(self):
        h = self._handle
        if h is None:
            return 0, 0
        a, b = ctypes.c_int64(), ctypes.c_int64()
        _lib.check(_lib.lib().ifd_memory(h.h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value


UNetModelHIP = DiffusionInpaintingModel
