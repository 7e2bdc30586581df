"""libifd.so loads, exports every symbol of include/ifd.h, and reports the reference's parameter list
(no GPU compute is issued here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "ifd.h")).read()
    return sorted(set(re.findall(r"\b(ifd_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_header_symbols():
    from ifd import _lib
    L = _lib.lib()
    syms = header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(_lib.EXPORTS)


@pytest.mark.parametrize("cfgname", ["REDUCED", "FULL"])
def test_param_inventory_matches_spec(cfgname):
    import ifd.topology as T
    from ifd.model import Handle
    cfg = getattr(T, cfgname)
    h = Handle(cfg)
    assert h.param_names() == [(k, tuple(s)) for k, s in T.state_dict_spec(cfg, prefix="")]


def test_bad_config_is_rejected():
    from ifd import _lib
    L = _lib.lib()
    c = _lib.IfdConfig()
    c.image_size = 64
    c.num_levels = 0
    h = ctypes.c_void_p()
    assert L.ifd_create(ctypes.byref(c), ctypes.byref(h)) != 0
    assert b"unsupported" in L.ifd_last_error()


def test_unknown_weight_name_is_an_error():
    from ifd import _lib
    from ifd.model import Handle
    from ifd.topology import REDUCED
    h = Handle(REDUCED)
    shape = (ctypes.c_int64 * 1)(3)
    buf = (ctypes.c_float * 3)()
    rc = _lib.lib().ifd_load_weights(h.h, b"nope.weight", ctypes.cast(buf, ctypes.c_void_p), shape, 1)
    assert rc != 0 and b"unexpected parameter" in _lib.lib().ifd_last_error()


def test_library_exports_train_header_symbols():
    """include/ifd_train.h (the training-step ops) is exported in full and bound by ifd.train."""
    src = open(os.path.join(ROOT, "include", "ifd_train.h")).read()
    syms = sorted(set(re.findall(r"\b(ifd_tr_[a-z_0-9]+)\s*\(", src)))
    assert len(syms) >= 20
    from ifd import train
    L = train.lib()
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(train.TRAIN_EXPORTS)


def test_train_host_helpers():
    """Split-K / workspace size queries need no GPU: the wgrad split covers the chip for small layers."""
    import ctypes as c
    from ifd import train
    L = train.lib()
    S = c.c_int()
    n = L.ifd_tr_wgrad_part_floats(128, 128, 9, 2 * 64 * 64, c.byref(S))
    assert S.value >= 2 and n == S.value * 128 * 128 * 9
    assert L.ifd_tr_attention_bwd_scratch_floats(2, 16, 128) == 2 * 2 * 2 * 16 * 16


@pytest.mark.parametrize("n_in,n_out", [(1024, 256), (300, 256), (64, 256), (256, 256), (31, 7)])
def test_resize_coeffs_match_oracle(n_in, n_out):
    """The library's Pillow-resample coefficients (host side, no GPU) equal the oracle's restatement,
    which tests/test_cpu_data_oracle.py pins to Pillow itself."""
    import numpy as np
    from ifd import _lib
    from oracle import ref_data
    b_ref, k_ref, ks_ref = ref_data.precompute_coeffs(n_in, n_out)
    L = _lib.lib()
    ks = ctypes.c_int()
    assert L.ifd_resize_coeffs(n_in, n_out, None, None, ctypes.byref(ks)) == 0 and ks.value == ks_ref
    b = np.zeros(2 * n_out, np.int32)
    k = np.zeros(n_out * ks.value, np.int32)
    assert L.ifd_resize_coeffs(n_in, n_out, b.ctypes.data_as(ctypes.c_void_p), k.ctypes.data_as(ctypes.c_void_p),
                               ctypes.byref(ks)) == 0
    assert np.array_equal(b.reshape(-1, 2), b_ref) and np.array_equal(k.reshape(n_out, -1), k_ref)


def test_workspace_plan_is_activation_bound():
    """The arena plan (host arithmetic, no GPU) reserves split-K slabs only for the (conv, resolution)
    pairs the plan runs: ~4.1 GB at B=16 and ~16.6 GB at B=64 for the full 256x256 model (round 2
    bounded every conv at every resolution: 67.9 GB at B=64, mostly qkv slabs sized for 256x256),
    growing linearly with the batch; the handle's own arena is untouched (still empty)."""
    from ifd import _lib
    from ifd.model import Handle
    from ifd.topology import FULL
    h = Handle(FULL)
    L = _lib.lib()
    got = {}
    for B in (1, 16, 64, 128):
        v = ctypes.c_int64()
        assert L.ifd_workspace_plan(h.h, B, ctypes.byref(v)) == 0
        got[B] = v.value
    assert got[16] <= 4.5e9 and got[64] <= 17.5e9
    assert abs(got[128] / got[64] - 2.0) < 0.02
    wb, ws = ctypes.c_int64(), ctypes.c_int64()
    assert L.ifd_memory(h.h, ctypes.byref(wb), ctypes.byref(ws)) == 0 and ws.value == 0
    assert L.ifd_workspace_plan(h.h, 0, ctypes.byref(ws)) != 0


def test_every_launch_status_sets_its_message():
    """Error contract (SURVEY §8(b) "Errors"): no entry point hands back a raw hipGetLastError() status without
    setting a message for it; hipGetLastError is read only by ifd::launch_status (csrc/common.h), which names the
    function it is called from."""
    csrc = os.path.join(ROOT, "face-inpainting-diffusion-models_amd", "csrc")
    offenders = []
    for fn in sorted(os.listdir(csrc)):
        if not fn.endswith((".hip", ".h")):
            continue
        for i, line in enumerate(open(os.path.join(csrc, fn)), 1):
            if "hipGetLastError" in line and not line.lstrip().startswith("//"):
                offenders.append(f"{fn}:{i}: {line.strip()}")
    assert offenders == ["common.h:20: const hipError_t e = hipGetLastError();"], offenders
    tr = open(os.path.join(csrc, "train_ops.hip")).read()
    assert "#define TR_LAST() IFD_LAUNCH_STATUS()" in tr


def test_check_reports_then_clears_the_message():
    """_lib.check raises with the failing entry's message and clears it, so a later status is never reported
    with this call's message (the round-5 stale 'shape not eligible' message of a status-700 fault)."""
    from ifd import _lib
    L = _lib.lib()
    rc = L.ifd_workspace_plan(None, 1, None)
    assert rc != 0
    with pytest.raises(RuntimeError, match="ifd_workspace_plan"):
        _lib.check(rc)
    assert L.ifd_last_error() == b""
    rc = L.ifd_tr_scale(None, 4, 1.0, None)
    with pytest.raises(RuntimeError, match="ifd_tr_scale: bad arguments"):
        _lib.check(rc)


def test_empty_batches_are_no_ops():
    """The elementwise entry points take an empty batch as a no-op (as torch does on empty tensors) instead of
    launching a zero-size grid, which HIP reports as a launch error; no GPU is touched."""
    from ifd import _lib
    L = _lib.lib()
    c = _lib.StepCoeffs()
    assert L.ifd_blend(None, None, None, 0, 3, 8, 8, None, None) == 0
    assert L.ifd_ddim_update(None, 0, 8, 8, None, None, None, None, None, ctypes.byref(c), None) == 0
    assert L.ifd_ddpm_update(None, 0, 8, 8, None, None, None, None, None, ctypes.byref(c), None) == 0
    assert L.ifd_to_u8(None, 0, 3, 8, 8, None, None) == 0
    assert L.ifd_blend(None, None, None, -1, 3, 8, 8, None, None) != 0
