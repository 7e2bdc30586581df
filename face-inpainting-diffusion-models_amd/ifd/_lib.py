"""ctypes binding of libifd.so (the C ABI declared in include/ifd.h).

The library is built in-tree (`make -C face-inpainting-diffusion-models_amd`, or
`__graft_entry__.build()`) and loaded AFTER torch so both share torch's HIP runtime
(same SONAME libamdhip64.so.7). There is no fallback: if the library is missing or fails to
load, every product entry point raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must be loaded first: provides the HIP runtime the library binds to)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("IFD_LIB_PATH") or os.path.join(_HERE, "libifd.so")  # override: dev ablation builds

c_i64p = ctypes.POINTER(ctypes.c_int64)


class IfdConfig(ctypes.Structure):
    _fields_ = [
        ("image_size", ctypes.c_int),
        ("in_channels", ctypes.c_int),
        ("model_channels", ctypes.c_int),
        ("out_channels", ctypes.c_int),
        ("num_res_blocks", ctypes.c_int),
        ("num_levels", ctypes.c_int),
        ("channel_mult", ctypes.c_int * 8),
        ("num_attention", ctypes.c_int),
        ("attention_ds", ctypes.c_int * 8),
        ("num_head_channels", ctypes.c_int),
    ]


class StepCoeffs(ctypes.Structure):
    _fields_ = [(n, ctypes.c_float) for n in (
        "c_sqrt_1m_at", "c_sqrt_at", "c_sqrt_ap", "c_dir", "c_sigma",
        "c_min_log", "c_max_log", "c_recip", "c_recipm1", "c_coef1", "c_coef2", "c_nonzero",
        "c_inj_a", "c_inj_b")] + [(n, ctypes.c_int) for n in ("use_noise", "inject", "clip", "pad")]


class LibCoeffs(ctypes.Structure):
    _fields_ = [(n, ctypes.c_float) for n in (
        "c_recip", "c_recipm1", "c_ab", "c_abp", "c_eta", "c_nonzero", "c_min_log", "c_max_log", "c_coef1",
        "c_coef2")] + [(n, ctypes.c_int) for n in ("clip", "pad")]


EXPORTS = {
    "ifd_create": (ctypes.c_int, [ctypes.POINTER(IfdConfig), ctypes.POINTER(ctypes.c_void_p)]),
    "ifd_destroy": (None, [ctypes.c_void_p]),
    "ifd_last_error": (ctypes.c_char_p, []),
    "ifd_clear_error": (None, []),
    "ifd_version": (ctypes.c_char_p, []),
    "ifd_profile_enable": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "ifd_profile_report": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64]),
    "ifd_profile_filter": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p]),
    "ifd_num_params": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
    "ifd_param_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), c_i64p,
                                      ctypes.POINTER(ctypes.c_int)]),
    "ifd_load_weights": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p, c_i64p, ctypes.c_int]),
    "ifd_finalize": (ctypes.c_int, [ctypes.c_void_p]),
    "ifd_memory": (ctypes.c_int, [ctypes.c_void_p, c_i64p, c_i64p]),
    "ifd_workspace_plan": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, c_i64p]),
    "ifd_set_option": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int]),
    "ifd_guard_reset": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "ifd_guard_read": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.c_void_p]),
    "ifd_guard_copy_async": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "ifd_get_option": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]),
    "ifd_set_precision": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "ifd_get_precision": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
    "ifd_unet_forward": (ctypes.c_int, [ctypes.c_void_p] + [ctypes.c_void_p] * 4 + [ctypes.c_int64, ctypes.c_int,
                                                                                      ctypes.c_int, ctypes.c_void_p,
                                                                                      ctypes.c_void_p]),
    "ifd_ddim_step": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int]
                      + [ctypes.c_void_p] * 5 + [ctypes.POINTER(StepCoeffs), ctypes.c_void_p]),
    "ifd_ddpm_step": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int]
                      + [ctypes.c_void_p] * 5 + [ctypes.POINTER(StepCoeffs), ctypes.c_void_p]),
    "ifd_ddim_update": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int]
                        + [ctypes.c_void_p] * 5 + [ctypes.POINTER(StepCoeffs), ctypes.c_void_p]),
    "ifd_ddpm_update": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int]
                        + [ctypes.c_void_p] * 5 + [ctypes.POINTER(StepCoeffs), ctypes.c_void_p]),
    "ifd_blend": (ctypes.c_int, [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                         ctypes.c_void_p, ctypes.c_void_p]),
    "ifd_to_u8": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_void_p, ctypes.c_void_p]),
    "ifd_mask_from_gray": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
    "ifd_lib_inject": (ctypes.c_int, [ctypes.c_void_p] * 4 + [ctypes.c_float, ctypes.c_float, ctypes.c_int64]
                       + [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_void_p]),
    "ifd_lib_update": (ctypes.c_int, [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                                                            ctypes.POINTER(LibCoeffs)]
                       + [ctypes.c_void_p] * 3),
    "ifd_resize_coeffs": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.POINTER(ctypes.c_int)]),
    "ifd_resize_u8_workspace": (ctypes.c_int64, [ctypes.c_int64] + [ctypes.c_int] * 5),
    "ifd_resize_u8": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64] + [ctypes.c_int] * 5
                      + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
    "ifd_image_to_float": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_void_p, ctypes.c_void_p]),
    "ifd_make_inpaint_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_void_p]),
}

# conv arithmetic modes (include/ifd.h IFD_PREC_*)
PRECISIONS = {"fp32": 0, "3xf16": 1, "f16": 2}

_lib = None


def lib():
    """Load libifd.so once; raise (never fall back) if it is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"ifd: HIP library not built ({LIB_PATH} missing); run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in EXPORTS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc):
    """Raise on a non-zero status with the message the failing entry point set (include/ifd.h: every non-zero
    status sets one naming its entry). The message is cleared once read, so it is never reported again for a
    later call's status."""
    if rc != 0:
        L = lib()
        msg = L.ifd_last_error()
        L.ifd_clear_error()
        raise RuntimeError(f"ifd: {msg.decode() if msg else 'error (no message set)'} (status {rc})")


def ptr(t):
    """Raw device pointer of a contiguous fp32/int64 tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_contiguous():  # (a raise, not an assert: python -O must not hand a strided tensor to the library)
        raise ValueError("ifd: tensors must be contiguous")
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
