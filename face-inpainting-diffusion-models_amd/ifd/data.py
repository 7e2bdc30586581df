"""Data formats either side of the sampler, on the HIP library.

* `toU8` mirrors code/test_inp_ddim_50.py:33-41: [B,C,H,W] fp32 in [-1,1] -> numpy uint8 [B,H,W,C]
  (None passes through). `to_u8_device` keeps the result on the GPU.
* `mask_from_gray` is the mask convention of OrderedMaskDataset (code/data/dataset.py:278-286):
  a grayscale uint8 mask, already resized, -> fp32 mask, 1 = hole (black), 0 = keep (white).
  `masked_image` is image * (1 - mask) (dataset.py:289), the same arithmetic as model_fn.
Image decode and PIL resize stay on the host (out of scope).
"""
from __future__ import annotations

import torch

from . import _lib


def _need_gpu(t, name):
    if not t.is_cuda:
        raise RuntimeError(f"ifd.data.{name}: expects a GPU tensor (no CPU path)")


def to_u8_device(sample: torch.Tensor) -> torch.Tensor:
    _need_gpu(sample, "to_u8_device")
    if sample.dtype != torch.float32 or sample.dim() != 4:
        raise ValueError("ifd.data.to_u8_device: expects a [B,C,H,W] float32 tensor")
    x = sample.contiguous()
    B, C, H, W = x.shape
    out = torch.empty((B, H, W, C), dtype=torch.uint8, device=x.device)
    _lib.check(_lib.lib().ifd_to_u8(_lib.ptr(x), B, C, H, W, _lib.ptr(out), _lib.stream_ptr(x.device)))
    return out


def toU8(sample):
    if sample is None:
        return sample
    return to_u8_device(sample.detach()).cpu().numpy()


def mask_from_gray(gray: torch.Tensor) -> torch.Tensor:
    """gray: uint8 tensor of any shape (e.g. [B,1,H,W]) -> float32 mask of the same shape."""
    _need_gpu(gray, "mask_from_gray")
    if gray.dtype != torch.uint8:
        raise ValueError("ifd.data.mask_from_gray: expects a uint8 tensor")
    g = gray.contiguous()
    out = torch.empty(g.shape, dtype=torch.float32, device=g.device)
    _lib.check(_lib.lib().ifd_mask_from_gray(_lib.ptr(g), g.numel(), _lib.ptr(out), _lib.stream_ptr(g.device)))
    return out
