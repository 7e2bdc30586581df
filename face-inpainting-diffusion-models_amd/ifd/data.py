"""Data formats either side of the sampler, on the HIP library.

* `toU8` mirrors code/test_inp_ddim_50.py:33-41: [B,C,H,W] float in [-1,1] -> numpy uint8 [B,H,W,C]
  (None passes through; CPU or non-fp32 inputs are moved to the GPU as fp32 first — the
  conversion itself always runs on the HIP kernel). `to_u8_device` keeps the result on the GPU.
* `mask_from_gray` is the mask convention of OrderedMaskDataset (code/data/dataset.py:278-286):
  a grayscale uint8 mask, already resized, -> fp32 mask, 1 = hole (black), 0 = keep (white).
  `masked_image` is image * (1 - mask) (dataset.py:289), the same arithmetic as model_fn.
* `resize_u8` / `images_to_float` / `OrderedMaskBank`: the dataset's Resize (Pillow BILINEAR,
  bit-exact), ToTensor + Normalize, ordered mask cycling, mask rule and masked image, on the device.
Image file decode stays on the host (out of scope).
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


def toU8(sample, device=None):
    """Like the reference's toU8, any float dtype and any device: the tensor is moved to the GPU
    (`device`, default the current one) as fp32 and converted there by the HIP kernel."""
    if sample is None:
        return sample
    x = sample.detach()
    if not x.is_cuda or x.dtype != torch.float32:
        x = x.to(device=device if device is not None else ("cuda" if not x.is_cuda else x.device),
                 dtype=torch.float32)
    return to_u8_device(x).cpu().numpy()


def mask_from_gray(gray: torch.Tensor) -> torch.Tensor:
    """gray: uint8 tensor of any shape (e.g. [B,1,H,W]) -> float32 mask of the same shape."""
    _need_gpu(gray, "mask_from_gray")
    if gray.dtype != torch.uint8:
        raise ValueError("ifd.data.mask_from_gray: expects a uint8 tensor")
    g = gray.contiguous()
    out = torch.empty(g.shape, dtype=torch.float32, device=g.device)
    _lib.check(_lib.lib().ifd_mask_from_gray(_lib.ptr(g), g.numel(), _lib.ptr(out), _lib.stream_ptr(g.device)))
    return out


# ---- input side: dataset transforms on the device (code/data/dataset.py:231-240, 273-286) ----------

def resize_u8(img: torch.Tensor, out_h: int, out_w: int) -> torch.Tensor:
    """Pillow BILINEAR resample (torchvision Resize((out_h, out_w)) of a PIL image), bit-exact.
    img: uint8 GPU tensor [N,H,W,C] (or [N,H,W] for grayscale) -> same layout at (out_h, out_w)."""
    _need_gpu(img, "resize_u8")
    if img.dtype != torch.uint8 or img.dim() not in (3, 4):
        raise ValueError("ifd.data.resize_u8: expects a uint8 [N,H,W] or [N,H,W,C] tensor")
    x = img.contiguous()
    gray = x.dim() == 3
    N, H, W = x.shape[:3]
    C = 1 if gray else x.shape[3]
    L = _lib.lib()
    out = torch.empty((N, out_h, out_w) + (() if gray else (C,)), dtype=torch.uint8, device=x.device)
    wb = L.ifd_resize_u8_workspace(N, C, H, W, out_h, out_w)
    work = torch.empty(max(wb, 1), dtype=torch.uint8, device=x.device)
    _lib.check(L.ifd_resize_u8(_lib.ptr(x), N, C, H, W, out_h, out_w, _lib.ptr(out), _lib.ptr(work), wb,
                               _lib.stream_ptr(x.device)))
    return out


def images_to_float(img: torch.Tensor) -> torch.Tensor:
    """ToTensor + Normalize([0.5]*3, [0.5]*3): uint8 [N,H,W,C] -> float32 [N,C,H,W] in [-1, 1]."""
    _need_gpu(img, "images_to_float")
    if img.dtype != torch.uint8 or img.dim() != 4:
        raise ValueError("ifd.data.images_to_float: expects a uint8 [N,H,W,C] tensor")
    x = img.contiguous()
    N, H, W, C = x.shape
    out = torch.empty((N, C, H, W), dtype=torch.float32, device=x.device)
    _lib.check(_lib.lib().ifd_image_to_float(_lib.ptr(x), N, C, H, W, _lib.ptr(out), _lib.stream_ptr(x.device)))
    return out


class OrderedMaskBank:
    """OrderedMaskDataset's masks (code/data/dataset.py:191-295) resident on the GPU: decoded once
    (grayscale 'L', host), resized on the device (Pillow BILINEAR, bit-exact), then every batch
    takes mask idx % M (ordered cycling, :273-274), the threshold rule (:283) and
    masked_image = image * (1 - mask) (:286) in one kernel."""

    def __init__(self, masks_u8, img_size=256, device="cuda"):
        """masks_u8: a list of HxW uint8 arrays / tensors (any sizes, e.g. decoded mask files) or a
        uint8 [M,H,W] tensor."""
        dev = torch.device(device)
        if isinstance(masks_u8, torch.Tensor) and masks_u8.dim() == 3:
            items = [masks_u8[i] for i in range(masks_u8.shape[0])]
        else:
            items = list(masks_u8)
        if not items:
            raise ValueError("OrderedMaskBank: no masks")
        bank = []
        for m in items:
            t = torch.as_tensor(m, dtype=torch.uint8).to(dev)
            if t.dim() != 2:
                raise ValueError("OrderedMaskBank: masks must be 2-D grayscale")
            bank.append(resize_u8(t[None], img_size, img_size)[0])
        self.bank = torch.stack(bank).contiguous()
        self.img_size = img_size

    @classmethod
    def from_files(cls, paths, img_size=256, device="cuda"):
        from PIL import Image  # decode only (host); resize happens on the device
        import numpy as np
        return cls([np.asarray(Image.open(p).convert("L")) for p in sorted(paths)], img_size, device)

    def __len__(self):
        return self.bank.shape[0]

    def batch(self, images: torch.Tensor, indices):
        """images [N,3,S,S] fp32 (GPU), indices [N] dataset indices -> the dataset's dict entries."""
        _need_gpu(images, "OrderedMaskBank.batch")
        x = images.to(torch.float32).contiguous()
        N, C, H, W = x.shape
        if C != 3 or (H, W) != (self.img_size, self.img_size):
            raise ValueError(f"images must be [N,3,{self.img_size},{self.img_size}], got {tuple(x.shape)}")
        idx = torch.as_tensor(indices, dtype=torch.int64, device=x.device).reshape(-1).contiguous()
        if idx.numel() != N:
            raise ValueError("one index per image")
        mask = torch.empty((N, 1, H, W), dtype=torch.float32, device=x.device)
        masked = torch.empty_like(x)
        _lib.check(_lib.lib().ifd_make_inpaint_batch(_lib.ptr(x), N, H, W, _lib.ptr(self.bank), len(self), _lib.ptr(idx),
                                                     _lib.ptr(mask), _lib.ptr(masked), _lib.stream_ptr(x.device)))
        return {"image": x, "masked_image": masked, "mask": mask, "mask_idx": idx % len(self)}
