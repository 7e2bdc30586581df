"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the data formats on either side of the sampler:

  * PIL's BILINEAR resample of 8-bit images, which torchvision's `transforms.Resize((s, s))`
    applies to the dataset's PIL images (code/data/dataset.py:231-240: masks, then images):
    Pillow's Resample.c algorithm — per output pixel a triangle filter of support max(1, scale)
    centred at (x + 0.5) * scale, normalised, converted to 22-bit fixed point, horizontal pass
    over the needed rows then vertical pass, each rounding to uint8 (ImagingResampleInner).
    The third-party dependency is Pillow (installed here: 12.2.0); `resize_u8` is checked against
    PIL.Image.resize itself in tests/test_cpu_data_oracle.py.
  * ToTensor + Normalize([0.5]*3, [0.5]*3) (dataset.py:238-240), the mask rule
    `(mask < 0.5).float()` and `masked_image = image * (1 - mask)` (dataset.py:283-286), and the
    ordered mask cycling `mask_idx = idx % len(mask_paths)` (dataset.py:273-274).

Only tests/ may import this module.
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2


def _bilinear(x):
    x = abs(x)
    return 1.0 - x if x < 1.0 else 0.0


def precompute_coeffs(in_size, out_size, in0=0.0, in1=None):
    """Resample.c precompute_coeffs + normalize_coeffs_8bpc: (bounds [out][2], int coeffs [out][ksize], ksize)."""
    in1 = float(in_size) if in1 is None else in1
    scale = (in1 - in0) / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int64)
    kk = np.zeros((out_size, ksize), np.int64)
    for xx in range(out_size):
        center = in0 + (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = int(center - support + 0.5)
        xmin = max(xmin, 0)
        xmax = int(center + support + 0.5)
        xmax = min(xmax, in_size) - xmin
        w = [_bilinear((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = sum(w)
        if ww != 0.0:
            w = [v / ww for v in w]
        for x, v in enumerate(w):
            kk[xx, x] = int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else int(0.5 + v * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return bounds, kk, ksize


def _clip8(v):
    v = v >> PRECISION_BITS
    return np.clip(v, 0, 255)


def _pass(img, bounds, kk, axis):
    """One 8bpc pass along `axis` (1 = horizontal over width, 0 = vertical over height), HWC uint8."""
    img = img.astype(np.int64)
    out_n = bounds.shape[0]
    if axis == 1:
        out = np.empty((img.shape[0], out_n, img.shape[2]), np.int64)
        for xx in range(out_n):
            xmin, xmax = bounds[xx]
            ss = np.full((img.shape[0], img.shape[2]), 1 << (PRECISION_BITS - 1), np.int64)
            for x in range(xmax):
                ss += img[:, xmin + x, :] * kk[xx, x]
            out[:, xx, :] = _clip8(ss)
    else:
        out = np.empty((out_n, img.shape[1], img.shape[2]), np.int64)
        for yy in range(out_n):
            ymin, ymax = bounds[yy]
            ss = np.full((img.shape[1], img.shape[2]), 1 << (PRECISION_BITS - 1), np.int64)
            for y in range(ymax):
                ss += img[ymin + y, :, :] * kk[yy, y]
            out[yy] = _clip8(ss)
    return out.astype(np.uint8)


def resize_u8(img, out_h, out_w):
    """PIL Image.resize((out_w, out_h), BILINEAR) of an HWC (or HW) uint8 array (ImagingResampleInner)."""
    squeeze = img.ndim == 2
    if squeeze:
        img = img[:, :, None]
    H, W = img.shape[:2]
    if (H, W) == (out_h, out_w):
        out = img.copy()
        return out[:, :, 0] if squeeze else out
    bh, kh, _ = precompute_coeffs(W, out_w)
    bv, kv, _ = precompute_coeffs(H, out_h)
    need_h = out_w != W
    need_v = out_h != H
    cur = img
    if need_h:
        y_first = bv[0, 0]
        y_last = bv[-1, 0] + bv[-1, 1]
        bv = bv.copy()
        bv[:, 0] -= y_first
        cur = _pass(img[y_first:y_last], bh, kh, axis=1)
    if need_v:
        cur = _pass(cur, bv, kv, axis=0)
    return cur[:, :, 0] if squeeze else cur


def to_tensor_normalize(img_hwc_u8):
    """ToTensor + Normalize(0.5, 0.5): CHW float32 in [-1, 1] with torchvision's fp32 arithmetic."""
    x = img_hwc_u8.astype(np.float32).transpose(2, 0, 1) / np.float32(255)
    return (x - np.float32(0.5)) / np.float32(0.5)


def mask_rule(gray_u8):
    """ToTensor then (mask < 0.5).float(): 1 = hole (black)."""
    return ((gray_u8.astype(np.float32) / np.float32(255)) < np.float32(0.5)).astype(np.float32)


def ordered_mask_index(idx, n_masks):
    return idx % n_masks
