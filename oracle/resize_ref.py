"""PIL bilinear resize restated in NumPy (ORACLE -- test infrastructure only).

The reference's input contract is ``transforms.Resize(img_size)`` on the PIL image
(``src/data/datasets/speed.py:66-69``, image opened and ``.convert("RGB")`` at ``src/data/utils.py:215``),
which for a PIL input is ``Image.resize(size, BILINEAR)`` (torchvision functional_pil.resize; reducing_gap
None). Pillow's ``ImagingResample`` (libImaging/Resample.c) computes, per axis,

  scale = in / out; filterscale = max(scale, 1); support = 1.0 * filterscale
  center = (x + 0.5) * scale; xmin = max(int(center - support + 0.5), 0); xmax = min(int(center + support + 0.5), in)
  w_i = max(0, 1 - |(i + xmin - center + 0.5) / filterscale|), normalised to sum 1   (float64)
  k_i = int(w_i * 2**22 + 0.5) (or - 0.5 for negative w)                            (PRECISION_BITS = 22)
  out = clip8((2**21 + sum_i in_i k_i) >> 22)

horizontally over the source rows the vertical pass needs (``ybox_first .. ybox_last``) into an 8-bit
temporary image, then vertically. ``pil_resize`` mirrors that exactly (checked against Pillow itself in
tests/test_resize_oracle.py); the MI355X kernel (csrc/k_pre.hip) uses the same integer tables.
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 22


def coeffs(in_size: int, out_size: int):
    """-> (bounds int32 [out][2] = (xmin, count), k int32 [out][ksize]) as Pillow's precompute_coeffs +
    normalize_coeffs_8bpc compute them."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int32)
    kk = np.zeros((out_size, ksize), np.float64)
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = int(center - support + 0.5)
        xmin = max(xmin, 0)
        xmax = int(center + support + 0.5)
        xmax = min(xmax, in_size) - xmin
        ww = 0.0
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            w = 1.0 - t if t < 1.0 else 0.0
            kk[xx, x] = w
            ww += w
        if ww != 0.0:
            kk[xx, :xmax] /= ww
        bounds[xx] = (xmin, xmax)
    ki = np.where(kk < 0, np.trunc(-0.5 + kk * (1 << PRECISION_BITS)),
                  np.trunc(0.5 + kk * (1 << PRECISION_BITS))).astype(np.int64)
    return bounds, ki


def _pass(img: np.ndarray, bounds, k, axis: int) -> np.ndarray:
    """One resampling pass along ``axis`` (0 = rows/vertical, 1 = columns/horizontal) of an HxWxC uint8."""
    src = np.moveaxis(img.astype(np.int64), axis, 0)
    out = np.empty((bounds.shape[0],) + src.shape[1:], np.uint8)
    for o in range(bounds.shape[0]):
        xmin, n = bounds[o]
        acc = np.full(src.shape[1:], 1 << (PRECISION_BITS - 1), np.int64)
        for i in range(n):
            acc += src[xmin + i] * k[o, i]
        out[o] = np.clip(acc >> PRECISION_BITS, 0, 255)
    return np.moveaxis(out, 0, axis)


def pil_resize(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """HxWx3 uint8 -> out_h x out_w x 3 uint8, bit-identical to ``Image.fromarray(img).resize((w, h), BILINEAR)``."""
    h, w = img.shape[:2]
    bh, kh = coeffs(w, out_w)
    bv, kv = coeffs(h, out_h)
    need_h, need_v = out_w != w, out_h != h
    if need_h:
        y0 = int(bv[0, 0])
        y1 = int(bv[-1, 0] + bv[-1, 1])
        img = _pass(img[y0:y1], bh, kh, 1)
        bv = bv.copy()
        bv[:, 0] -= y0
    if need_v:
        img = _pass(img, bv, kv, 0)
    return img
