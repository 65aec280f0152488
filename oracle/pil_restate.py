"""ORACLE (test infrastructure only): numpy restatement of the two Pillow
algorithms on the reference's transform path, pinned bit-exactly against
Pillow 12.2.0 (tests/test_oracle_pil.py):

* Image.resize(size, BILINEAR) — libImaging/Resample.c: precompute_coeffs
  (triangle filter, support 1 * max(scale, 1), bounds rounded with
  (int)(center +- support + 0.5)), normalize_coeffs_8bpc (22-bit fixed
  point, round half away from zero), horizontal pass then vertical pass,
  each accumulating from 1 << 21 and clipping `>> 22` to [0, 255].
* Image.rotate(angle, NEAREST, expand=False, fillcolor=0) — Image.rotate's
  matrix (round(cos/sin, 15), centre w/2, h/2) fed to
  libImaging/Geometry.c ImagingTransformAffine's 16.16 fixed-point walk
  (FIX(v) = floor(v*65536 + 0.5); xin = xx >> 16).
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 22


def resample_coeffs(in_size: int, out_size: int):
    """(bounds[out][2] = (xmin, count), int32 coeffs[out][ksize], ksize)"""
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
        ws = []
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            ws.append(1.0 - t if t < 1.0 else 0.0)
        ww = sum(ws)
        for x in range(xmax):
            kk[xx, x] = ws[x] / ww if ww != 0.0 else ws[x]
        bounds[xx] = (xmin, xmax)
    scaled = kk * (1 << PRECISION_BITS)
    ik = np.where(kk < 0, np.trunc(-0.5 + scaled), np.trunc(0.5 + scaled)).astype(np.int64)
    return bounds, ik.astype(np.int32), ksize


def _resample_axis(a: np.ndarray, bounds, ik, axis: int) -> np.ndarray:
    a = np.moveaxis(a, axis, 0).astype(np.int64)
    out = np.zeros((len(bounds),) + a.shape[1:], np.int64)
    for i, (xmin, n) in enumerate(bounds):
        ss = np.full(a.shape[1:], 1 << (PRECISION_BITS - 1), np.int64)
        for x in range(n):
            ss += a[xmin + x] * int(ik[i, x])
        out[i] = np.clip(ss >> PRECISION_BITS, 0, 255)
    return np.moveaxis(out.astype(np.uint8), 0, axis)


def resize_bilinear(img: np.ndarray, out_w: int, out_h: int) -> np.ndarray:
    """uint8 HxWxC -> uint8 out_h x out_w x C, Pillow-exact."""
    a = img
    h, w = a.shape[:2]
    if out_w != w:
        b, k, _ = resample_coeffs(w, out_w)
        a = _resample_axis(a, b, k, 1)
    if out_h != h:
        b, k, _ = resample_coeffs(h, out_h)
        a = _resample_axis(a, b, k, 0)
    return a


def rotate_params(angle: float, w: int, h: int):
    """(a0, a1, a3, a4, xo, yo) of Pillow's fixed-point affine walk."""
    angle = angle % 360.0
    cx, cy = w / 2, h / 2
    a = -math.radians(angle)
    m = [round(math.cos(a), 15), round(math.sin(a), 15), 0.0, round(-math.sin(a), 15), round(math.cos(a), 15), 0.0]
    m[2], m[5] = m[0] * (-cx) + m[1] * (-cy) + m[2], m[3] * (-cx) + m[4] * (-cy) + m[5]
    m[2] += cx
    m[5] += cy

    def fix(v):
        return int(math.floor(v * 65536.0 + 0.5))

    return (fix(m[0]), fix(m[1]), fix(m[3]), fix(m[4]), fix(m[2] + m[1] * 0.5 + m[0] * 0.5),
            fix(m[5] + m[4] * 0.5 + m[3] * 0.5))


def rotate_nearest(img: np.ndarray, angle: float) -> np.ndarray:
    h, w = img.shape[:2]
    if angle % 360.0 == 0.0:
        return img.copy()
    a0, a1, a3, a4, xo, yo = rotate_params(angle, w, h)
    y = np.arange(h, dtype=np.int64)[:, None]
    x = np.arange(w, dtype=np.int64)[None, :]
    xin = (xo + y * a1 + x * a0) >> 16
    yin = (yo + y * a4 + x * a3) >> 16
    ok = (xin >= 0) & (xin < w) & (yin >= 0) & (yin < h)
    out = np.zeros_like(img)
    out[ok] = img[yin[ok], xin[ok]]
    return out


def normalize(u8: np.ndarray, mean, std) -> np.ndarray:
    """ToTensor + Normalize in float32: HxWx3 uint8 -> 3xHxW float32."""
    t = u8.astype(np.float32).transpose(2, 0, 1) / np.float32(255)
    m = np.asarray(mean, np.float32)[:, None, None]
    s = np.asarray(std, np.float32)[:, None, None]
    return (t - m) / s
