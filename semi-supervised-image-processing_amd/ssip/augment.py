"""GPU input pipeline: Pillow-exact Resize / flip / rotate / ToTensor /
Normalize on uint8 batches (kernels in csrc/augment.hip).

Reference transforms:
  build_transforms  src/training/common.py:96-119
      train = Resize((S,S)) -> RandomHorizontalFlip -> RandomRotation(10)
              -> ToTensor -> Normalize
      eval  = Resize((S,S)) -> ToTensor -> Normalize
  build_transform   src/feature_extraction.py:184-207
      Resize(256) -> CenterCrop(224) -> ToTensor -> Normalize

The host keeps the part that is control, not data: Pillow's filter tables
(built here exactly as libImaging/Resample.c does) and the per-sample random
parameters, drawn with torchvision's RNG recipe (flip: ``torch.rand(1) <
0.5``; angle: ``torch.empty(1).uniform_(-10, 10)``) so a DataLoader worker
that draws them consumes the RNG exactly like the reference's transforms.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from .resnet import DeviceImages

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
PARAM_FIELDS = 16  # sizeof(ssip_aug_param) / 4


# ---------------------------------------------------------------------------
# Pillow tables
# ---------------------------------------------------------------------------
def resize_tables(in_size: int, out_size: int) -> Tuple[np.ndarray, np.ndarray, int]:
    """Pillow BILINEAR resample tables: bounds [out][2] (xmin, count),
    22-bit fixed-point coefficients [out][ksize] (libImaging/Resample.c
    precompute_coeffs + normalize_coeffs_8bpc)."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = filterscale  # bilinear filter support = 1.0
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int32)
    coeffs = np.zeros((out_size, ksize), np.int32)
    one = float(1 << 22)
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        inv = 1.0 / filterscale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = []
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * inv)
            w.append(1.0 - t if t < 1.0 else 0.0)
        tot = sum(w)
        for x in range(xmax):
            k = w[x] / tot if tot != 0.0 else w[x]
            coeffs[xx, x] = int(-0.5 + k * one) if k < 0 else int(0.5 + k * one)
        bounds[xx] = (xmin, xmax)
    return bounds, coeffs, ksize


def rotate_fixed_point(angle: float, w: int, h: int) -> Tuple[int, int, int, int, int, int]:
    """Image.rotate(angle, NEAREST, expand=False) -> the 16.16 terms
    (a0, a1, a3, a4, xo, yo) of libImaging/Geometry.c's affine walk."""
    angle = angle % 360.0
    cx, cy = w / 2, h / 2
    a = -math.radians(angle)
    m = [round(math.cos(a), 15), round(math.sin(a), 15), 0.0, round(-math.sin(a), 15), round(math.cos(a), 15), 0.0]
    m2 = m[0] * (-cx) + m[1] * (-cy) + m[2]
    m5 = m[3] * (-cx) + m[4] * (-cy) + m[5]
    m[2], m[5] = m2 + cx, m5 + cy

    def fix(v):
        return int(math.floor(v * 65536.0 + 0.5))

    return (fix(m[0]), fix(m[1]), fix(m[3]), fix(m[4]), fix(m[2] + m[1] * 0.5 + m[0] * 0.5),
            fix(m[5] + m[4] * 0.5 + m[3] * 0.5))


# ---------------------------------------------------------------------------
# per-sample parameters
# ---------------------------------------------------------------------------
@dataclass
class AugDraw:
    flip: bool = False
    angle: Optional[float] = None      # None = no rotation op in the pipeline
    brightness: float = 1.0
    contrast: float = 1.0
    cutout: Optional[Tuple[int, int, int, int]] = None  # x0, y0, x1, y1

    def encode(self, w: int, h: int) -> List[int]:
        p = [0] * PARAM_FIELDS
        p[0] = int(self.flip)
        if self.angle is not None and (self.angle % 360.0) != 0.0:
            p[1] = 1
            p[2:8] = rotate_fixed_point(self.angle, w, h)
        if self.brightness != 1.0 or self.contrast != 1.0:
            p[8] = 1
        p[9] = int(np.array(self.brightness, np.float32).view(np.int32))
        p[10] = int(np.array(self.contrast, np.float32).view(np.int32))
        if self.cutout is not None:
            p[11:15] = list(self.cutout)
        return p


def draw_train_params(degrees: float = 10.0, generator: Optional[torch.Generator] = None) -> AugDraw:
    """RandomHorizontalFlip(0.5) then RandomRotation(degrees), drawn exactly
    like torchvision (flip first, because it is first in the Compose)."""
    flip = bool(torch.rand(1, generator=generator) < 0.5)
    angle = float(torch.empty(1).uniform_(-degrees, degrees, generator=generator).item())
    return AugDraw(flip=flip, angle=angle)


def draw_strong_params(size: int, generator: Optional[torch.Generator] = None, degrees: float = 30.0,
                       jitter: float = 0.4, cut: float = 0.25) -> AugDraw:
    """Strong view for the consistency step (build extension, no reference):
    flip, rotation up to +-30 deg, brightness/contrast jitter, one cutout
    square of side cut*size."""
    flip = bool(torch.rand(1, generator=generator) < 0.5)
    angle = float(torch.empty(1).uniform_(-degrees, degrees, generator=generator).item())
    u = torch.rand(4, generator=generator)
    b = 1.0 + jitter * (2 * float(u[0]) - 1)
    c = 1.0 + jitter * (2 * float(u[1]) - 1)
    side = max(1, int(cut * size))
    x0 = int(float(u[2]) * (size - side))
    y0 = int(float(u[3]) * (size - side))
    return AugDraw(flip=flip, angle=angle, brightness=b, contrast=c, cutout=(x0, y0, x0 + side, y0 + side))


def encode_params(draws: Sequence[AugDraw], w: int, h: int) -> torch.Tensor:
    return torch.tensor([d.encode(w, h) for d in draws], dtype=torch.int32)


def draw_params_batch(n: int, size: int, strong: bool, generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """Vectorised parameter draw for synthetic batches (bench): same
    distributions as draw_train_params / draw_strong_params, fixed-point
    terms computed with numpy in float64 (the 15-digit rounding Pillow
    applies is skipped — irrelevant for synthetic inputs)."""
    deg = 30.0 if strong else 10.0
    flip = (torch.rand(n, generator=generator) < 0.5).numpy()
    ang = (torch.rand(n, generator=generator, dtype=torch.float64) * 2 * deg - deg).numpy()
    a = -np.radians(ang % 360.0)
    c, s_ = np.cos(a), np.sin(a)
    cx = cy = size / 2
    m2 = c * (-cx) + s_ * (-cy) + cx
    m5 = -s_ * (-cx) + c * (-cy) + cy

    def fix(v):
        return np.floor(v * 65536.0 + 0.5).astype(np.int64)

    p = np.zeros((n, PARAM_FIELDS), np.int64)
    p[:, 0] = flip
    p[:, 1] = 1
    p[:, 2], p[:, 3], p[:, 4], p[:, 5] = fix(c), fix(s_), fix(-s_), fix(c)
    p[:, 6] = fix(m2 + s_ * 0.5 + c * 0.5)
    p[:, 7] = fix(m5 + c * 0.5 - s_ * 0.5)
    one = np.array(1.0, np.float32).view(np.int32)
    p[:, 9] = one
    p[:, 10] = one
    if strong:
        u = torch.rand(n, 4, generator=generator).numpy()
        p[:, 8] = 1
        p[:, 9] = (1.0 + 0.4 * (2 * u[:, 0] - 1)).astype(np.float32).view(np.int32)
        p[:, 10] = (1.0 + 0.4 * (2 * u[:, 1] - 1)).astype(np.float32).view(np.int32)
        side = max(1, int(0.25 * size))
        x0 = (u[:, 2] * (size - side)).astype(np.int64)
        y0 = (u[:, 3] * (size - side)).astype(np.int64)
        p[:, 11], p[:, 12], p[:, 13], p[:, 14] = x0, y0, x0 + side, y0 + side
    return torch.from_numpy(p.astype(np.int32))


# ---------------------------------------------------------------------------
# the transform
# ---------------------------------------------------------------------------
class GpuTransform:
    """uint8 [B,H,W,3] (device) -> DeviceImages (NHWC4, dtype).

    mode "resize":  Resize((size,size)) [+ per-sample flip/rotate params]
    mode "short":   Resize(short side -> resize) + CenterCrop(crop)
    """

    def __init__(self, size: int = 224, dtype: torch.dtype = torch.float32, mode: str = "resize",
                 resize: int = 256, crop: int = 224, mean=IMAGENET_MEAN, std=IMAGENET_STD, pad: int = 3):
        # pad: zero border written around each image (the stem conv's padding, pre-applied)
        self.size, self.dtype, self.mode, self.pad = size, dtype, mode, pad
        self.resize, self.crop = resize, crop
        import ctypes

        self._mean_arr = (ctypes.c_float * 3)(*[float(v) for v in mean])
        self._std_arr = (ctypes.c_float * 3)(*[float(v) for v in std])
        # passed as the ctypes arrays (host pointers): a launch plan copies them
        self.mean = self._mean_arr
        self.std = self._std_arr
        self._tables: Dict[Tuple[int, int, str], Tuple[torch.Tensor, torch.Tensor, int]] = {}

    def _table(self, n_in: int, n_out: int, dev) -> Tuple[torch.Tensor, torch.Tensor, int]:
        key = (n_in, n_out, str(dev))
        t = self._tables.get(key)
        if t is None:
            b, c, k = resize_tables(n_in, n_out)
            t = (torch.from_numpy(b).to(dev), torch.from_numpy(c).to(dev), k)
            self._tables[key] = t
        return t

    def geometry(self, H: int, W: int) -> Tuple[int, int, int, int, int, int]:
        """(Hr, Wr, Ho, Wo, crop_x, crop_y) for a source of H x W."""
        if self.mode == "resize":
            return self.size, self.size, self.size, self.size, 0, 0
        s = self.resize
        if W <= H:
            Wr, Hr = s, int(s * H / W)
        else:
            Hr, Wr = s, int(s * W / H)
        c = self.crop
        return Hr, Wr, c, c, int(round((Wr - c) / 2.0)), int(round((Hr - c) / 2.0))

    def __call__(self, images: torch.Tensor, params: Optional[torch.Tensor] = None,
                 out: Optional[torch.Tensor] = None) -> DeviceImages:
        if images.dtype != torch.uint8 or images.dim() != 4 or images.shape[-1] != 3:
            raise ValueError("GpuTransform expects uint8 [B,H,W,3]")
        if not images.is_cuda:
            raise ValueError("GpuTransform expects a device tensor")
        images = images.contiguous()
        B, H, W, _ = images.shape
        dev = images.device
        Hr, Wr, Ho, Wo, cx, cy = self.geometry(H, W)
        stream = torch.cuda.current_stream().cuda_stream
        src, src_h, src_w = images, H, W
        bstride = H * W * 3
        if Wr != W:
            bh, ch, kh = self._table(W, Wr, dev)
            tmp = torch.empty((B, H, Wr, 3), device=dev, dtype=torch.uint8)
            _lib.call("ssip_resize_h_u8", B, _lib.ptr(images), bstride, H, W, Wr, kh, _lib.ptr(bh), _lib.ptr(ch),
                      _lib.ptr(tmp), stream)
            src, src_w, bstride = tmp, Wr, H * Wr * 3
        kv, bv, cv = 0, None, None
        if Hr != H:
            bv, cv, kv = self._table(H, Hr, dev)
        p = self.pad
        shape = (B, Ho + 2 * p, Wo + 2 * p, 4)
        if out is None:
            out = torch.empty(shape, device=dev, dtype=self.dtype)
        elif tuple(out.shape) != shape or out.dtype != self.dtype or not out.is_contiguous():
            raise ValueError(f"GpuTransform: `out` must be a contiguous {shape} {self.dtype} buffer")
        pptr = None
        if params is not None:
            params = params.to(dev, torch.int32).contiguous()
            assert params.shape == (B, PARAM_FIELDS)
            pptr = _lib.ptr(params)
        _lib.call("ssip_augment_u8", _lib.F32 if self.dtype == torch.float32 else _lib.BF16, B, _lib.ptr(src),
                  bstride, src_h, src_w, Hr, Wr, Ho, Wo, cx, cy, kv, None if bv is None else _lib.ptr(bv),
                  None if cv is None else _lib.ptr(cv), pptr, self.mean, self.std, p, _lib.ptr(out), stream)
        return DeviceImages(out, p)


def to_nchw(images: DeviceImages) -> torch.Tensor:
    """NHWC4 -> f32 NCHW [B,3,H,W] (for comparisons with the reference tensor contract)."""
    return images.nhwc4[..., :3].permute(0, 3, 1, 2).float().contiguous()
