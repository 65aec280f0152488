"""ORACLE restatement of torchvision.transforms for PIL inputs.

Each transform delegates to the same Pillow call torchvision makes
(torchvision/transforms/functional_pil.py), with torchvision's RNG recipe:
RandomHorizontalFlip draws `torch.rand(1) < p`; RandomRotation draws
`float(torch.empty(1).uniform_(-d, d).item())` (flip is drawn first when
both are in a Compose, because it comes first).
"""
from __future__ import annotations

import numbers
from typing import Sequence

import numpy as np
import torch
from PIL import Image


class Compose:
    def __init__(self, transforms):
        self.transforms = list(transforms)

    def __call__(self, img):
        for t in self.transforms:
            img = t(img)
        return img


class InterpolationMode:
    NEAREST = "nearest"
    BILINEAR = "bilinear"


_PIL_INTERP = {InterpolationMode.NEAREST: Image.NEAREST, InterpolationMode.BILINEAR: Image.BILINEAR}


def _resized_size(w, h, size):
    if isinstance(size, numbers.Number) or (isinstance(size, Sequence) and len(size) == 1):
        s = int(size if isinstance(size, numbers.Number) else size[0])
        short, long = (w, h) if w <= h else (h, w)
        new_short, new_long = s, int(s * long / short)
        return (new_short, new_long) if w <= h else (new_long, new_short)  # (w, h)
    h2, w2 = size
    return (int(w2), int(h2))


class Resize:
    def __init__(self, size, interpolation=InterpolationMode.BILINEAR, max_size=None, antialias=True):
        self.size = size
        self.interpolation = interpolation

    def __call__(self, img):
        w, h = img.size
        ow, oh = _resized_size(w, h, self.size)
        if (ow, oh) == (w, h):
            return img
        return img.resize((ow, oh), _PIL_INTERP[self.interpolation])


class CenterCrop:
    def __init__(self, size):
        self.size = (int(size), int(size)) if isinstance(size, numbers.Number) else tuple(size)

    def __call__(self, img):
        w, h = img.size
        th, tw = self.size
        top = int(round((h - th) / 2.0))
        left = int(round((w - tw) / 2.0))
        return img.crop((left, top, left + tw, top + th))


class RandomHorizontalFlip:
    def __init__(self, p=0.5):
        self.p = p

    def __call__(self, img):
        if torch.rand(1) < self.p:
            return img.transpose(Image.FLIP_LEFT_RIGHT)
        return img


class RandomRotation:
    def __init__(self, degrees, interpolation=InterpolationMode.NEAREST, expand=False, center=None, fill=0):
        if isinstance(degrees, numbers.Number):
            degrees = (-degrees, degrees)
        self.degrees = [float(d) for d in degrees]
        self.interpolation = interpolation
        self.expand = expand
        self.center = center
        self.fill = fill

    @staticmethod
    def get_params(degrees):
        return float(torch.empty(1).uniform_(float(degrees[0]), float(degrees[1])).item())

    def __call__(self, img):
        angle = self.get_params(self.degrees)
        n = len(img.getbands())
        fill = self.fill
        fill = tuple([float(fill)] * n) if isinstance(fill, (int, float)) else tuple(fill)
        if img.mode != "F":
            fill = tuple(int(f) for f in fill) if n > 1 else int(fill[0])
        return img.rotate(angle, _PIL_INTERP[self.interpolation], self.expand, self.center, fillcolor=fill)


class ToTensor:
    def __call__(self, pic):
        a = np.array(pic, np.uint8, copy=True)
        if a.ndim == 2:
            a = a[:, :, None]
        t = torch.from_numpy(a).permute(2, 0, 1).contiguous()
        return t.to(dtype=torch.float32).div(255)


class Normalize:
    def __init__(self, mean, std, inplace=False):
        self.mean, self.std = mean, std

    def __call__(self, t):
        mean = torch.as_tensor(self.mean, dtype=t.dtype).view(-1, 1, 1)
        std = torch.as_tensor(self.std, dtype=t.dtype).view(-1, 1, 1)
        return t.sub(mean).div(std)
