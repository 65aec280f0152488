"""Host data plumbing for the GPU input pipeline.

The reference decodes JPEGs and runs the whole torchvision transform chain
inside DataLoader worker processes (src/training/common.py:126-194, 249-292)
and ships f32 [B,3,S,S] batches to the device.  Here the workers only decode
(PIL) and draw the per-sample random parameters with torchvision's RNG
recipe (so the parameters are the ones the reference would have drawn); the
batch crosses PCIe as uint8 (786 KB per 512x512 image instead of 602 KB of
f32 per 224x224 view) and ``HostImageBatch.to(device)`` runs the
Pillow-exact resize/flip/rotate/normalize kernels (ssip.augment).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
from PIL import Image

from .augment import PARAM_FIELDS, AugDraw, GpuTransform, draw_train_params

IMG_EXTENSIONS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")


def pil_loader(path) -> Image.Image:
    with open(path, "rb") as f:
        img = Image.open(f)
        return img.convert("RGB")


class ImageFolder:
    """torchvision.datasets.ImageFolder semantics: sorted class folders ->
    indices, files gathered with sorted os.walk, extension filter, RGB
    loader (used by the reference at src/training/common.py:258)."""

    def __init__(self, root, transform=None, loader=pil_loader):
        self.root = os.fspath(root)
        classes = sorted(e.name for e in os.scandir(self.root) if e.is_dir())
        if not classes:
            raise FileNotFoundError(f"Couldn't find any class folder in {self.root}.")
        self.classes = classes
        self.class_to_idx = {c: i for i, c in enumerate(classes)}
        samples = []
        for c in classes:
            for r, _, files in sorted(os.walk(os.path.join(self.root, c), followlinks=True)):
                for fn in sorted(files):
                    p = os.path.join(r, fn)
                    if p.lower().endswith(IMG_EXTENSIONS):
                        samples.append((p, self.class_to_idx[c]))
        self.samples = samples
        self.imgs = samples
        self.targets = [s[1] for s in samples]
        self.transform = transform
        self.loader = loader

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, i):
        path, target = self.samples[i]
        img = self.loader(path)
        if self.transform is not None:
            img = self.transform(img)
        return img, target


# ---------------------------------------------------------------------------
# transform specs: callable on a PIL image in the worker; the heavy part is
# deferred to the device
# ---------------------------------------------------------------------------
@dataclass
class HostImage:
    pixels: torch.Tensor   # uint8 [H,W,3]
    params: torch.Tensor   # int32 [PARAM_FIELDS]


class DeviceTransformSpec:
    """Mirror of one torchvision Compose of the reference.

    kind "train":   Resize((S,S)) -> RandomHorizontalFlip -> RandomRotation(deg) -> ToTensor -> Normalize
    kind "eval":    Resize((S,S)) -> ToTensor -> Normalize
    kind "extract": Resize(resize) -> CenterCrop(crop) -> ToTensor -> Normalize
    """

    def __init__(self, kind: str, size: int = 224, degrees: float = 10.0, resize: int = 256, crop: int = 224):
        if kind not in ("train", "eval", "extract"):
            raise ValueError(kind)
        self.kind, self.size, self.degrees, self.resize, self.crop = kind, size, degrees, resize, crop

    def __call__(self, img: Image.Image) -> HostImage:
        a = np.array(img)
        if a.ndim == 2:
            a = np.stack([a] * 3, -1)
        if a.shape[-1] != 3:
            raise ValueError(f"expected an RGB image, got mode {img.mode}")
        draw = draw_train_params(self.degrees) if self.kind == "train" else AugDraw()
        s = self.size if self.kind != "extract" else self.crop
        g = self.size if self.kind != "extract" else None
        p = torch.tensor(draw.encode(g or s, g or s), dtype=torch.int32)
        return HostImage(torch.from_numpy(np.ascontiguousarray(a)), p)

    def gpu(self, dtype: torch.dtype) -> GpuTransform:
        if self.kind == "extract":
            return GpuTransform(dtype=dtype, mode="short", resize=self.resize, crop=self.crop)
        return GpuTransform(self.size, dtype, "resize")


class HostImageBatch:
    """What the DataLoader yields in place of an f32 [B,3,S,S] tensor;
    ``.to(device)`` = H2D of the uint8 pixels + GPU transform."""

    def __init__(self, pixels, params: torch.Tensor, spec: DeviceTransformSpec):
        self.pixels = pixels      # uint8 [B,H,W,3] tensor, or a list of [H,W,3] if sizes differ
        self.params = params      # int32 [B, PARAM_FIELDS]
        self.spec = spec
        self.dtype = torch.float32

    def __len__(self):
        return self.params.shape[0]

    def pin_memory(self):
        if isinstance(self.pixels, torch.Tensor):
            self.pixels = self.pixels.pin_memory()
        self.params = self.params.pin_memory()
        return self

    def to(self, device, non_blocking: bool = True, dtype: Optional[torch.dtype] = None):
        from .resnet import DeviceImages

        dt = dtype or self.dtype
        tf = _gpu_tf(self.spec, dt)
        dev = torch.device(device)
        if dev.type != "cuda":
            raise RuntimeError("ssip's input pipeline runs on the HIP device; use --device cuda/auto")
        params = self.params.to(dev, non_blocking=non_blocking)
        if isinstance(self.pixels, torch.Tensor):
            return tf(self.pixels.to(dev, non_blocking=non_blocking), params)
        # ragged sources (eval/extraction): one launch per image into one padded batch buffer
        out = None
        for i, p in enumerate(self.pixels):
            if out is None:
                Hr, Wr, Ho, Wo, _, _ = tf.geometry(p.shape[0], p.shape[1])
                out = torch.empty((len(self.pixels), Ho + 2 * tf.pad, Wo + 2 * tf.pad, 4), device=dev, dtype=dt)
            tf(p.unsqueeze(0).to(dev, non_blocking=non_blocking), params[i:i + 1], out=out[i:i + 1])
        return DeviceImages(out, tf.pad)


_TF_CACHE = {}


def _gpu_tf(spec: DeviceTransformSpec, dtype):
    key = (spec.kind, spec.size, spec.resize, spec.crop, dtype)
    tf = _TF_CACHE.get(key)
    if tf is None:
        tf = spec.gpu(dtype)
        _TF_CACHE[key] = tf
    return tf


class Collate:
    """Collate bound to the transform spec of its dataset."""

    def __init__(self, spec: DeviceTransformSpec):
        self.spec = spec

    def __call__(self, batch):
        first = batch[0]
        imgs: List[HostImage] = [b[0] for b in batch]
        params = torch.stack([h.params for h in imgs])
        shapes = {tuple(h.pixels.shape) for h in imgs}
        pixels = torch.stack([h.pixels for h in imgs]) if len(shapes) == 1 else [h.pixels for h in imgs]
        out = [HostImageBatch(pixels, params, self.spec)]
        for k in range(1, len(first)):
            col = [b[k] for b in batch]
            if isinstance(col[0], (int, np.integer)):
                out.append(torch.tensor(col, dtype=torch.int64))
            else:
                out.append(list(col))
        return tuple(out)
