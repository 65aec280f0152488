"""A tiny deterministic on-disk dataset in the reference's layout
(<root>/avec_labels/{cancer,normal}/*.png and <root>/sans_label/*.png), used
by make_goldens.py (to run the reference's own pipelines) and by the GPU
pipeline tests (to run ours on the same files).  PNG: lossless, so both sides
decode the same pixels whatever zlib wrote them.  Test data, not reference
code."""
from __future__ import annotations

from pathlib import Path

import numpy as np


def make(root: Path, n_per_class: int = 10, n_unl: int = 12, size: int = 64, seed: int = 0) -> Path:
    from PIL import Image

    rng = np.random.default_rng(seed)
    root = Path(root)
    for cls, bias in (("cancer", 70), ("normal", 170)):
        d = root / "avec_labels" / cls
        d.mkdir(parents=True, exist_ok=True)
        for i in range(n_per_class):
            a = np.clip(rng.normal(bias, 45, (size, size, 3)), 0, 255).astype(np.uint8)
            Image.fromarray(a).save(d / f"{cls}_{i:02d}.png")
    u = root / "sans_label"
    u.mkdir(parents=True, exist_ok=True)
    for i in range(n_unl):
        a = np.clip(rng.normal(rng.choice([70, 170]), 45, (size, size, 3)), 0, 255).astype(np.uint8)
        Image.fromarray(a).save(u / f"u_{i:03d}.png")
    return root


def pretrained_state_dict(seed: int = 1234):
    """The "ImageNet" stand-in both sides load: a torchvision-initialised
    ResNet-18 under `seed` (torchvision init, restated in
    oracle/torchvision_restate and bit-identical in ssip.SSIPResNet)."""
    import torch

    from oracle.torchvision_restate.torchvision import models as tvm

    torch.manual_seed(seed)
    return tvm.resnet18().state_dict()
