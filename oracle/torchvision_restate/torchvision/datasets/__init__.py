"""ORACLE restatement of torchvision.datasets.ImageFolder
(torchvision/datasets/folder.py: sorted class dirs, sorted os.walk,
IMG_EXTENSIONS filter, PIL loader with convert('RGB'))."""
from __future__ import annotations

import os

from PIL import Image

IMG_EXTENSIONS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")


def pil_loader(path):
    with open(path, "rb") as f:
        img = Image.open(f)
        return img.convert("RGB")


class ImageFolder:
    def __init__(self, root, transform=None, target_transform=None, loader=pil_loader):
        self.root = os.fspath(root)
        classes = sorted(e.name for e in os.scandir(self.root) if e.is_dir())
        if not classes:
            raise FileNotFoundError(f"Couldn't find any class folder in {self.root}.")
        self.classes = classes
        self.class_to_idx = {c: i for i, c in enumerate(classes)}
        samples = []
        for c in sorted(self.class_to_idx):
            d = os.path.join(self.root, c)
            for r, _, fnames in sorted(os.walk(d, followlinks=True)):
                for fn in sorted(fnames):
                    p = os.path.join(r, fn)
                    if p.lower().endswith(IMG_EXTENSIONS):
                        samples.append((p, self.class_to_idx[c]))
        self.samples = samples
        self.imgs = samples
        self.targets = [s[1] for s in samples]
        self.transform = transform
        self.target_transform = target_transform
        self.loader = loader

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, index):
        path, target = self.samples[index]
        sample = self.loader(path)
        if self.transform is not None:
            sample = self.transform(sample)
        if self.target_transform is not None:
            target = self.target_transform(target)
        return sample, target
